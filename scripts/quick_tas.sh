#!/bin/bash
# GPU tests (TAS only) + tas bench + emit ablations + write ceiling
set -u
cd "$(dirname "$0")/.."; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_tas_gpu.py -q --timeout 500 -p no:cacheprovider > gpurun_out/pytest_tas.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_tas.log
if [ $rc -ne 0 ]; then exit $rc; fi
for m in 0 ${ABLATE:-}; do
  PAS_EMIT_ABLATE=$m timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null > gpurun_out/bench_tas_m$m.log || exit $?
  python -c "import json;d=json.load(open('gpurun_out/bench_tas_m$m.log'));print('mode $m', round(d['ms_per_step'],4), round(d['roofline']['frac'],3), 'span', round(d['roofline']['kernel_ms'],4), {k:round(v,4) for k,v in d['config']['kernel_ms_per_step'].items()})"
done
timeout -k 10 120 python scripts/write_ceiling.py 2>/dev/null

#!/bin/bash
# Diagnostic sweep of TAS launch shapes / ablations given as env assignments, e.g.
#   tas_sweep.sh "PAS_EVAL_WAVES=8" "PAS_EVAL_SEGS=2".  Runs the TAS GPU tests first.
# (Ablations are compile-time: scripts/diag/build_variant.sh with -DPAS_EVAL_ABLATE=N.)
set -u
cd "$(dirname "$0")/.."; mkdir -p gpurun_out/sweep
timeout -k 10 300 python -u -m pytest tests/test_tas_gpu.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sweep/pytest.log 2>&1 || exit $?
tail -1 gpurun_out/sweep/pytest.log
run() {
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline \
    > gpurun_out/sweep/b.json 2> gpurun_out/sweep/b.err || exit $?
  python -c "import json,sys;d=json.load(open('gpurun_out/sweep/b.json'));print(sys.argv[1:], round(d['ms_per_step'],4), round(d['roofline']['frac'],3), {k:round(v,4) for k,v in d['config']['kernel_ms_per_step'].items()})" "$@"
}
for spec in "${@:-PAS_EMIT_CHUNK=0}"; do run $spec; done

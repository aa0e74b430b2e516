#!/bin/bash
# Diagnostic: the deschedule line with the fused sweep + plan against the two-call path and
# against the fused path of A/B libraries (lib_ab/*.so), alternating on one box, after the
# label / sweep GPU tests.  usage: c4_ab.sh [lib_ab/x.so ...]
set -u
cd "$(dirname "$0")/../.."
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_labels.py tests/test_tas_gpu.py tests/test_shard.py tests/test_env_knobs.py > gpurun_out/c4_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/c4_tests.log | tail -3
[ $rc -ne 0 ] && { tail -60 gpurun_out/c4_tests.log; exit $rc; }
B="--workload deschedule --steps 50 --warmup 5 --no-cpu-baseline"
show() {
  tail -1 /tmp/c4.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$1', round(d['ms_per_step'],4), round(r['kernel_ms'],4), round(r['frac'],3), d['label_plan_ms'])"
}
for i in 1 2 3 4; do
  timeout -k 10 150 python3 bench.py $B > /tmp/c4.json 2>/tmp/c4.err || { tail /tmp/c4.err; exit 1; }
  show fused
  timeout -k 10 150 python3 bench.py $B --deschedule-separate > /tmp/c4.json 2>/tmp/c4.err || { tail /tmp/c4.err; exit 1; }
  show separate
  for L in "$@"; do
    timeout -k 10 150 bash scripts/diag/with_lib.sh "$L" python3 bench.py $B > /tmp/c4.json 2>/tmp/c4.err || { tail /tmp/c4.err; exit 1; }
    show "$(basename "$L" .so)"
  done
done

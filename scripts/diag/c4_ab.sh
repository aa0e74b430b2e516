#!/bin/bash
# Diagnostic: the deschedule line with the fused sweep + plan against the two-call path,
# alternating on one box (after the label / sweep GPU tests).
set -u
cd "$(dirname "$0")/../.."
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_labels.py tests/test_tas_gpu.py tests/test_shard.py tests/test_env_knobs.py > gpurun_out/c4_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/c4_tests.log | tail -3
[ $rc -ne 0 ] && { tail -60 gpurun_out/c4_tests.log; exit $rc; }
for i in 1 2 3 4; do
  for mode in fused separate; do
    extra=""; [ $mode = separate ] && extra="--deschedule-separate"
    timeout -k 10 150 python3 bench.py --workload deschedule --steps 50 --warmup 5 $extra > /tmp/c4.json 2>/tmp/c4.err || { tail /tmp/c4.err; exit 1; }
    tail -1 /tmp/c4.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$mode', round(d['ms_per_step'],4), round(r['kernel_ms'],4), round(r['frac'],3), d['label_plan_ms'])"
  done
done

#!/bin/bash
# One GPU iteration on the GAS path: the GAS / stream / slot parity tests, then an alternating
# A/B of bench.py --workload gas (in-tree library against lib_ab/*.so), then the in-tree
# library's per-step launch timeline.  usage: iter_gas.sh [lib_ab/x.so ...]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_gas_gpu.py tests/test_gas_wide.py tests/test_gas_many_selections.py \
  tests/test_gas_commit.py tests/test_streams_gpu.py tests/test_configs_full.py \
  tests/test_labels.py tests/test_prioritize_request.py > gpurun_out/iter_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/iter_tests.log | tail -3
[ $rc -ne 0 ] && { tail -40 gpurun_out/iter_tests.log; exit $rc; }
timeout -k 10 500 bash scripts/diag/bench_ab.sh "--workload gas --steps 20 --warmup 3 --no-pipelined" ${AB_ROUNDS:-3} "$@" \
  > gpurun_out/iter_ab.log 2>&1
rc=$?; cat gpurun_out/iter_ab.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 bash scripts/diag/gas_timeline.sh > gpurun_out/iter_timeline.log 2>&1
rc=$?; cat gpurun_out/iter_timeline.log
exit $rc

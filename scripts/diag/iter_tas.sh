#!/bin/bash
# One GPU iteration on the TAS path: the TAS parity tests, then an alternating A/B of
# bench.py --workload tas (in-tree library against lib_ab/*.so).  usage: iter_tas.sh lib...
set -u
cd "$(dirname "$0")/../.."
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_tas_gpu.py tests/test_configs_full.py tests/test_streams_gpu.py tests/test_shard.py \
  > gpurun_out/iter_tas_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/iter_tas_tests.log | tail -3
[ $rc -ne 0 ] && { tail -40 gpurun_out/iter_tas_tests.log; exit $rc; }
timeout -k 10 800 bash scripts/diag/bench_ab.sh "--workload tas --steps 20 --warmup 3 --no-pipelined" ${AB_ROUNDS:-4} "$@"

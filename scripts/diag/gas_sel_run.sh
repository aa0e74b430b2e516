#!/bin/bash
# GPU run of the GAS / shard test files (fit, wide shapes, many selections, commit, shard
# top-k and full lists, extender), then the full-list merge diagnostic at the C2 shape.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gas_many_selections.py tests/test_gas_wide.py \
  tests/test_gas_gpu.py tests/test_gas_commit.py tests/test_shard.py tests/test_extender.py \
  -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gas_sel.log 2>&1
rc=$?; tail -25 gpurun_out/gas_sel.log; [ $rc -eq 0 ] || exit $rc
for s in 2 8; do
  timeout -k 10 300 python -u scripts/diag/full_list_bench.py --shards $s || exit $?
done

#!/bin/bash
# GPU: the full-list merge tests, then the merge diagnostic at the C2 shape (2 and 8 shards).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_shard.py -x -q -m gpu -k "merge or full_list" \
  --timeout 120 --timeout-method thread > gpurun_out/merge.log 2>&1
rc=$?; tail -5 gpurun_out/merge.log; [ $rc -eq 0 ] || exit $rc
for s in 2 8; do
  timeout -k 10 300 python -u scripts/diag/full_list_bench.py --shards $s || exit $?
done

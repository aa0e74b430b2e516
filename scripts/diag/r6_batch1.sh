#!/bin/bash
# Round 6: GPU tests of the round's TAS-side changes, then the TAS store microbenchmark.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
bash scripts/gpu_tests.sh tests/test_submilli_gpu.py tests/test_tas_gpu.py tests/test_labels.py tests/test_extender.py tests/test_shard.py tests/test_snapshot_builders.py tests/test_env_knobs.py || exit $?
timeout -k 10 300 python scripts/diag/tas_store.py 2>&1 | tee gpurun_out/r6_tas_store.log

#!/bin/bash
# Round 6: the GAS GPU tests, then the fork / join diagnostics (stream / buffer variants and
# the bench's pipelined sweep).
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gas_sync.py tests/test_gas_gpu.py tests/test_gas_commit.py tests/test_gas_wide.py tests/test_gas_many_selections.py tests/test_streams_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6_gas_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/r6_gas_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python scripts/diag/gas_pipe_buffers.py 2>&1 | grep streams | tee gpurun_out/r6_gas_buffers.log
bash scripts/diag/gas_pipe.sh 2>&1 | tee gpurun_out/r6_gas_pipe.log

#!/bin/bash
# GPU parity tests (optionally a subset: gpu_tests.sh tests/test_x.py ...) + smoke.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
T=("$@"); [ ${#T[@]} -eq 0 ] && T=(tests)
timeout -k 10 900 python -u -m pytest "${T[@]}" -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider --durations=15 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
exit $rc

#!/bin/bash
# Round-end evidence, part 1: every GPU test, the four bench workloads, smoke.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > gpurun_out/bench_tas.log 2>&1 || exit $?
tail -1 gpurun_out/bench_tas.log
for w in gas deschedule c5; do
  timeout -k 10 400 python bench.py --workload $w --steps 20 --warmup 3 > gpurun_out/bench_$w.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_$w.log
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
echo smoke ok

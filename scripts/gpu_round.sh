#!/bin/bash
# tests + smoke + bench workloads (default: tas) + profile of the first workload
# usage: gpu_round.sh [workload ...]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
WL=("$@"); [ ${#WL[@]} -eq 0 ] && WL=(tas)
for w in "${WL[@]}"; do
  timeout -k 10 400 python bench.py --workload $w --steps 20 --warmup 3 > gpurun_out/bench_$w.log 2>&1
  rc=$?; echo "bench $w rc=$rc"; tail -1 gpurun_out/bench_$w.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
bash scripts/profile.sh "${WL[0]}" "${WL[0]}" || exit $?

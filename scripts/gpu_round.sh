#!/bin/bash
# tests + bench workloads (default: tas) + profile of the first workload
# usage: gpu_round.sh [workload ...]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
WL=("$@"); [ ${#WL[@]} -eq 0 ] && WL=(tas)
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 600 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for w in "${WL[@]}"; do
  timeout -k 10 400 python bench.py --workload $w --steps 20 --warmup 3 > gpurun_out/bench_$w.log 2>&1
  rc=$?; echo "bench $w rc=$rc"; tail -1 gpurun_out/bench_$w.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
bash scripts/profile.sh "${WL[0]}" "${WL[0]}" || exit $?

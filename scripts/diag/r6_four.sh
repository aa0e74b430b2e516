#!/bin/bash
# Round 6: the closed-form four-selection class — GAS GPU tests, C3 bench lines, the fit
# kernels' SQ_INSTS_VALU (prof_kernels.sh gas).
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gas_gpu.py tests/test_gas_wide.py tests/test_gas_many_selections.py tests/test_gas_commit.py tests/test_gas_sync.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6_four_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/r6_four_tests.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload gas --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r6_four_bench$i.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r6_four_bench$i.log').read().strip().splitlines()[-1]); print('gas ms', d['ms_per_step'], 'kernel_ms', d['roofline']['kernel_ms'], 'pipe', d.get('pipelined',{}).get('ms_per_step'))"
done
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_INSTS_SMEM"
timeout -k 10 400 bash scripts/prof_kernels.sh gas "$P1" > gpurun_out/r6_four_pmc.txt 2>&1; rc=$?
cat gpurun_out/r6_four_pmc.txt | grep -E "rfit|rank_prep|gas_prep|avg_us"; exit $rc

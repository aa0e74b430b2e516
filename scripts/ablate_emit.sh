#!/bin/bash
# Diagnostic: emit kernel time with stores / drop loads ablated, plus SQ counters.
set -u
R="$(cd "$(dirname "$0")/.." && pwd)"; cd "$R"; mkdir -p gpurun_out/ablate
for m in 0 1 2; do
  PAS_EMIT_ABLATE=$m timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ablate/mode$m.json 2>gpurun_out/ablate/mode$m.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ablate/mode$m.json'));print($m, d['config']['kernel_ms_per_step'])"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_SMEM -d gpurun_out/ablate/sq -o sq --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ablate/sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -d gpurun_out/ablate/sq2 -o sq --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ablate/sq2.log 2>&1 || exit $?
echo done

#!/bin/bash
# tas bench with each filter ablation (diagnostic; outputs of ablated runs are wrong)
set -u
cd "$(dirname "$0")/.."; mkdir -p gpurun_out
for m in 0 1 2 4 8 0; do
  PAS_FILTER_ABLATE=$m timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null > gpurun_out/bench_filter_a$m.log || exit $?
  python -c "import json;d=json.load(open('gpurun_out/bench_filter_a$m.log'));print('filter ablate $m', {k:round(v,4) for k,v in d['config']['kernel_ms_per_step'].items()})"
done

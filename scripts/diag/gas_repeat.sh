#!/bin/bash
# Diagnostic: the GAS line three times on one box (full bench.py defaults for --workload gas).
set -u
cd "$(dirname "$0")/../.."
TAG="${1:-x}"
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --workload gas --steps 20 --warmup 3 > gpurun_out/gas_rep_${TAG}_$i.log 2>&1 || exit 1
  tail -1 gpurun_out/gas_rep_${TAG}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$TAG', $i, round(d['ms_per_step'],4), round(d['roofline']['frac'],3), round(d['pipelined']['ms_per_step'],4))"
done

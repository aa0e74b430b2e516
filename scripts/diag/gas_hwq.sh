#!/bin/bash
# Diagnostic: the GAS line (D = 1, 2) by hardware-queue count.
set -u
cd "$(dirname "$0")/../.."
for Q in 4 6 8; do
  for D in 1 2; do
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 150 python3 bench.py --workload gas --steps 20 --warmup 3 --no-cpu-baseline --no-request-latency --no-pipelined --pipeline $D > /tmp/gp.json 2>/tmp/gp.err || { tail /tmp/gp.err; exit 1; }
    tail -1 /tmp/gp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('Q=$Q D=$D', round(d['ms_per_step'],4))"
  done
done

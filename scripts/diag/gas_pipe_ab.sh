#!/bin/bash
# Diagnostic: bench.py's GAS line at 1..4 pipelined streams, fits ordered after other streams'
# fits (default) and not (PAS_GAS_NO_ORDER=1), alternating.
set -u
cd "$(dirname "$0")/../.."
for i in 1 2; do
  for O in order no_order; do
    if [ $O = no_order ]; then export PAS_GAS_NO_ORDER=1; else unset PAS_GAS_NO_ORDER; fi
    for D in 1 2 3 4; do
      timeout -k 10 150 python3 bench.py --workload gas --steps 20 --warmup 3 --no-cpu-baseline --no-request-latency --no-pipelined --pipeline $D > /tmp/gp.json 2>/tmp/gp.err || { tail /tmp/gp.err; exit 1; }
      tail -1 /tmp/gp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$O D=$D', round(d['ms_per_step'],4), round(d['roofline']['frac'],3))"
    done
  done
done

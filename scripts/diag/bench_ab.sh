#!/bin/bash
# Diagnostic: bench.py lines with the in-tree libpas.so and with A/B builds, alternating,
# on one box.  usage: bench_ab.sh "<bench args>" ROUNDS lib...   (prints ms/step and kernel ms)
set -u
R="$(cd "$(dirname "$0")/../.." && pwd)"; A="$1"; N="$2"; shift 2
trees=("$R")
for L in "$@"; do
  T="/tmp/ab_$(basename "$L" .so)"; rm -rf "$T"; mkdir -p "$T"
  cp -r "$R/bench.py" "$R/platform-aware-scheduling_amd" "$R/oracle" "$T/"
  cp "$R/$L" "$T/platform-aware-scheduling_amd/lib/libpas.so"; trees+=("$T")
done
for i in $(seq "$N"); do
  for T in "${trees[@]}"; do
    timeout -k 10 150 python3 "$T/bench.py" $A --no-cpu-baseline --no-request-latency > /tmp/ab_out.json 2>/tmp/ab_err.log || { cat /tmp/ab_err.log; exit 1; }
    tail -1 /tmp/ab_out.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; print('$(basename $T)', round(d['ms_per_step'],4), round(r.get('kernel_ms',0),4), round(r.get('frac',0),4), {k: round(v,3) for k,v in (d['config'].get('kernel_ms_per_step') or {}).items()})"
  done
done

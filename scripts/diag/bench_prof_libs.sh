#!/bin/bash
# Diagnostic: rocprofv3 kernel stats of the bench's D = 1 GAS line per library (in-tree first).
# usage: bench_prof_libs.sh "<bench args>" lib...
set -u
R="$(cd "$(dirname "$0")/../.." && pwd)"; A="$1"; shift
OUT="$R/gpurun_out/bench_prof_libs"; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
i=0
for L in tree "$@"; do
  i=$((i+1)); T="$R"
  if [ "$L" != tree ]; then
    T="/tmp/bpl_$i"; rm -rf "$T"; mkdir -p "$T"
    cp -r "$R/bench.py" "$R/platform-aware-scheduling_amd" "$R/oracle" "$T/"
    cp "$R/$L" "$T/platform-aware-scheduling_amd/lib/libpas.so"
  fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/$i" -o kt --output-format csv -- python3 "$T/bench.py" $A --no-cpu-baseline --no-request-latency --no-pipelined > "$OUT/$i.log" 2>&1 || { echo "lib $L failed"; tail "$OUT/$i.log"; exit 1; }
  tail -1 "$OUT/$i.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L', 'ms_per_step', round(d['ms_per_step'],4))"
  python3 - "$OUT/$i" "$L" <<'PY'
import csv, glob, sys, re
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(gas_\w+|tas_\w+)", r["Name"])
        if m:
            print(f'  {sys.argv[2]:20s} {m.group(1):32s} avg_us={float(r["AverageNs"])/1e3:8.1f} min_us={float(r["MinNs"])/1e3:8.1f} calls={r["Calls"]}')
PY
done

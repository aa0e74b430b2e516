#!/bin/bash
# Diagnostic: rocprofv3 kernel stats of scripts/diag/gas_mix.py for one case, per library.
# usage: prof_libs.sh CASE P lib...   (in-tree lib first)
set -u
R="$(cd "$(dirname "$0")/../.." && pwd)"; CASE="$1"; P="$2"; shift 2
OUT="$R/gpurun_out/prof_libs"; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
i=0
for L in tree "$@"; do
  i=$((i+1)); PKG="$R/platform-aware-scheduling_amd"
  if [ "$L" != tree ]; then
    PKG="/tmp/pl_$i"; rm -rf "$PKG"; mkdir -p "$PKG/lib"; cp -r "$R/platform-aware-scheduling_amd/pas_amd" "$PKG/"; cp "$R/$L" "$PKG/lib/libpas.so"
  fi
  PAS_DIAG_PKG="$PKG" PAS_DIAG_ONLY="$CASE" timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/$i" -o kt --output-format csv -- python3 "$R/scripts/diag/gas_mix.py" "$P" > "$OUT/$i.log" 2>&1 || { echo "lib $L failed"; tail "$OUT/$i.log"; exit 1; }
  python3 - "$OUT/$i" "$L" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "pas::" in r["Name"] and "gas_" in r["Name"]:
            n = r["Name"].split("(anonymous namespace)::")[-1].split("(")[0]
            print(f'{sys.argv[2]:24s} {n:40s} avg_us={float(r["AverageNs"])/1e3:9.1f} calls={r["Calls"]}')
PY
done

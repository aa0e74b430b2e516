#!/bin/bash
# Diagnostic: SQ counters of the GAS fit kernels for one gas_mix.py case (PAS_DIAG_ONLY),
# with the in-tree libpas.so and an A/B build.  usage: gas_pmc.sh CASE P [lib]
# Output: gpurun_out/gas_pmc/summary.txt
set -u
R="$(cd "$(dirname "$0")/../.." && pwd)"; CASE="$1"; P="$2"; ALT="${3:-}"
OUT="$R/gpurun_out/gas_pmc"; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
PASSES=("SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_INSTS_SMEM"
        "SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_INSTS_VMEM")
run() {  # tag pkgdir
  local i=0
  for C in "${PASSES[@]}"; do
    i=$((i+1))
    PAS_DIAG_PKG="$2" PAS_DIAG_ONLY="$CASE" timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/$1_p$i" -o p --output-format csv -- python3 "$R/scripts/diag/gas_mix.py" "$P" > "$OUT/$1_p$i.log" 2>&1 || { echo "pass $1 $i failed rc=$?"; return 1; }
  done
}
run tree "$R/platform-aware-scheduling_amd" || exit 1
if [ -n "$ALT" ]; then
  T="/tmp/ab_pmc"; rm -rf "$T"; mkdir -p "$T/lib"; cp -r "$R/platform-aware-scheduling_amd/pas_amd" "$T/"; cp "$R/$ALT" "$T/lib/libpas.so"
  run alt "$T" || exit 1
fi
python3 - "$OUT" > "$OUT/summary.txt" <<'PY'
import csv, glob, sys, collections, os
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/*_p*/**/*counter_collection.csv", recursive=True):
    tag = os.path.relpath(f, out).split("_p")[0]
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "pas::" not in n or "gas_" not in n: continue
        k = n.split("(anonymous namespace)::")[1].split("(")[0]
        agg[(tag, k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (t, k, c), v in sorted(agg.items()):
    print(f"{t:5s} {k:36s} {c:24s} {sum(v)/len(v):16.0f}")
PY
cat "$OUT/summary.txt"

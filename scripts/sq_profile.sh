#!/bin/bash
# SQ counter passes for the tas bench (separate passes; no trace domains with --pmc)
set -u
R="$(cd "$(dirname "$0")/.." && pwd)"; OUT="$R/gpurun_out/sq"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
B=(python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1)
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C -d "$OUT/p$i" -o p --output-format csv -- "${B[@]}" > "$OUT/p$i.log" 2>&1 || exit $?
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "pas::" not in n: continue
        k = n.split("(anonymous namespace)::")[1].split("(")[0].split("<")[0]
        agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:24s} {c:22s} {sum(v)/len(v):16.0f}")
PY

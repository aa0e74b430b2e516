#!/bin/bash
# Counter passes for the tas bench (each pass its own rocprofv3 run; no trace domains with
# --pmc).  Usage: sq_profile.sh "<pass1 counters>" "<pass2 counters>" ...   Output:
# gpurun_out/sq/summary.txt (per kernel averages), gpurun_out/sq/avail.txt (counter list).
set -u
R="$(cd "$(dirname "$0")/.." && pwd)"; OUT="$R/gpurun_out/sq"; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
[ -f "$R/profiles/avail_counters.txt" ] || timeout -k 10 120 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
B=(python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1)
i=0
for C in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C -d "$OUT/p$i" -o p --output-format csv -- "${B[@]}" > "$OUT/p$i.log" 2>&1 || echo "pass $i ($C) failed rc=$?"
done
python3 - "$OUT" > "$OUT/summary.txt" <<'PY'
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
    print(f"{k:24s} {c:28s} {sum(v)/len(v):16.0f}")
PY
cat "$OUT/summary.txt"

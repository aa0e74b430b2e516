#!/bin/bash
# Diagnostic: rocprofv3 kernel stats + SQ counters for one bench workload.
# usage: prof_kernels.sh <workload> ["<pmc pass>" ...]   Output: gpurun_out/pk_<workload>/
set -u
R="$(cd "$(dirname "$0")/.." && pwd)"; W="${1:-tas}"; shift || true
OUT="$R/gpurun_out/pk_$W"; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
B=(python3 "$R/bench.py" --workload "$W" --no-cpu-baseline --no-request-latency --no-pipelined --settle 0 --steps 5 --warmup 1)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- "${B[@]}" > "$OUT/kt.log" 2>&1 || exit $?
python3 - "$OUT/kt" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "pas::" in r["Name"]:
            print(f'{r["Name"].split("(")[0][-60:]:60s} calls={r["Calls"]:>4s} avg_us={float(r["AverageNs"])/1e3:10.1f}')
PY
i=0
for C in "$@"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $C -d "$OUT/p$i" -o p --output-format csv -- "${B[@]}" > "$OUT/p$i.log" 2>&1 || exit $?
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "pas::" not in n: continue
        k = n.split("(anonymous namespace)::")[1].split("(")[0][:40]
        agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:40s} {c:24s} {sum(v)/len(v):16.0f}")
PY

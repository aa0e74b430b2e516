#!/bin/bash
set -u
R=/root/repo
OUT=$R/gpurun_out/sqc; rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp; cd /tmp
export PAS_DIAG_ONLY=real:None
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_REQ SQ_WAVE_CYCLES SQ_WAVES -d $OUT/p1 -o p --output-format csv -- python3 $R/scripts/diag/gas_mix.py 10000 > $OUT/p1.log 2>&1 || exit $?
python3 - $OUT <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p1/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "pas::" not in n: continue
        k = n.split("(anonymous namespace)::")[1].split("(")[0][:32]
        agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:34s} {c:22s} {sum(v)/len(v):14.0f}")
PY

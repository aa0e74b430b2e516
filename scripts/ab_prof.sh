#!/bin/bash
# Diagnostic: kernel stats of bench.py with lib/libpas.so and with an A/B build, same box.
# usage: ab_prof.sh <workload> <alt lib>   Output: gpurun_out/ab_<workload>/
set -u
R="$(cd "$(dirname "$0")/.." && pwd)"; W="$1"; ALT="$(cd "$(dirname "$2")" && pwd)/$(basename "$2")"
OUT="$R/gpurun_out/ab_$W"; rm -rf "$OUT"; mkdir -p "$OUT"
# the alternative tree: bench.py + the package with libpas.so replaced by the A/B build
T=/tmp/ab_tree; rm -rf "$T"; mkdir -p "$T"
cp -r "$R/bench.py" "$R/platform-aware-scheduling_amd" "$R/oracle" "$T/"
cp "$ALT" "$T/platform-aware-scheduling_amd/lib/libpas.so"
export TMPDIR=/tmp; cd /tmp
A=(--workload "$W" --no-cpu-baseline --steps 10 --warmup 2)
for round in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/new$round" -o kt --output-format csv -- python3 "$R/bench.py" "${A[@]}" > "$OUT/new$round.log" 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/alt$round" -o kt --output-format csv -- python3 "$T/bench.py" "${A[@]}" > "$OUT/alt$round.log" 2>&1 || exit $?
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, os
for d in sorted(glob.glob(sys.argv[1] + "/*/")):
    for f in glob.glob(d + "**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "pas::" in r["Name"]:
                n = r["Name"].split("(anonymous namespace)::")[-1].split("(")[0]
                print(f'{os.path.basename(d[:-1]):6s} {n:40s} avg_us={float(r["AverageNs"])/1e3:10.1f}')
PY

#!/bin/bash
# Diagnostic: per-step launch timeline of the GAS fit (rocprofv3 kernel trace of bench.py's
# one-stream line) per library (in-tree first).  usage: gas_timeline.sh lib...
set -u
R="$(cd "$(dirname "$0")/../.." && pwd)"
OUT="$R/gpurun_out/gas_timeline"; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
i=0
for L in tree "$@"; do
  i=$((i+1)); T="$R"
  if [ "$L" != tree ]; then
    T="/tmp/gtl_$i"; rm -rf "$T"; mkdir -p "$T"
    cp -r "$R/bench.py" "$R/platform-aware-scheduling_amd" "$R/oracle" "$T/"
    cp "$R/$L" "$T/platform-aware-scheduling_amd/lib/libpas.so"
  fi
  timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/$i" -o kt --output-format csv -- python3 "$T/bench.py" --workload gas --steps 10 --warmup 2 --no-cpu-baseline --no-pipelined > "$OUT/$i.log" 2>&1 || { echo "lib $L failed"; tail "$OUT/$i.log"; exit 1; }
  echo "== $L"
  python3 - "$OUT/$i" <<'PY'
import csv, glob, re, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(gas_\w+)", r["Kernel_Name"])
        if m:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1), r["Queue_Id"]))
rows.sort()
starts = [i for i, r in enumerate(rows) if r[2] in ("gas_prep_kernel", "gas_prep_fused_kernel")]
for si, ei in list(zip(starts, starts[1:]))[-3:-1]:
    t0 = rows[si][0]
    print("  step", (rows[ei][0] - t0) / 1e3, "us")
    for r in rows[si:ei]:
        print(f"    {r[2]:26s} {(r[0]-t0)/1e3:7.1f} .. {(r[1]-t0)/1e3:7.1f}  q{r[3]}")
PY
done

#!/bin/bash
# Diagnostic: kernel-trace timelines of C3 fits on 1 and 2 streams (gas_pipe_buffers.py).
set -u
R="$(cd "$(dirname "$0")/../.." && pwd)"
OUT="$R/gpurun_out/gas_pipe_tl"; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
for NS in 1 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/$NS" -o kt --output-format csv -- python3 "$R/scripts/diag/gas_pipe_buffers.py" $NS > "$OUT/$NS.log" 2>&1 || { tail "$OUT/$NS.log"; exit 1; }
  echo "== streams $NS: $(grep streams "$OUT/$NS.log")"
  python3 - "$OUT/$NS" <<'PY'
import csv, glob, re, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(gas_\w+)", r["Kernel_Name"])
        if m:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1), r["Queue_Id"]))
rows.sort()
starts = [i for i, r in enumerate(rows) if r[2] == "gas_prep_kernel"]
for si, ei in list(zip(starts, starts[1:]))[-4:-1]:
    t0 = rows[si][0]
    print("  step", (rows[ei][0] - t0) / 1e3, "us")
    for r in rows[si:ei]:
        print(f"    {r[2]:26s} {(r[0]-t0)/1e3:7.1f} .. {(r[1]-t0)/1e3:7.1f}  q{r[3]}")
PY
done

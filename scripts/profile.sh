#!/bin/bash
# rocprofv3 passes for one bench workload: kernel trace + stats, then separate PMC passes
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).  Output: gpurun_out/prof_<tag>/
set -u
R="$(cd "$(dirname "$0")/.." && pwd)"
W="${1:-tas}"; TAG="${2:-$W}"; shift 2 || true
OUT="$R/gpurun_out/prof_$TAG"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
B=(python3 "$R/bench.py" --workload "$W" --no-cpu-baseline --no-request-latency --no-pipelined "$@")
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- "${B[@]}" --steps 10 --warmup 2 > "$OUT/kt.log" 2>&1 || exit $?
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS"; do
  N="$(echo $C | tr ' ' '_')"
  timeout -k 10 300 rocprofv3 --pmc $C -d "$OUT/pmc_$N" -o pmc --output-format csv -- "${B[@]}" --steps 3 --warmup 1 > "$OUT/pmc_$N.log" 2>&1 || exit $?
done
echo "profile $TAG done"

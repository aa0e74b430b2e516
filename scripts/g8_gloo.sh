#!/bin/bash
# One-GPU rehearsal of the driver's 8-rank bench.py run: eight ranks
# share the box's GPU over gloo at the default (full) sizes; the timings are meaningless,
# the point is the orchestration's wall time and host memory.
mkdir -p gpurun_out
( while sleep 45; do date +%T >> gpurun_out/g8_heartbeat.txt; done ) &
HB=$!
T0=$(date +%s); timeout -k 10 1080 python -u bench.py --gpus 8 --backend gloo \
    > gpurun_out/g8_gloo.json 2> gpurun_out/g8_gloo.err
rc=$?; echo "wall_s=$(( $(date +%s) - T0 ))"
kill $HB
echo "rc=$rc"
tail -c 3000 gpurun_out/g8_gloo.err
exit $rc

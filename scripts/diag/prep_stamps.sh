#!/bin/bash
# Diagnostic: phase times of the TAS prep launch (lib_ab/prep_stamps.so, -DPAS_PREP_STAMPS=1:
# 100 MHz ticks printed by the kernel) over a short C2 bench run.
set -u
cd "$(dirname "$0")/../.."
timeout -k 10 200 bash scripts/diag/with_lib.sh lib_ab/prep_stamps.so python3 bench.py --steps 3 --warmup 1 --settle 0 --no-pipelined --no-request-latency --no-cpu-baseline > /tmp/ps.log 2>&1 || { tail /tmp/ps.log; exit 1; }
grep "STAMP group" /tmp/ps.log | tail -8
grep "STAMP" /tmp/ps.log | grep -v group | tail -12

#!/bin/bash
# Diagnostic: phase times of the threaded request decode (lib_ab/decode_trace.so, a build with
# -DPAS_DECODE_TRACE) at 1, 8 and 16 threads on the bench's 100k-node body.
set -u
R="$(cd "$(dirname "$0")/../.." && pwd)"
T=/tmp/ab_decode_trace; rm -rf "$T"; mkdir -p "$T"
cp -r "$R/bench.py" "$R/platform-aware-scheduling_amd" "$R/scripts" "$T/"
cp "$R/lib_ab/${LIB:-decode_trace}.so" "$T/platform-aware-scheduling_amd/lib/libpas.so"
timeout -k 10 120 python3 "$T/scripts/diag/decode_threads.py" 1 8 16 2>&1 | grep -v amdgpu.ids | awk '{print}' | tail -60

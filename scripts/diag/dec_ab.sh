#!/bin/bash
# Diagnostic: the threaded request decode and filter-result encode, in-tree library against
# lib_ab/dec_base.so (alternating, 16 and 8 threads), then phase times of the two decode trace
# builds (lib_ab/dec_trace_new.so, lib_ab/dec_trace_base.so: -DPAS_DECODE_TRACE).
set -u
cd "$(dirname "$0")/../.."
for i in 1 2 3 4; do
  echo "== tree"; timeout -k 10 120 python3 scripts/diag/decode_threads.py 16 8 || exit 1
  timeout -k 10 120 python3 scripts/diag/encode_threads.py 16 || exit 1
  echo "== base"; timeout -k 10 120 bash scripts/diag/with_lib.sh lib_ab/dec_base.so python3 scripts/diag/decode_threads.py 16 8 || exit 1
  timeout -k 10 120 bash scripts/diag/with_lib.sh lib_ab/dec_base.so python3 scripts/diag/encode_threads.py 16 || exit 1
done
for i in 1 2; do
  for L in dec_trace_new dec_trace_base; do
    echo "== $L"; LIB=$L timeout -k 10 150 bash scripts/diag/decode_phases.sh || exit 1
  done
done

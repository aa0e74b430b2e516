#!/bin/bash
# Diagnostic: C3 fits on 1 / 2 streams by hardware-queue count and cross-stream ordering.
set -u
cd "$(dirname "$0")/../.."
for Q in 4 8 16; do
  for O in order no_order; do
    if [ $O = no_order ]; then export PAS_GAS_NO_ORDER=1; else unset PAS_GAS_NO_ORDER; fi
    echo "== GPU_MAX_HW_QUEUES=$Q $O"
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 120 python scripts/diag/gas_pipe_buffers.py 2>&1 | grep "buffers=2"
  done
done

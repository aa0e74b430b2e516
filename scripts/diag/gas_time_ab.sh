#!/bin/bash
# Diagnostic: gas_time.py with the in-tree libpas.so and with A/B builds, alternating on one box.
# usage: gas_time_ab.sh ROUNDS lib...
set -u
R="$(cd "$(dirname "$0")/../.." && pwd)"; N="$1"; shift
trees=("$R")
for L in "$@"; do
  T="/tmp/gt_$(basename "$L" .so)"; rm -rf "$T"; mkdir -p "$T/scripts/diag"
  cp -r "$R/platform-aware-scheduling_amd" "$T/"; cp "$R/scripts/diag/gas_time.py" "$T/scripts/diag/"
  cp "$R/$L" "$T/platform-aware-scheduling_amd/lib/libpas.so"; trees+=("$T")
done
for i in $(seq "$N"); do
  for T in "${trees[@]}"; do
    timeout -k 10 150 python3 "$T/scripts/diag/gas_time.py" 50 || exit $?
  done
done

#!/bin/bash
# Diagnostic: scripts/diag/gas_mix.py with the in-tree libpas.so and with each A/B build given.
# usage: gas_ab.sh P lib...   (prints per-S fit spans per library)
set -u
R="$(cd "$(dirname "$0")/../.." && pwd)"; P="$1"; shift
echo "== in-tree"; timeout -k 10 150 python3 -u "$R/scripts/diag/gas_mix.py" "$P" || exit $?
for L in "$@"; do
  T="/tmp/ab_$(basename "$L" .so)"; rm -rf "$T"; mkdir -p "$T"
  cp -r "$R/platform-aware-scheduling_amd/pas_amd" "$T/"; mkdir -p "$T/lib"; cp "$R/$L" "$T/lib/libpas.so"
  echo "== $L"; PAS_DIAG_PKG="$T" timeout -k 10 150 python3 -u "$R/scripts/diag/gas_mix.py" "$P" || exit $?
done

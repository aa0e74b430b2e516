#!/bin/bash
# Diagnostic: run a command in a copy of the tree whose libpas.so is lib_ab/NAME.so.
# usage: with_lib.sh lib_ab/NAME.so command...
set -u
R="$(cd "$(dirname "$0")/../.." && pwd)"; L="$1"; shift
T="/tmp/wl_$(basename "$L" .so)"; rm -rf "$T"; mkdir -p "$T"
cp -r "$R/tests" "$R/oracle" "$R/platform-aware-scheduling_amd" "$R/scripts" "$R/bench.py" \
  "$R/__graft_entry__.py" "$R/pytest.ini" "$T/"
cp "$R/$L" "$T/platform-aware-scheduling_amd/lib/libpas.so"
cd "$T" && "$@"

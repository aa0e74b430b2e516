#!/bin/bash
# Diagnostic: run GPU tests against an A/B library: a copy of the tree with lib_ab/NAME.so as
# libpas.so.  usage: lib_tests.sh lib_ab/NAME.so "pytest args"
set -u
R="$(cd "$(dirname "$0")/../.." && pwd)"; L="$1"; shift
T="/tmp/lt_$(basename "$L" .so)"; rm -rf "$T"; mkdir -p "$T"
cp -r "$R/tests" "$R/oracle" "$R/platform-aware-scheduling_amd" "$R/bench.py" "$R/__graft_entry__.py" "$T/"
[ -f "$R/pytest.ini" ] && cp "$R/pytest.ini" "$T/"
[ -f "$R/conftest.py" ] && cp "$R/conftest.py" "$T/"
cp "$R/$L" "$T/platform-aware-scheduling_amd/lib/libpas.so"
cd "$T" && timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 120 --timeout-method thread $@

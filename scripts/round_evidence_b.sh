#!/bin/bash
# Round-end evidence, part 2: rocprofv3 kernel-trace/stats + PMC passes per bench workload.
set -u
cd "$(dirname "$0")/.."
for w in "$@"; do
  bash scripts/profile.sh $w $w || exit $?
done

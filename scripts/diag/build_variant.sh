#!/bin/bash
# Diagnostic: an A/B build of libpas.so with extra -D flags for one source file.
# usage: build_variant.sh NAME SRC "-DFOO=1 -DBAR=2"   -> lib_ab/NAME.so
# (SRCFILE=path compiles that file in place of csrc/SRC.hip, e.g. a git show of HEAD)
set -eu
R="$(cd "$(dirname "$0")/../.." && pwd)"; NAME="$1"; SRC="$2"; DEFS="$3"
P="$R/platform-aware-scheduling_amd"
make -s -C "$P"
mkdir -p "$R/lib_ab" "/tmp/ab_build_$NAME"
objs=()
for o in "$P"/build/*.o; do
  case "$o" in *_fault.o) continue ;; esac  # (lib/libpas_fault.so's objects)
  if [ "$(basename "$o" .o)" = "$SRC" ]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result \
      -I"$R/include" -I"$P/csrc" $DEFS -c "${SRCFILE:-$P/csrc/$SRC.hip}" -o "/tmp/ab_build_$NAME/$SRC.o"
    objs+=("/tmp/ab_build_$NAME/$SRC.o")
  else
    objs+=("$o")
  fi
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$R/lib_ab/$NAME.so" "${objs[@]}"
echo "lib_ab/$NAME.so"

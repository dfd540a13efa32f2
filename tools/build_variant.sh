#!/bin/bash
# Build an A/B variant of libnfk.so under build_ab/NAME/ (in-tree, so it
# travels to the GPU box; select it with NFK_LIBRARY=build_ab/NAME/libnfk.so).
# usage: bash tools/build_variant.sh NAME [REV|-] [EXTRA compiler flags...]
#   REV: git revision whose csrc/ and include/ to build ('-' = working tree)
set -eu
NAME=$1; REV=${2:--}; shift; [ $# -gt 0 ] && shift
EXTRA="$*"
ROOT=$(cd "$(dirname "$0")/.." && pwd)
V=$ROOT/build_ab/$NAME
rm -rf "$V/src"; mkdir -p "$V/src/normalizingflow_amd/csrc" "$V/src/include" "$V/obj"
if [ "$REV" = "-" ]; then
  cp -p "$ROOT"/normalizingflow_amd/csrc/* "$V/src/normalizingflow_amd/csrc/"
  cp -p "$ROOT"/include/* "$V/src/include/"
else
  git -C "$ROOT" archive "$REV" normalizingflow_amd/csrc include | tar -x -C "$V/src"
fi
# reuse the main build's objects for sources identical to the working tree's
for o in "$ROOT"/build/*.o; do
  b=$(basename "$o" .o)
  if [ -z "$EXTRA" ] && cmp -s "$V/src/normalizingflow_amd/csrc/$b.hip" "$ROOT/normalizingflow_amd/csrc/$b.hip" \
     && [ "$REV" = "-" ] && [ ! "$V/obj/$b.o" -nt "$o" ]; then cp -p "$o" "$V/obj/"; fi
done
make -C "$V/src/normalizingflow_amd/csrc" -j8 OUT="$V/libnfk.so" BUILD="$V/obj" EXTRA="$EXTRA" >"$V/build.log" 2>&1 \
  || { tail -20 "$V/build.log"; exit 1; }
echo "built $V/libnfk.so"

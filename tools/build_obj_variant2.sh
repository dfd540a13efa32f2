#!/bin/bash
# One translation unit rebuilt with extra flags, linked with the main build's
# other objects into build_ab/NAME/libnfk.so (select with NFK_LIBRARY=...).
# usage: bash tools/build_obj_variant2.sh NAME UNIT EXTRA-FLAGS...
set -eu
NAME=$1; UNIT=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
V=$ROOT/build_ab/$NAME; mkdir -p "$V/obj"
NOPK="-Xclang -target-feature -Xclang -packed-fp32-ops"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off -Wall -Wno-unused-function \
    -Wno-unused-result $NOPK "$@" -c "$ROOT/normalizingflow_amd/csrc/$UNIT.hip" -o "$V/obj/$UNIT.o" \
    -Rpass-analysis=kernel-resource-usage 2> "$V/build.log" || { tail -20 "$V/build.log"; exit 1; }
objs=""
for o in "$ROOT"/build/*.o; do b=$(basename "$o"); [ "$b" = "$UNIT.o" ] && objs="$objs $V/obj/$UNIT.o" || objs="$objs $o"; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o "$V/libnfk.so" $objs
grep -A8 "k_nsf_chain2ILi3ELb1ELi8ELb0" "$V/build.log" | grep -E "VGPRs:|Spill|Scratch" | head -4
echo "built $V/libnfk.so"

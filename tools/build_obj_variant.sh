#!/bin/bash
# Diagnostic variant of libnfk.so that differs from the main build only in one
# source file's compile flags: build_ab/NAME/libnfk.so (travels to the GPU box;
# select it with NFK_LIBRARY).  usage: tools/build_obj_variant.sh NAME SRC [flags...]
#   SRC: a file under normalizingflow_amd/csrc, e.g. nfk_fused_ar.hip
set -eu
NAME=$1; SRC=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
V=$ROOT/build_ab/$NAME
mkdir -p "$V"
C=$ROOT/normalizingflow_amd/csrc
B=$(basename "$SRC" .hip)
/opt/rocm/bin/hipcc "$@" -O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off -Wall -Wno-unused-function \
    -Wno-unused-result -c "$C/$SRC" -o "$V/$B.o"
objs=$(ls "$ROOT"/build/*.o | grep -v "/$B.o")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o "$V/libnfk.so" $objs "$V/$B.o"
echo "built $V/libnfk.so"

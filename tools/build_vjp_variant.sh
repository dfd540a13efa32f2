#!/bin/bash
# Diagnostic variant of libnfk.so that differs from the main build only in
# nfk_fused_vjp.hip's compile flags: build_ab/NAME/libnfk.so (travels to the
# GPU box; select it with NFK_LIBRARY).  usage: tools/build_vjp_variant.sh NAME [flags...]
set -eu
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
V=$ROOT/build_ab/$NAME
mkdir -p "$V"
C=$ROOT/normalizingflow_amd/csrc
/opt/rocm/bin/hipcc "$@" -O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off -Wall -Wno-unused-function \
    -Wno-unused-result -c "$C/nfk_fused_vjp.hip" -o "$V/nfk_fused_vjp.o"
objs=$(ls "$ROOT"/build/*.o | grep -v nfk_fused_vjp.o)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o "$V/libnfk.so" $objs "$V/nfk_fused_vjp.o"
echo "built $V/libnfk.so"

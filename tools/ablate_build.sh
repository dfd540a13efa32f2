#!/bin/bash
# Build diagnostic variants of libnfk.so (ablation hooks in nfk_fused_impl.h).
# usage: bash tools/ablate_build.sh   -> normalizingflow_amd/libnfk_abl_*.so
set -e
cd "$(dirname "$0")/../normalizingflow_amd/csrc"
build() {  # name, defines
  make -s -j8 EXTRA="$2" OUT=../libnfk_abl_$1.so BUILD=../../build/abl_$1 >/dev/null
  echo "built libnfk_abl_$1.so ($2)"
}
build nostage "-DNFK_ABL_NOSTAGE"
build noepi "-DNFK_ABL_NOEPI"
build nostage_noepi "-DNFK_ABL_NOEPI -DNFK_ABL_NOSTAGE"

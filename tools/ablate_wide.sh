#!/bin/bash
# Diagnostic variants of libnfk.so for the wide fused kernel (hooks in nfk_fused_wide.h).
# usage: bash tools/ablate_wide.sh   -> normalizingflow_amd/libnfk_wabl_*.so
set -e
cd "$(dirname "$0")/../normalizingflow_amd/csrc"
build() {  # name, defines
  make -s -j8 EXTRA="$2" OUT=../libnfk_wabl_$1.so BUILD=../../build/wabl_$1 >/dev/null
  echo "built libnfk_wabl_$1.so ($2)"
}
build l2hot "-DNFK_WABL_L2HOT"
build noepi "-DNFK_WABL_NOEPI"
build l2hot_noepi "-DNFK_WABL_L2HOT -DNFK_WABL_NOEPI"
build nostage_noepi "-DNFK_WABL_NOSTAGE -DNFK_WABL_NOEPI"

#!/bin/bash
# Round 4: wide fused NSF_AR at KBH 6/9/10 -- waits between a tile pair's MFMAs / after the bias init
set -u
O=gpurun_out/r4l; mkdir -p $O
for v in armn arbn; do
  NFK_LIBRARY=$PWD/build_ab/$v/libnfk.so DBG_HS=192,288,320 DBG_DIMS=2,8 timeout -k 10 300 python -u tools/dbg_ar_wide.py > $O/$v.log 2>&1
  rc=$?; echo "== $v"; grep -h "^H " $O/$v.log; [ $rc -ne 0 ] && { tail -5 $O/$v.log; exit $rc; }
done
exit 0

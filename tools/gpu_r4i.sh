#!/bin/bash
# Round 4: wide fused NSF_AR -- KBH 6/7/9/10 and the copy-serialised build
set -u
O=gpurun_out/r4i; mkdir -p $O
for v in arkbh2 arsync; do
  export NFK_LIBRARY=$PWD/build_ab/$v/libnfk.so
  DBG_HS=192,224,288,320,354 DBG_DIMS=2,8 timeout -k 10 200 python -u tools/dbg_ar_wide.py > $O/$v.log 2>&1
  rc=$?; echo "== $v"; grep -h "^H " $O/$v.log; [ $rc -ne 0 ] && { tail -5 $O/$v.log; exit $rc; }
done
exit 0

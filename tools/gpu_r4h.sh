#!/bin/bash
# Round 4: wide fused NSF_AR -- hidden widths with (352, 354) and without (160, 192, 256) scratch spills
set -u
O=gpurun_out/r4h; mkdir -p $O
export NFK_LIBRARY=$PWD/build_ab/arkbh/libnfk.so
DBG_HS=160,192,256,354 DBG_DIMS=2,8 timeout -k 10 200 python -u tools/dbg_ar_wide.py > $O/arkbh.log 2>&1
rc=$?; grep -h "^H " $O/arkbh.log; [ $rc -ne 0 ] && tail -5 $O/arkbh.log; exit $rc

#!/bin/bash
# Round 4: wide fused NSF_AR with a long wait after every GEMM's last MFMA
set -u
O=gpurun_out/r4j; mkdir -p $O
NFK_LIBRARY=$PWD/build_ab/arpn/libnfk.so DBG_HS=192,224,288,320,352,354 DBG_DIMS=2,8 timeout -k 10 200 python -u tools/dbg_ar_wide.py > $O/arpn.log 2>&1
rc=$?; grep -h "^H " $O/arpn.log; [ $rc -ne 0 ] && { tail -5 $O/arpn.log; exit $rc; }
NFK_LIBRARY=$PWD/build_ab/arpndump/libnfk.so DBG_HS=192,224,288,320,352,354 timeout -k 10 200 python -u tools/dbg_ar_dump.py > $O/arpndump.log 2>&1
rc=$?; grep -h "rep 0" $O/arpndump.log; [ $rc -ne 0 ] && tail -5 $O/arpndump.log; exit $rc

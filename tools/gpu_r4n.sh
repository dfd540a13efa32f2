#!/bin/bash
# Round 4: wide fused NSF_AR KBH 6/9/10 -- intermediate dumps (current code) and the no-packed-FP32 build
set -u
O=gpurun_out/r4n; mkdir -p $O
NFK_LIBRARY=$PWD/build_ab/ardump2/libnfk.so DBG_HS=192,288,320 timeout -k 10 200 python -u tools/dbg_ar_dump.py > $O/dump.log 2>&1
rc=$?; cat $O/dump.log | grep "^H"; [ $rc -ne 0 ] && { tail -5 $O/dump.log; exit $rc; }
for r in 1 2; do
NFK_LIBRARY=$PWD/build_ab/arnopk/libnfk.so DBG_HS=192,288,320 DBG_DIMS=2,8 timeout -k 10 200 python -u tools/dbg_ar_wide.py > $O/nopk$r.log 2>&1
rc=$?; echo "== nopk $r"; grep -h "^H " $O/nopk$r.log; [ $rc -ne 0 ] && { tail -5 $O/nopk$r.log; exit $rc; }
done
exit 0

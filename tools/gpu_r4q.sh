#!/bin/bash
# Round 4: the GEMM fence (MFMAs pinned above the segment barrier) -- wide AR widths, and the fused VJP
# WITH packed-FP32 code, fenced vs unfenced
set -u
O=gpurun_out/r4q; mkdir -p $O
for r in 1 2; do
  NFK_LIBRARY=$PWD/build_ab/arfence/libnfk.so DBG_HS=192,224,288,320,354 DBG_DIMS=2,8 timeout -k 10 200 python -u tools/dbg_ar_wide.py > $O/ar$r.log 2>&1
  rc=$?; echo "== arfence $r"; grep -h "^H " $O/ar$r.log; [ $rc -ne 0 ] && { tail -5 $O/ar$r.log; exit $rc; }
done
for v in vjppk vjppknofence; do
  NFK_LIBRARY=$PWD/build_ab/$v/libnfk.so DBG_ROWS=65536,262144,1048576 DBG_REPS=4 DBG_MODELS=0 timeout -k 10 200 python -u tools/dbg_vjp_poison.py > $O/$v.log 2>&1
  rc=$?; echo "== $v"; grep -h "vjp inv" $O/$v.log | awk '{d=0; for(i=1;i<=NF;i++) if($i=="diff" && $(i+1)+0>d) d=$(i+1)+0; print $1,$2,$3, "maxdiff", d}' | sort | uniq -c; [ $rc -ne 0 ] && { tail -5 $O/$v.log; exit $rc; }
done
exit 0

#!/bin/bash
# Round 4: isolate the wide fused NSF_AR error (H 354 vs 352 vs 130; 2-tile sub-records; one wave per SIMD; VGPR-form MFMA)
set -u
O=gpurun_out/r4g; mkdir -p $O
for v in arshapes arns2 aronew arvgpr; do
  export NFK_LIBRARY=$PWD/build_ab/$v/libnfk.so
  DBG_HS=354,352,130 DBG_DIMS=2,8 timeout -k 10 200 python -u tools/dbg_ar_wide.py > $O/$v.log 2>&1
  rc=$?; echo "== $v rc=$rc"; grep -h "^H " $O/$v.log
  [ $rc -ne 0 ] && { tail -5 $O/$v.log; exit $rc; }
done
exit 0

#!/bin/bash
# Round 5 (c): is the fused VJP's divergence the back-to-back packed-FP32 read-after-write?
# Each variant's device assembly reassembled as compiled (*re) and with s_nop 0 inserted between
# every packed/64-bit VALU write and a packed-FP32 read of it at gap 1 (*nop; tools/patch_pk.py)
set -u
O=gpurun_out/r5c; mkdir -p $O
export TMPDIR=/tmp
for v in fastre fastnop exactre exactnop; do
  echo "== $v"
  DBG_ROWS=262144 DBG_REPS=3 NFK_LIBRARY=$PWD/build_ab/$v/libnfk.so \
    timeout -k 10 240 python -u tools/dbg_vjp_save.py > $O/vjp_$v.log 2>&1
  rc=$?; grep -h "inv=" $O/vjp_$v.log | head -20; [ $rc -ne 0 ] && { tail -5 $O/vjp_$v.log; exit $rc; }
done
echo done

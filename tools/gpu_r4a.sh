#!/bin/bash
# Round 4 diagnostic: fused VJP run-to-run reproducibility per build variant
set -u
mkdir -p gpurun_out/r4a
for v in base nop onewg plain vgprc exact nopk; do
  echo "== $v"
  DBG_ROWS=262144,1048576 DBG_REPS=3 DBG_MODELS=0 NFK_LIBRARY=$PWD/build_ab/$v/libnfk.so \
    timeout -k 10 120 python -u tools/dbg_vjp_poison.py > gpurun_out/r4a/$v.log 2>&1
  rc=$?; grep -h "vjp inv" gpurun_out/r4a/$v.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/r4a/$v.log; exit $rc; }
done
exit 0

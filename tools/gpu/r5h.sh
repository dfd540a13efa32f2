#!/bin/bash
# Round 5 (h): full GPU suite (incl. the forward full-occupancy reproducibility tests and the
# host helper), smoke, then the fused-VJP probe variant (first differing intermediate of two
# evaluations of the element backward on the same registers)
set -u
O=gpurun_out/r5h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -8 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -2 $O/smoke.log
for v in twice probe; do
  echo "== $v"
  DBG_ROWS=262144 DBG_REPS=2 DBG_INV=0 NFK_LIBRARY=$PWD/build_ab/$v/libnfk.so \
    timeout -k 10 240 python -u tools/dbg_vjp_save.py > $O/vjp_$v.log 2>&1
  rc=$?; grep -h "inv=\|twice\|probe" $O/vjp_$v.log | head -24; [ $rc -ne 0 ] && { tail -5 $O/vjp_$v.log; exit $rc; }
done
echo done

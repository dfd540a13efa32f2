#!/bin/bash
# Round 5 (a): GPU suite on the tree (exponent clamp, tiny-row tests, bench self-spawn),
# the fused-VJP input/output capture per build variant (tools/dbg_vjp_save.py), a c3 line
set -u
O=gpurun_out/r5a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in exactsave fastsave nopksave; do
  echo "== $v"
  DBG_ROWS=262144 DBG_REPS=3 NFK_LIBRARY=$PWD/build_ab/$v/libnfk.so \
    timeout -k 10 240 python -u tools/dbg_vjp_save.py > $O/vjp_$v.log 2>&1
  rc=$?; grep -h "inv=" $O/vjp_$v.log | head -20; [ $rc -ne 0 ] && { tail -5 $O/vjp_$v.log; exit $rc; }
done
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
tail -1 $O/c3.json | cut -c1-300
echo done

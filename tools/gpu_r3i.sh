#!/bin/bash
# Round 3 session i: the 32x32 chain, 4-wave (form 2) and ping-pong (form 3):
# parity, then A/B against the two-tile chain (form 1) at 2^20 and 2^17.
set -u
O=gpurun_out/r3i; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -2 $O/$name.log | cut -c1-200; return $rc; }
run chain32_tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_chain32.py || exit $?
for r in 1 2; do
  for f in 1 2 3; do
    NFK_CHAIN_FORM=$f run c3_f${f}_$r 300 python bench.py --no-cpu-baseline --parity-rows 16384 || exit $?
  done
done
for f in 1 2 3; do
  NFK_CHAIN_FORM=$f run c3_f${f}_2e17 300 python bench.py --no-cpu-baseline --batch 131072 --steps 50 || exit $?
done
for f in 1 2 3; do
  grep -h '"value"' $O/c3_f${f}_*.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('form $f', d['config']['global_batch'], d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('mean_ms'), d['parity']['pass'] if d.get('parity') else None)
"
done

#!/bin/bash
# Round 3 session k: 32x32 chain with 4-wave (two per CU) vs 12-wave (one per CU,
# three waves per SIMD) workgroups, against the two-tile chain (form 1).
set -u
O=gpurun_out/r3k; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc=$rc"; return $rc; }
NFK_C32_WAVES=12 run w12_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_chain32.py -k "4096 or round or sample" || exit $?
for r in 1 2; do
  NFK_CHAIN_FORM=1 run f1_$r 300 python bench.py --no-cpu-baseline --parity-rows 4096 || exit $?
  NFK_CHAIN_FORM=2 NFK_C32_WAVES=4 run f2w4_$r 300 python bench.py --no-cpu-baseline --parity-rows 4096 || exit $?
  NFK_CHAIN_FORM=2 NFK_C32_WAVES=12 run f2w12_$r 300 python bench.py --no-cpu-baseline --parity-rows 4096 || exit $?
done
for f in $O/f*.log; do echo -n "$f "; grep -h '"value"' $f | python -c "
import sys,json
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity']['pass'])"; done

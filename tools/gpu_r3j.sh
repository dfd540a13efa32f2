#!/bin/bash
# Round 3 session j: ping-pong wave grouping A/B (waves 0-3/4-7 vs even/odd).
set -u
O=gpurun_out/r3j; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc=$rc"; return $rc; }
NFK_CHAIN_FORM=3 NFK_C32_GROUP=1 run grp1_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_chain32.py -k "f3pingpong and (4096 or round)" || exit $?
for r in 1 2; do
  NFK_CHAIN_FORM=1 run f1_$r 300 python bench.py --no-cpu-baseline --parity-rows 4096 || exit $?
  NFK_CHAIN_FORM=3 NFK_C32_GROUP=0 run f3g0_$r 300 python bench.py --no-cpu-baseline --parity-rows 4096 || exit $?
  NFK_CHAIN_FORM=3 NFK_C32_GROUP=1 run f3g1_$r 300 python bench.py --no-cpu-baseline --parity-rows 4096 || exit $?
done
for f in $O/f*.log; do echo -n "$f "; grep -h '"value"' $f | python -c "
import sys,json
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity']['pass'])"; done

#!/bin/bash
# Round 3 session l: ablations of the 32x32 chain (diagnostic builds, results
# not valid): no weight-record copies after the prologue, no spline epilogue, both.
set -u
O=gpurun_out/r3l; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc=$rc"; return $rc; }
export NFK_CHAIN_FORM=2
for r in 1 2; do
  run base_$r 300 python bench.py --no-cpu-baseline --parity-rows 0 --no-status-checks || exit $?
  for v in c32nostage c32noepi c32both; do
    NFK_LIBRARY=build_ab/$v/libnfk.so run ${v}_$r 300 python bench.py --no-cpu-baseline --parity-rows 0 --no-status-checks || exit $?
  done
done
for f in $O/*.log; do echo -n "$f "; grep -h '"value"' $f | python -c "
import sys,json
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; done

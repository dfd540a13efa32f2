#!/bin/bash
# Round 3 session v: fused AR (16-feature tail) with 4- vs 8-wave workgroups.
set -u
O=gpurun_out/r3v; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc=$rc"; return $rc; }
for r in 1 2; do
  NFK_AR_WAVES=4 run w4_$r 300 python bench.py --workload ar --no-cpu-baseline --parity-rows 2048 || exit $?
  NFK_AR_WAVES=8 run w8_$r 300 python bench.py --workload ar --no-cpu-baseline --parity-rows 2048 || exit $?
done
for f in $O/w*.log; do echo -n "$f "; grep -h '"value"' $f | python -c "
import sys,json
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity']['pass'])"; done

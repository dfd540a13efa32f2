#!/bin/bash
# Round 3 session w: compiler scheduling strategies (whole library built with
# -mllvm -amdgpu-sched-strategy=gcn-max-ilp / gcn-max-memory-clause,
# -amdgpu-set-wave-priority) vs the default, c3 and ar.
set -u
O=gpurun_out/r3w; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc=$rc"; return $rc; }
for r in 1 2; do
  run c3_tree_$r 300 python bench.py --no-cpu-baseline --parity-rows 4096 || exit $?
  for v in maxilp memclause wprio; do
    NFK_LIBRARY=build_ab/$v/libnfk.so run c3_${v}_$r 300 python bench.py --no-cpu-baseline --parity-rows 4096 || exit $?
  done
done
run ar_tree 300 python bench.py --workload ar --no-cpu-baseline --parity-rows 2048 || exit $?
for v in maxilp memclause wprio; do
  NFK_LIBRARY=build_ab/$v/libnfk.so run ar_$v 300 python bench.py --workload ar --no-cpu-baseline --parity-rows 2048 || exit $?
done
for f in $O/*.log; do echo -n "$f "; grep -h '"value"' $f | python -c "
import sys,json
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity']['pass'])"; done

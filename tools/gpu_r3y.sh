#!/bin/bash
# Round 3 session y: two-tile chain with two-tile sub-records through two
# slots (one barrier per sub-record, no copy waited for right after its
# issue) vs HEAD (one slot, four-tile sub-records).
set -u
O=gpurun_out/r3y; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc=$rc"; return $rc; }
run tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_parity.py tests/test_gpu_errors.py tests/test_gpu_graphs.py || exit $?
for r in 1 2 3; do
  NFK_LIBRARY=build_ab/head/libnfk.so run head_$r 300 python bench.py --no-cpu-baseline --parity-rows 4096 || exit $?
  run tree_$r 300 python bench.py --no-cpu-baseline --parity-rows 4096 || exit $?
done
NFK_LIBRARY=build_ab/head/libnfk.so run head_2e17 300 python bench.py --no-cpu-baseline --batch 131072 --steps 50 || exit $?
run tree_2e17 300 python bench.py --no-cpu-baseline --batch 131072 --steps 50 || exit $?
for f in $O/head_*.log $O/tree_*.log; do echo -n "$f "; grep -h '"value"' $f | python -c "
import sys,json
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity']['pass'])"; done

#!/bin/bash
# Round 3 session o: the two-tile chain's branch-free reads, A/B of build
# variants: v0 (none), v1 (knot edge select), v2 (+ spline-input reads),
# tree (+ layer-1 reads).
set -u
O=gpurun_out/r3o; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc=$rc"; return $rc; }
run tests 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_parity.py || exit $?
for r in 1 2; do
  for v in v0 v1 v2; do
    NFK_LIBRARY=build_ab/$v/libnfk.so run ${v}_$r 300 python bench.py --no-cpu-baseline --parity-rows 4096 || exit $?
  done
  run tree_$r 300 python bench.py --no-cpu-baseline --parity-rows 4096 || exit $?
done
for f in $O/v*.log $O/tree*.log; do echo -n "$f "; grep -h '"value"' $f | python -c "
import sys,json
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity']['pass'])"; done
# fused AR: the staging cursor (no 64-bit division per sub-record) vs HEAD
run ar_tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_nsfar_fused.py || exit $?
for r in 1 2; do
  NFK_LIBRARY=build_ab/head/libnfk.so run ar_head_$r 300 python bench.py --workload ar --no-cpu-baseline --parity-rows 2048 || exit $?
  run ar_tree_$r 300 python bench.py --workload ar --no-cpu-baseline --parity-rows 2048 || exit $?
done
for f in $O/ar_*.log; do echo -n "$f "; grep -h '"value"' $f | python -c "
import sys,json
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity']['pass'])"; done

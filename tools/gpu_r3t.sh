#!/bin/bash
# Round 3 session t: fused AR with a 16-feature tail step (H = 80 as 64 + 16)
# vs HEAD (H padded to 96): parity, forward / inverse A/B.
set -u
O=gpurun_out/r3t; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc=$rc"; return $rc; }
run ar_tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_nsfar_fused.py || exit $?
for r in 1 2; do
  NFK_LIBRARY=build_ab/head/libnfk.so run ar_head_$r 300 python bench.py --workload ar --no-cpu-baseline --parity-rows 2048 || exit $?
  run ar_tree_$r 300 python bench.py --workload ar --no-cpu-baseline --parity-rows 2048 || exit $?
done
NFK_LIBRARY=build_ab/head/libnfk.so run inv_head 200 python tools/diag/ar_inverse_time.py || exit $?
run inv_tree 200 python tools/diag/ar_inverse_time.py || exit $?
for f in $O/ar_*_*.log; do echo -n "$f "; grep -h '"value"' $f | python -c "
import sys,json
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity']['pass'])"; done
tail -n1 $O/inv_*.log

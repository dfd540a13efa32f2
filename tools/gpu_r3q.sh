#!/bin/bash
# Round 3 session q: fused AR with LDS-DMA spline inputs and unconditional
# prologue loads vs HEAD; two-tile chain with s_setprio over its GEMMs (prio1).
set -u
O=gpurun_out/r3q; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc=$rc"; return $rc; }
run ar_tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_nsfar_fused.py || exit $?
for r in 1 2; do
  NFK_LIBRARY=build_ab/head/libnfk.so run ar_head_$r 300 python bench.py --workload ar --no-cpu-baseline --parity-rows 2048 || exit $?
  run ar_tree_$r 300 python bench.py --workload ar --no-cpu-baseline --parity-rows 2048 || exit $?
  NFK_LIBRARY=build_ab/prio1/libnfk.so run c3_prio1_$r 300 python bench.py --no-cpu-baseline --parity-rows 4096 || exit $?
  run c3_tree_$r 300 python bench.py --no-cpu-baseline --parity-rows 4096 || exit $?
done
run ar_inv 300 python tools/diag/ar_inverse_time.py || true
for f in $O/ar_*_*.log $O/c3_*.log; do echo -n "$f "; grep -h '"value"' $f | python -c "
import sys,json
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity']['pass'])"; done
cat $O/ar_inv.log | tail -5

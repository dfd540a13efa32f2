#!/bin/bash
# Round 3 session z: fused AR sub-record size (tiles per sub-record: 3 default,
# 5 = whole hidden layers, 2) x workgroup size (4 / 8 waves).
set -u
O=gpurun_out/r3z; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc=$rc"; return $rc; }
NFK_LIBRARY=build_ab/arns5/libnfk.so NFK_AR_WAVES=8 run ns5_tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_nsfar_fused.py -k "d40 or 3000 or 2049" || exit $?
for w in 4 8; do
  NFK_AR_WAVES=$w run ns3_w$w 300 python bench.py --workload ar --no-cpu-baseline --parity-rows 2048 || exit $?
  NFK_LIBRARY=build_ab/arns5/libnfk.so NFK_AR_WAVES=$w run ns5_w$w 300 python bench.py --workload ar --no-cpu-baseline --parity-rows 2048 || exit $?
  NFK_LIBRARY=build_ab/arns2/libnfk.so NFK_AR_WAVES=$w run ns2_w$w 300 python bench.py --workload ar --no-cpu-baseline --parity-rows 2048 || exit $?
done
for f in $O/ns*_w*.log; do echo -n "$f "; grep -h '"value"' $f | python -c "
import sys,json
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity']['pass'])"; done

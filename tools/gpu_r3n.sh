#!/bin/bash
# Round 3 session n: spline constants held by value (SGPRs) in the fused
# kernels -- chain / chain32 / wide parity, then A/B against the HEAD build.
set -u
O=gpurun_out/r3n; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc=$rc"; return $rc; }
run tests 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_chain32.py tests/test_gpu_wide.py || exit $?
for r in 1 2; do
  NFK_LIBRARY=build_ab/head/libnfk.so run head_f1_$r 300 python bench.py --no-cpu-baseline --parity-rows 4096 || exit $?
  NFK_CHAIN_FORM=1 run f1_$r 300 python bench.py --no-cpu-baseline --parity-rows 4096 || exit $?
  for w in 4 8 12; do
    NFK_CHAIN_FORM=2 NFK_C32_WAVES=$w run f2w${w}_$r 300 python bench.py --no-cpu-baseline --parity-rows 4096 || exit $?
  done
done
NFK_LIBRARY=build_ab/head/libnfk.so run head_c5 300 python bench.py --workload c5 --steps 10 --no-cpu-baseline --parity-rows 2048 || exit $?
run c5 300 python bench.py --workload c5 --steps 10 --no-cpu-baseline --parity-rows 2048 || exit $?
for f in $O/*f*.log $O/*c5.log; do echo -n "$f "; grep -h '"value"' $f | python -c "
import sys,json
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity']['pass'])"; done

#!/bin/bash
# Round 3 session c: unfused ar, chain2 tests + A/B vs the one-tile chain, c3 bench, GPU suite, rocprof.
set -u
O=gpurun_out/r3c; mkdir -p $O
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; tail -3 $O/$n.log
  [ $rc -eq 0 ] || exit $rc
}
#run bench_ar_unfused 400 python bench.py --workload ar --unfused --steps 2 --warmup 1 --no-cpu-baseline --parity-rows 2048
NFK_CHAIN2=1 run chain2_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_parity.py -k "chain or c3"
for r in 1 2; do
  NFK_CHAIN2=0 run c3_one_$r 300 python bench.py --no-cpu-baseline --parity-rows 16384
  NFK_CHAIN2=1 run c3_two_$r 300 python bench.py --no-cpu-baseline --parity-rows 16384
done
NFK_CHAIN2=0 run c3_one_2e17 300 python bench.py --no-cpu-baseline --batch 131072 --steps 50
NFK_CHAIN2=1 run c3_two_2e17 300 python bench.py --no-cpu-baseline --batch 131072 --steps 50

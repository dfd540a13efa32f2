#!/bin/bash
# Round 3 session g: the 32x32x16 chain (form 2) -- parity, then A/B against
# the two-tile chain (form 1) at 2^20 and 2^17; c5 with whole-line z stores.
set -u
O=gpurun_out/r3g; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -3 $O/$name.log | cut -c1-300; return $rc; }
run chain32_tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_chain32.py || exit $?
for r in 1 2; do
  NFK_CHAIN_FORM=1 run c3_f1_$r 300 python bench.py --no-cpu-baseline --parity-rows 16384 || exit $?
  NFK_CHAIN_FORM=2 run c3_f2_$r 300 python bench.py --no-cpu-baseline --parity-rows 16384 || exit $?
done
NFK_CHAIN_FORM=1 run c3_f1_2e17 300 python bench.py --no-cpu-baseline --batch 131072 --steps 50 || exit $?
NFK_CHAIN_FORM=2 run c3_f2_2e17 300 python bench.py --no-cpu-baseline --batch 131072 --steps 50 || exit $?
run c5_tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wide.py || exit $?
run c5_bench 300 python bench.py --workload c5 --no-cpu-baseline --parity-rows 4096 || exit $?
grep -h '"value"' $O/*.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['config']['workload'][:3], d['config']['global_batch'], d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('mean_ms'))
"

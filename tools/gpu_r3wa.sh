#!/bin/bash
# Round 3, wide kernel: two sample tiles per wave (NFK_WIDE_FORM=2) vs one:
# parity tests, then c5 bench lines of both forms alternated on one box.
set -u
O=gpurun_out/${TAG:-r3wa}; mkdir -p $O
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; tail -2 $O/$n.log | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
run pytest_wide 400 python -u -m pytest tests/test_gpu_wide.py -x -v --timeout 120 --timeout-method thread
for i in 1 2; do
  NFK_WIDE_FORM=1 run c5_f1_$i 300 python bench.py --workload c5 --no-cpu-baseline --steps 5 --warmup 2
  NFK_WIDE_FORM=2 run c5_f2_$i 300 python bench.py --workload c5 --no-cpu-baseline --steps 5 --warmup 2
done

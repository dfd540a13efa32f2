#!/bin/bash
# c5: one vs two sample tiles per wave, full and without frame copies after the prologue
set -u
O=gpurun_out/r3wd; mkdir -p $O
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; tail -1 $O/$n.log | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
}
for f in 1 2; do
  NFK_WIDE_FORM=$f run c5_f${f} 300 python bench.py --workload c5 --no-cpu-baseline --steps 5 --warmup 2
  NFK_WIDE_FORM=$f NFK_LIBRARY=$PWD/normalizingflow_amd/libnfk_wabl_nostage.so run c5_f${f}_nostage 300 python bench.py --workload c5 --no-cpu-baseline --parity-rows 0 --steps 5 --warmup 2
done

#!/bin/bash
# Round 5 (q): what bounds the fused NSF_AR at the applications' batches -- HEAD vs 1-tile
# sub-records for the wide conditioners (nsw1: twice the sub-records, half the bytes each)
# vs every copy waited for before its GEMM (arsync: no copy in flight during a GEMM);
# forward at the training batch, inverse at sample(500)
set -u
O=gpurun_out/r5q; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in cur nsw1 arsync; do
    if [ $v = cur ]; then unset NFK_LIBRARY; else export NFK_LIBRARY=build_ab/$v/libnfk.so; fi
    for shape in "96 354 32 40 500" "162 354 32 50 500"; do
      timeout -k 10 200 python tools/time_ar.py $shape > $O/t-$v-$r.txt 2>&1 || { tail -5 $O/t-$v-$r.txt; exit 1; }
      echo "$v $r: $(tail -1 $O/t-$v-$r.txt)"
    done
  done
done
unset NFK_LIBRARY
echo done

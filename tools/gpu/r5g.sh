#!/bin/bash
# Round 5 (g): transcendental -> packed-FP32 read microbenchmark under contention
# (tools/ubench_trans_pk2.hip); same-box c3 A/B of the branch-free chain2 map reads
# (product build) vs the previous chain2 (build_ab/c2old), alternating
set -u
O=gpurun_out/r5g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 ./tools/ubench_trans_pk2 > $O/ubench_trans_pk2.txt 2>&1 || { tail -5 $O/ubench_trans_pk2.txt; exit 1; }
cat $O/ubench_trans_pk2.txt
for i in 1 2 3; do
  for v in base c2old; do
    L=""; [ $v = c2old ] && L="NFK_LIBRARY=$PWD/build_ab/c2old/libnfk.so"
    env $L timeout -k 10 200 python bench.py --no-cpu-baseline --parity-rows 2048 > $O/c3_${v}_$i.json 2> $O/c3_${v}_$i.err || { tail -5 $O/c3_${v}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$O/c3_${v}_$i.json'));print('c3 $v $i', round(d['value']/1e6,2),'M/s', d['roofline']['mean_ms'],'ms')"
  done
done
echo done

#!/bin/bash
# Round 4: c3 chain (k_nsf_chain2) A/B over build variants, alternating, 2 rounds
set -u
O=gpurun_out/r4o; mkdir -p $O
for r in 1 2; do
  for v in c2base c2nopk c2lut0 c2pk2; do
    NFK_LIBRARY=$PWD/build_ab/$v/libnfk.so timeout -k 10 200 python bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline > $O/$v-$r.json 2> $O/$v-$r.err || { echo "bench $v failed"; tail -5 $O/$v-$r.err; exit 1; }
    echo "$v $r: $(python -c "import json; d=json.loads(open('$O/$v-$r.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['mean_ms'])")"
  done
done

#!/bin/bash
# Round 5 (r): A/B of the 6-VALU tanh (NFK_TANH6: 2^15/(1+t) - 2^14 instead of (1-t)/((1+t)/2^14))
# on c3, c2, c5 (parity on 16 K / 4 K rows each run)
set -u
O=gpurun_out/r5r; mkdir -p $O
export TMPDIR=/tmp
for w in c3 c2; do
  for r in 1 2 3; do
    for v in cur tanh6; do
      if [ $v = cur ]; then unset NFK_LIBRARY; else export NFK_LIBRARY=build_ab/$v/libnfk.so; fi
      timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > $O/$w-$v-$r.json 2> $O/$w-$v-$r.err || { echo "bench $w $v failed"; tail -5 $O/$w-$v-$r.err; exit 1; }
      echo "$w $v $r: $(python3 tools/bench_line.py $O/$w-$v-$r.json) $(python3 -c "import json;d=json.load(open('$O/$w-$v-$r.json'));r=d['roofline'];p=d['parity'];print(r['kernel'],r['mean_ms'],'maxrel',p['max_rel_dlog_prob'])")"
    done
  done
done
unset NFK_LIBRARY
echo done

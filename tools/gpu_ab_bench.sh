#!/bin/bash
# A/B of bench.py lines: working tree vs build_ab/$1, alternating, per workload
# usage: bash tools/gpu_ab_bench.sh VARIANT "c3 c2 c5" [reps]
set -u
V=$1; WL=${2:-c3}; REPS=${3:-2}
O=gpurun_out/ab; mkdir -p $O
for w in $WL; do
  for r in $(seq $REPS); do
    for v in cur $V; do
      if [ $v = cur ]; then unset NFK_LIBRARY; else export NFK_LIBRARY=build_ab/$v/libnfk.so; fi
      timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --parity-rows 4096 > $O/$w-$v-$r.json 2> $O/$w-$v-$r.err || { echo "bench $w $v failed"; tail -5 $O/$w-$v-$r.err; exit 1; }
      echo "$w $v $r: $(python3 tools/bench_line.py $O/$w-$v-$r.json)"
    done
  done
done

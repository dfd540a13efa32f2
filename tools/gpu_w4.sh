# A/B: default build vs the 4-waves-per-SIMD chain (build_ab/w4) at c3 per-rank sizes
set -u
O=gpurun_out/w4; mkdir -p $O
for r in 1 2; do
for b in 131072 1048576; do
  for v in cur w4; do
    if [ $v = cur ]; then unset NFK_LIBRARY; else export NFK_LIBRARY=build_ab/w4/libnfk.so; fi
    timeout -k 10 200 python bench.py --batch $b --steps 20 --warmup 3 --no-cpu-baseline --parity-rows 4096 > $O/$b-$v-$r.json 2> $O/$b-$v-$r.err || { echo "bench $b $v failed"; tail -5 $O/$b-$v-$r.err; exit 1; }
    echo "$b $v $r: $(python3 tools/bench_line.py $O/$b-$v-$r.json)"
  done
done
done

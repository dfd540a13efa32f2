# c3 at serving batch sizes, eager vs HIP-graph replay (graphs.GraphedLogProb)
set -u
O=gpurun_out/serving; mkdir -p $O
for b in 4096 65536; do
  for gr in off on; do
    timeout -k 10 200 python bench.py --batch $b --graph $gr --steps 50 --warmup 5 --no-cpu-baseline --parity-rows 1024 > $O/c3_b${b}_g$gr.json 2> $O/c3_b${b}_g$gr.err; rc=$?
    echo "c3 b=$b graph=$gr rc=$rc: $(python3 tools/bench_line.py $O/c3_b${b}_g$gr.json)"; [ $rc -eq 0 ] || exit $rc
  done
done

# round-2 closing measurements: strong-scaling per-rank sizes of c3, c2, c5 bench lines
set -u
OUT=gpurun_out/r2j; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_graphs.py tests/test_gpu_grad.py -k "graph or realnvp" -rs > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for b in 524288 262144 131072; do
  timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --parity-rows 4096 > $OUT/c3_b$b.json 2> $OUT/c3_b$b.err; rc=$?
  echo "c3 b=$b rc=$rc"; cut -c1-220 $OUT/c3_b$b.json; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python bench.py --workload c2 > $OUT/c2.json 2> $OUT/c2.err; rc=$?; echo "c2 rc=$rc"; cut -c1-220 $OUT/c2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err; rc=$?; echo "c5 rc=$rc"; cut -c1-220 $OUT/c5.json; [ $rc -eq 0 ] || exit $rc
exit 0

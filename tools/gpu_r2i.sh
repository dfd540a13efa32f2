set -u
OUT=gpurun_out/r2i; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rnvp_chain.py tests/test_gpu_graphs.py tests/test_gpu_parity.py tests/test_gpu_grad.py -rs > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --workload c1 > $OUT/c1_graph.json 2> $OUT/c1_graph.err; rc=$?; echo "c1 graph rc=$rc"; cat $OUT/c1_graph.json; tail -3 $OUT/c1_graph.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --workload c1 --graph off --no-cpu-baseline > $OUT/c1_eager.json 2> $OUT/c1_eager.err; rc=$?; echo "c1 eager rc=$rc"; cat $OUT/c1_eager.json; [ $rc -eq 0 ] || exit $rc
exit 0

set -o pipefail
mkdir -p gpurun_out/wide1
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -v --timeout 120 --timeout-method thread > gpurun_out/wide1/pytest.log 2>&1; rc=$?
tail -30 gpurun_out/wide1/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/wide1/bench_c5.json 2> gpurun_out/wide1/bench_c5.err; rc=$?
cat gpurun_out/wide1/bench_c5.json; tail -3 gpurun_out/wide1/bench_c5.err
exit $rc

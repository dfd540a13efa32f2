#!/bin/bash
# Round 3 session b: fused NSF_AR tests, the GPU suite, c3 / ar benches, rocprof of c3.
set -u
O=gpurun_out/r3b; mkdir -p $O
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; tail -4 $O/$n.log
  [ $rc -eq 0 ] || exit $rc
}
#run ar_tests 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_nsfar_fused.py
#run bench_ar 300 python bench.py --workload ar --steps 10 --warmup 2
run bench_ar_unfused 400 python bench.py --workload ar --unfused --steps 2 --warmup 1 --no-cpu-baseline --parity-rows 2048
run bench_c3 300 python bench.py
run pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
export TMPDIR=/tmp
run prof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o trace -- python3 bench.py --no-cpu-baseline
run prof_ar 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ar -o trace -- python3 bench.py --workload ar --no-cpu-baseline

#!/bin/bash
# Round 3 session s (validation of the tuned chain): the GPU suite, smoke, c3 / ar / c2 / c5 bench
# lines, rocprofv3 kernel stats of the c3 and ar benches.
set -u
O=gpurun_out/r3s; mkdir -p $O
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; tail -2 $O/$n.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_c3 300 python bench.py
export TMPDIR=/tmp
run prof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o trace -- python3 bench.py --no-cpu-baseline
run bench_ar 300 python bench.py --workload ar
run prof_ar 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ar -o trace -- python3 bench.py --workload ar --no-cpu-baseline
run bench_c2 300 python bench.py --workload c2 --no-cpu-baseline
run bench_c5 300 python bench.py --workload c5 --no-cpu-baseline
run bench_c3_2e17 300 python bench.py --batch 131072 --steps 50 --no-cpu-baseline

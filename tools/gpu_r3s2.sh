#!/bin/bash
# Round 3 session s, part 2: c3 / ar / c2 / c5 bench lines, rocprofv3 kernel
# stats of the c3 and ar benches, c3 at 2^17.
set -u
O=gpurun_out/r3s; mkdir -p $O
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; tail -2 $O/$n.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
run bench_c3 300 python bench.py
export TMPDIR=/tmp
run prof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o trace -- python3 bench.py --no-cpu-baseline
run bench_ar 300 python bench.py --workload ar
run prof_ar 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ar -o trace -- python3 bench.py --workload ar --no-cpu-baseline
run bench_c2 300 python bench.py --workload c2 --no-cpu-baseline
run bench_c5 300 python bench.py --workload c5 --no-cpu-baseline
run bench_c3_2e17 300 python bench.py --batch 131072 --steps 50 --no-cpu-baseline
# HBM traffic of this build's kernels (pmc_traffic.json)
bash tools/pmc_traffic_passes.sh r3s_tr_c3 "k_nsf_chain2" --workload c3 || exit $?
bash tools/pmc_traffic_passes.sh r3s_tr_c2 "k_rnvp_chain" --workload c2 || exit $?
bash tools/pmc_traffic_passes.sh r3s_tr_c5 "k_fused_nsf_wide" --workload c5 --steps 1 || exit $?
bash tools/pmc_traffic_passes.sh r3s_tr_ar "k_fused_ar" --workload ar || exit $?

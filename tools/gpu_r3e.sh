#!/bin/bash
# Round 3 session e: PMC passes (HBM bytes, instruction mix, pipe busy) of the
# HEAD build's c3 chain, fused NSF_AR and c5 wide kernels; small-batch AR A/B.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/pmc_passes.sh r3e_c3 "k_nsf_chain2" --workload c3 || exit $?
bash tools/pmc_passes.sh r3e_ar "k_fused_ar" --workload ar || exit $?
bash tools/pmc_passes.sh r3e_c5 "k_fused_nsf_wide" --workload c5 || exit $?
O=gpurun_out/r3e; mkdir -p $O
for b in 4096 65536; do
  timeout -k 10 300 python bench.py --workload ar --batch $b --steps 20 --no-cpu-baseline --parity-rows 1024 > $O/ar_fused_$b.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --workload ar --batch $b --steps 5 --warmup 2 --unfused --no-cpu-baseline --parity-rows 1024 > $O/ar_unfused_$b.log 2>&1 || exit $?
  grep -h '"value"' $O/ar_fused_$b.log $O/ar_unfused_$b.log | cut -c1-200
done

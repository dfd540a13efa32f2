#!/bin/bash
# c5 wide-kernel ablations + PMC passes (one GPU call)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
STEPS=4 BENCH_ARGS="--workload c5" bash tools/gpu_variants.sh wabl libnfk.so libnfk_wabl_l2hot.so libnfk_wabl_noepi.so libnfk_wabl_l2hot_noepi.so libnfk_wabl_nostage_noepi.so || exit $?
bash tools/pmc_passes.sh wpmc k_fused_nsf_wide --workload c5 || exit $?
python tools/pmc_summary.py gpurun_out/wpmc > gpurun_out/wpmc/summary.txt 2>&1; cat gpurun_out/wpmc/summary.txt | head -60

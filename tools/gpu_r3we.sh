#!/bin/bash
# c5 PMC passes of the two-tile pipelined wide form (NFK_WIDE_FORM=2)
set -u
NFK_WIDE_FORM=2 bash tools/pmc_passes.sh r3we_pmc_c5_f2 k_fused_nsf_wide --workload c5 --steps 1 || exit $?
python tools/pmc_summary.py gpurun_out/r3we_pmc_c5_f2 > gpurun_out/r3we_pmc_c5_f2/summary.txt 2>&1; head -50 gpurun_out/r3we_pmc_c5_f2/summary.txt

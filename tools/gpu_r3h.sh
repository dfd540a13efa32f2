#!/bin/bash
# Round 3 session h: PMC passes of the 32x32x16 chain (form 2) at c3.
set -u
export NFK_CHAIN_FORM=2
bash tools/pmc_passes.sh r3h_c3f2 "k_nsf_chain32" --workload c3 || exit $?

#!/bin/bash
# Round 6 (am): c3 PMC passes on the final build (instruction mix, co-execution, traffic)
set -u
timeout -k 10 900 bash tools/pmc_passes.sh r6am 'k_nsf_chain2' --graph off

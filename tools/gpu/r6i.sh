#!/bin/bash
# Round 6 (i): phase clocks of the sequential NSF_AR inverse
set -u
O=gpurun_out/r6i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/sq_phase_timing.py > $O/phases.json 2> $O/phases.err; rc=$?
cat $O/phases.json; tail -3 $O/phases.err
exit $rc

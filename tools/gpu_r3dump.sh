#!/bin/bash
# Diagnostic: the fused VJP kernel with the element backward replaced by a pass-through of
# its inputs (logits in gp, x / gz / gld folded into gx): which inputs differ run to run.
set -u
mkdir -p gpurun_out
PYTHONPATH=. DBG_ROWS=262144,1048576 NFK_LIBRARY=$PWD/build_ab/vjpdump/libnfk.so timeout -k 10 200 python tools/dbg_vjp_det.py > gpurun_out/vjp_dump.txt 2>&1
rc=$?; grep -h "kernel g" gpurun_out/vjp_dump.txt; exit $rc

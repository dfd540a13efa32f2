#!/bin/bash
# Diagnostic: the fused VJP kernel built with the exact element math (NFK_VJP_FAST=0): reproducible?
set -u
mkdir -p gpurun_out
PYTHONPATH=. DBG_ROWS=262144,1048576 NFK_LIBRARY=$PWD/build_ab/vjpexact/libnfk.so timeout -k 10 200 python tools/dbg_vjp_det.py > gpurun_out/vjp_exact.txt 2>&1
rc=$?; grep -h "kernel g\|rep 1" gpurun_out/vjp_exact.txt; exit $rc

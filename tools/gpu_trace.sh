#!/bin/bash
# timeline of the wide kernel (trace build) on the c5 layer, forward and inverse
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; mkdir -p gpurun_out/trace
NFK_LIBRARY=$ROOT/normalizingflow_amd/libnfk_trace.so timeout -k 10 200 python tools/trace_wide.py "$@" > gpurun_out/trace/fwd.txt 2>&1; rc=$?
cat gpurun_out/trace/fwd.txt; [ $rc -eq 0 ] || exit $rc

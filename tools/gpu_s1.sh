#!/bin/bash
# single-slot 4-wave variant of the narrow kernel: parity, bench vs default, timeline
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; mkdir -p gpurun_out/s1
V=${V:-libnfk_s1w4}
NFK_LIBRARY=$ROOT/normalizingflow_amd/$V.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
   -k "c3 or golden or dim3 or large_n_up" > gpurun_out/s1/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/s1/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_variants.sh s1 libnfk.so $V.so || exit $?
if [ -f normalizingflow_amd/${V}_trace.so ]; then
NFK_LIBRARY=$ROOT/normalizingflow_amd/${V}_trace.so timeout -k 10 200 python tools/trace_wide.py --c3 > gpurun_out/s1/trace.txt 2>&1; rc=$?
cat gpurun_out/s1/trace.txt; [ $rc -eq 0 ] || exit $rc
fi

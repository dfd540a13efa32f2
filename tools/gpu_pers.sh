#!/bin/bash
# parity of the current libnfk.so, then bench vs the given variants
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; T=${T:-pers}; mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
   -k "c3 or golden or dim3 or large_n_up or ragged" > gpurun_out/$T/pytest.log 2>&1; rc=$?
echo "parity rc=$rc"; tail -4 gpurun_out/$T/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_variants.sh $T libnfk.so "$@" || exit $?

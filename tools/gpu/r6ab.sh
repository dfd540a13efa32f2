#!/bin/bash
# Round 6 (ab): c3 log_prob error against fp64 beside the reference's fp32 error
set -u
O=gpurun_out/r6ab; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -rP --timeout 300 --timeout-method thread -k "fp64" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|c3 log_prob vs fp64|assert" $O/pytest.log | tail -8
exit $rc

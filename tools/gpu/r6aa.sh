#!/bin/bash
# Round 6 (aa): nfk_ar_seqinv over its supported hidden widths and K
set -u
O=gpurun_out/r6aa; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_nsfar_fused.py -m gpu -v -rP --timeout 300 --timeout-method thread -k "seqinv" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error|assert" $O/pytest.log | tail -8
exit $rc

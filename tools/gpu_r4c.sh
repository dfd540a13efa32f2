#!/bin/bash
# Round 4: per-sample input scaling -- outlier tests + the whole GPU suite, then the no-packed-fp32 runs (r4b)
set -u
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_outlier.py -x -v --timeout 120 --timeout-method thread > $O/outlier.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $O/outlier.log | tail -25; [ $rc -ne 0 ] && { grep -B5 -A30 "Error\|assert" $O/outlier.log | head -80; exit $rc; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -ne 0 ] && { grep -B5 -A40 "^____\|Error" $O/suite.log | head -80; exit $rc; }
bash tools/gpu_r4b.sh

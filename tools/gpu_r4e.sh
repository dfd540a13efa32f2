#!/bin/bash
# Round 4: wide fused NSF_AR (H = 354) parity, then the VJP/outlier tests, train step and the suite
set -u
O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_nsfar_fused.py -x -v --timeout 200 --timeout-method thread > $O/ar.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $O/ar.log | tail -20; [ $rc -ne 0 ] && { grep -B5 -A30 "Error\|assert" $O/ar.log | head -60; exit $rc; }
bash tools/gpu_r4d.sh

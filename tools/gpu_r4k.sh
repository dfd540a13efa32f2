#!/bin/bash
# Round 4: wide fused NSF_AR with sub-record-relative biases and the post-GEMM wait
set -u
O=gpurun_out/r4k; mkdir -p $O
DBG_HS=354 DBG_DIMS=2,8,96 timeout -k 10 300 python -u tools/dbg_ar_wide.py > $O/arw.log 2>&1
rc=$?; grep -h "^H " $O/arw.log; [ $rc -ne 0 ] && { tail -5 $O/arw.log; exit $rc; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_nsfar_fused.py -x -v --timeout 300 --timeout-method thread > $O/ar.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $O/ar.log | tail -20; [ $rc -ne 0 ] && { grep -B5 -A30 "Error\|assert" $O/ar.log | head -60; exit $rc; }
bash tools/gpu_r4d.sh

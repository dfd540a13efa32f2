#!/bin/bash
# Round 6 (x): one-wave workgroups for the wide NSF_AR inverse at sampling batches
# (NFK_AR_INV_WAVES and the one-wave inverse it selected were measured slower and removed; profiles/r6/r6x_ar_inverse_waves_ab.txt)
set -u
O=gpurun_out/r6x; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_nsfar_fused.py tests/test_gpu_parity.py tests/test_gpu_forward_repro.py -m gpu -q -rP --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error" $O/pytest.log | tail -5
[ $rc -ne 0 ] && exit $rc
NFK_AR_INV_WAVES=4 timeout -k 10 300 python3 tools/time_ar_sample.py > $O/sample_w4.json 2> $O/sample_w4.err || { tail -5 $O/sample_w4.err; exit 1; }
timeout -k 10 300 python3 tools/time_ar_sample.py > $O/sample_w1.json 2> $O/sample_w1.err || { tail -5 $O/sample_w1.err; exit 1; }
grep -h "einstein96\|fe162" $O/sample_w4.err $O/sample_w1.err
echo done

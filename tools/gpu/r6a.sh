#!/bin/bash
# Round 6 (a): NSF_AR parity against the fp64 companions, host-helper watch and
# copies, row-block chunking of the streamed form
set -u
O=gpurun_out/r6a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_nsfar_fused.py tests/test_gpu_parity.py tests/test_host_helper.py -m gpu -v -rP --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" $O/pytest.log | tail -3
exit $rc

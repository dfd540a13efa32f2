#!/bin/bash
# Round 5 (d): the NSF_AR tests (streamed Polymer form bitwise vs the register form, Polymer
# forward speed, Fe), then tools/gpu/r5c.sh (the packed-FP32 nop-patch VJP experiment)
set -u
O=gpurun_out/r5d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_nsfar_fused.py -q -rf -s --timeout 300 --timeout-method thread > $O/pytest_ar.log 2>&1; echo "pytest_ar rc=$?"; grep -E "passed|failed|fe162|poly2048" $O/pytest_ar.log | tail -6
bash tools/gpu/r5c.sh

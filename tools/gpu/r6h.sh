#!/bin/bash
# Round 6 (h): sequential NSF_AR inverse, operands prefetched, padded weight rows
set -u
O=gpurun_out/r6h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_nsfar_fused.py -m gpu -v -rP --timeout 300 --timeout-method thread -k "seqinv or polymer2048" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error|poly2048" $O/pytest.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_seqinv -o run -- python3 tools/time_ar_sample.py > $O/prof_seqinv.log 2>&1 || { tail -5 $O/prof_seqinv.log; exit 1; }
grep -A6 polymer2048 $O/prof_seqinv.log | head -8
echo done

#!/bin/bash
# Round 6 (c): the weight-stream RealNVP (nfk_wide_rnvp) -- parity vs the
# library path / oracle / golden, reproducibility; timing both paths; rocprof
set -u
O=gpurun_out/r6c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rnvp_polymer.py -m gpu -v -rP --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error" $O/pytest.log | tail -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/time_rnvp2048.py > $O/time_rnvp2048.json 2> $O/time_rnvp2048.err || { tail -5 $O/time_rnvp2048.err; exit 1; }
cat $O/time_rnvp2048.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/time_rnvp2048.py > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
echo done

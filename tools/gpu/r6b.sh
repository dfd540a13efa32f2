#!/bin/bash
# Round 6 (b): Polymer_rnvp (RealNVP 2048 x 4000) parity and timing on the
# library-GEMM path; full-occupancy repro of the H=354 NSF_AR instances
set -u
O=gpurun_out/r6b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rnvp_polymer.py "tests/test_gpu_forward_repro.py::test_fused_ar_h354_reproducible" -m gpu -v -rP --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" $O/pytest.log | tail -3
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/time_rnvp2048.py > $O/time_rnvp2048.json 2> $O/time_rnvp2048.err || { tail -5 $O/time_rnvp2048.err; exit 1; }
cat $O/time_rnvp2048.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/time_rnvp2048.py > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
echo done

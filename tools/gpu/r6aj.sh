#!/bin/bash
# Round 6 (aj): the default bench line (c3, graph replay) and bench.py's own distributed tests
set -u
O=gpurun_out/r6aj; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { tail -5 $O/bench_c3.err; exit 1; }
tail -1 $O/bench_c3.json | cut -c1-400
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_dist.py tests/test_gpu_graphs.py -m gpu -q -rP --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest.log
exit $rc

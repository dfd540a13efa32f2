#!/bin/bash
# Round 5 (zb): the tree as it will be left -- full GPU suite + smoke + the default bench line
set -u
O=gpurun_out/r5zb; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
echo "c3: $(python3 tools/bench_line.py $O/c3.json)"
echo done

#!/bin/bash
# Round 6 (al): closing check on HEAD -- the whole GPU suite, smoke(), the default bench line and its rocprofv3 summary
set -u
O=gpurun_out/r6al; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 $O/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; cat $O/bench.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o trace -- python3 bench.py --no-cpu-baseline > $O/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; grep '^{' $O/prof.log || true
exit $rc

#!/bin/bash
# Round 4 closing run of the tree: full GPU suite, smoke, the default bench line (c3) with its
# rocprofv3 kernel trace, the other workloads' lines (ar354 at the applications' batch)
set -u
O=gpurun_out/r4y; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -10 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
tail -1 $O/c3.json | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4y_prof -o c3 -- python3 bench.py --no-cpu-baseline > $O/c3_prof.json 2> $O/c3_prof.err || { tail -5 $O/c3_prof.err; exit 1; }
for w in ar354 c5 c2 ar; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > $O/$w.json 2> $O/$w.err || { echo "$w failed"; tail -5 $O/$w.err; exit 1; }
  echo "$w: $(tail -1 $O/$w.json | cut -c1-160)"
done
echo done

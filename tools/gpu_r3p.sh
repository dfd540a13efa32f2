#!/bin/bash
# Round 3 session p: derivative logits by selects (dsel variant) vs the tree
# (LDS table); c3 at 2^17 with the graph replay; graphed bench workloads.
set -u
O=gpurun_out/r3p; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc=$rc"; return $rc; }
run tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_graphs.py tests/test_gpu_chain.py || exit $?
for r in 1 2; do
  NFK_LIBRARY=build_ab/dsel/libnfk.so run dsel_$r 300 python bench.py --no-cpu-baseline --parity-rows 4096 || exit $?
  run tree_$r 300 python bench.py --no-cpu-baseline --parity-rows 4096 || exit $?
done
run c3_2e17_graph 300 python bench.py --no-cpu-baseline --batch 131072 --steps 50 || exit $?
run c3_2e17_eager 300 python bench.py --no-cpu-baseline --batch 131072 --steps 50 --graph off || exit $?
for f in $O/dsel*.log $O/tree*.log $O/c3_*.log; do echo -n "$f "; grep -h '"value"' $f | python -c "
import sys,json
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity']['pass'], d['config'].get('hip_graph'))"; done

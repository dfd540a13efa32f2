#!/bin/bash
# Round 6 (v): graph replay staleness by the C++ watch; small-batch bench workloads replayed
set -u
O=gpurun_out/r6v; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_graphs.py -m gpu -v -rP --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error" $O/pytest.log | tail -5
[ $rc -ne 0 ] && exit $rc
for w in ar354 fe162 poly2048 rnvp2048 c1; do
  for gr in off auto; do
    timeout -k 10 240 python3 bench.py --workload $w --steps 40 --warmup 5 --no-cpu-baseline --graph $gr > $O/bench_${w}_$gr.json 2> $O/bench_${w}_$gr.err || { tail -5 $O/bench_${w}_$gr.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_${w}_$gr.json').read().strip().splitlines()[-1]); r=d['roofline'] or {}; print('$w graph=$gr', d['value'], d['ms_per_step'], 'ms', 'graph', d['config']['hip_graph'], 'frac', r.get('frac'), 'kernel', r.get('mean_ms'), 'parity', d['parity']['pass'])"
  done
done
echo done

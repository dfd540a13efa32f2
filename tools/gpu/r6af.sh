#!/bin/bash
# Round 6 (af): consecutive weight-stream RealNVP layers as one nfk_wide_rnvp_chain call
set -u
O=gpurun_out/r6af; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rnvp_polymer.py tests/test_gpu_graphs.py tests/test_gpu_parity.py -m gpu -v -rP --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error" $O/pytest.log | tail -5
[ $rc -ne 0 ] && exit $rc
for gr in off auto; do
  timeout -k 10 240 python3 bench.py --workload rnvp2048 --steps 40 --warmup 5 --no-cpu-baseline --graph $gr > $O/bench_$gr.json 2> $O/bench_$gr.err || { tail -5 $O/bench_$gr.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$gr.json').read().strip().splitlines()[-1]); r=d['roofline'] or {}; print('rnvp2048 graph=$gr', d['value'], d['ms_per_step'], 'ms', 'frac', r.get('frac'), 'kernel', r.get('kernel'), r.get('mean_ms'), 'parity', d['parity']['pass'])"
done
echo done

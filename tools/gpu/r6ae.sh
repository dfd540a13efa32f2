#!/bin/bash
# Round 6 (ae): rnvp2048 bench line with the chain call's roofline
set -u
O=gpurun_out/r6ae; mkdir -p $O
export TMPDIR=/tmp
for gr in off auto; do
  timeout -k 10 240 python3 bench.py --workload rnvp2048 --steps 40 --warmup 5 --no-cpu-baseline --graph $gr > $O/bench_$gr.json 2> $O/bench_$gr.err || { tail -5 $O/bench_$gr.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$gr.json').read().strip().splitlines()[-1]); r=d['roofline'] or {}; print('rnvp2048 graph=$gr', d['value'], d['ms_per_step'], 'ms', 'frac', r.get('frac'), r.get('kernel'), r.get('mean_ms'), r.get('per_launch'), 'parity', d['parity']['pass'])"
done
echo done

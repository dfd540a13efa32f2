#!/bin/bash
# Round 6 (ai): c3 at 2^20 rows, eager vs graph replay (A/B, interleaved)
set -u
O=gpurun_out/r6ai; mkdir -p $O
export TMPDIR=/tmp
run() {
    timeout -k 10 180 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --graph $2 > $O/$1.json 2> $O/$1.err || { tail -3 $O/$1.err; return 1; }
    python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', round(d['value']/1e6,2), 'M/s', d['ms_per_step'], 'ms', 'graph', d['config']['hip_graph'], 'kernel', d['roofline']['mean_ms'], 'parity', d['parity']['pass'])"
}
run off0 off && run on0 on && run off1 off && run on1 on && run off2 off && run on2 on
echo done

#!/bin/bash
# Round 6 (z4): closing bench lines (c3 with its CPU baseline, every other
# workload) and the c3 rocprofv3 kernel summary on this build
set -u
O=gpurun_out/r6z4; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { tail -5 $O/bench_c3.err; exit 1; }
tail -1 $O/bench_c3.json
for w in c2 c5 c1 ar ar354 fe162 poly2048 rnvp2048; do
    timeout -k 10 240 python3 bench.py --workload $w --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || { tail -5 $O/bench_$w.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_$w.json').read().strip().splitlines()[-1]); print('$w', d['value'], d['unit'], d['ms_per_step'], 'ms', 'frac', d['roofline']['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_c3.log 2>&1 || { tail -5 $O/prof_c3.log; exit 1; }
head -3 $O/prof_c3/run_kernel_stats.csv
echo done

#!/bin/bash
# Round 5 (e): kernel trace of the Polymer forward (poly2048 bench) and the Fe line, then the
# packed-FP32 nop-patch VJP experiment (tools/gpu/r5c.sh)
set -u
O=gpurun_out/r5e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5e_prof -o poly -- python3 bench.py --workload poly2048 --steps 5 --warmup 1 --no-cpu-baseline > $O/poly.json 2> $O/poly.err || { tail -5 $O/poly.err; exit 1; }
tail -1 $O/poly.json | cut -c1-400
find gpurun_out/r5e_prof -name "*kernel_stats.csv" -exec head -8 {} \;
bash tools/gpu/r5c.sh

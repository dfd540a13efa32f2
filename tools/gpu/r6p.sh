#!/bin/bash
# Round 6 (p): rnvp2048 per-kernel times on this build
set -u
O=gpurun_out/r6p; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --workload rnvp2048 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
cut -d, -f1-4 $O/prof/run_kernel_stats.csv | head -12
echo done

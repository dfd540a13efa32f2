#!/bin/bash
# Round 6 (q): attribute the Gaussian NSF_AR layer's HBM traffic (bench ar):
# FETCH/WRITE at three batch sizes (slope = bytes per row, intercept = per-launch),
# TCC hit/miss at 2^20
set -u
export TMPDIR=/tmp
for b in 65536 262144 1048576; do
  bash tools/pmc_traffic_passes.sh r6q/b$b k_fused_ar --workload ar --batch $b || exit 1
done
timeout -k 10 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --kernel-include-regex k_fused_ar --output-format csv \
    -d gpurun_out/r6q/tcc -o pmc -- python3 bench.py --workload ar --steps 2 --warmup 1 --no-cpu-baseline --no-timer --parity-rows 0 > gpurun_out/r6q/tcc.log 2>&1 || { tail -5 gpurun_out/r6q/tcc.log; exit 1; }
for d in gpurun_out/r6q/b* gpurun_out/r6q; do python3 tools/pmc_summary.py $d --kernel k_fused_ar 2>&1 | grep -E "==|FETCH|WRITE|TCC_|hbm" ; done
echo done

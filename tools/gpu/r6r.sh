#!/bin/bash
# Round 6 (r): attribute c5's HBM reads (bench c5): FETCH/WRITE at three batch
# sizes (slope = bytes per row, intercept = per launch), TCC hit/miss at 2^20
set -u
export TMPDIR=/tmp
for b in 65536 262144 1048576; do
  bash tools/pmc_traffic_passes.sh r6r/b$b k_fused --workload c5 --batch $b || exit 1
done
timeout -k 10 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --kernel-include-regex k_fused --output-format csv \
    -d gpurun_out/r6r/tcc -o pmc -- python3 bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline --no-timer --parity-rows 0 > gpurun_out/r6r/tcc.log 2>&1 || { tail -5 gpurun_out/r6r/tcc.log; exit 1; }
for d in gpurun_out/r6r/b*; do echo $d; python3 tools/pmc_summary.py $d --kernel k_fused 2>&1 | grep -E "==|hbm" ; done
echo done

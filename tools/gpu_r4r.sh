#!/bin/bash
# Round 4: ar354 bench (fused vs per-column, several batches) and PMC passes of the HEAD build
# (c3 chain, ar354 and ar fused NSF_AR) for the roofline inputs
set -u
O=gpurun_out/r4r; mkdir -p $O
for b in 4096 65536 262144; do
  timeout -k 10 300 python bench.py --workload ar354 --batch $b --steps 5 --warmup 2 --no-cpu-baseline --parity-rows 256 > $O/ar354_fused_$b.json 2> $O/ar354_fused_$b.err || { echo "fused $b failed"; tail -5 $O/ar354_fused_$b.err; exit 1; }
  echo "fused $b: $(tail -1 $O/ar354_fused_$b.json | cut -c1-150)"
done
for b in 4096 65536; do
  timeout -k 10 300 python bench.py --workload ar354 --batch $b --steps 3 --warmup 1 --unfused --no-cpu-baseline --parity-rows 256 > $O/ar354_unfused_$b.json 2> $O/ar354_unfused_$b.err || { echo "unfused $b failed"; tail -5 $O/ar354_unfused_$b.err; exit 1; }
  echo "unfused $b: $(tail -1 $O/ar354_unfused_$b.json | cut -c1-150)"
done
bash tools/pmc_passes.sh r4r_c3 "k_nsf_chain2" --workload c3 || exit $?
bash tools/pmc_passes.sh r4r_ar354 "k_fused_ar" --workload ar354 || exit $?
bash tools/pmc_passes.sh r4r_ar "k_fused_ar" --workload ar || exit $?
for t in c3 ar354 ar; do python tools/pmc_summary.py gpurun_out/r4r_$t --json gpurun_out/r4r_$t/summary.json > gpurun_out/r4r_$t/summary.txt; done
echo done

#!/bin/bash
# Round 4: uniform-address (saddr) LDS-DMA in every fused kernel's staging + the NSF_AR column
# split: full GPU suite, then c3/c5/c2/ar/ar354 benches (ar354 fused vs per-column at the
# applications' batch and larger), PMC of ar354 at small batches, the c3 train-step kernel trace
set -u
O=gpurun_out/r4t; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_nsfar_fused.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest0.log 2>&1 || { tail -30 $O/pytest0.log; exit 1; }
tail -2 $O/pytest0.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for w in c3 c5 c2 ar; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > $O/b_$w.json 2> $O/b_$w.err || { echo "bench $w failed"; tail -5 $O/b_$w.err; exit 1; }
  echo "$w: $(tail -1 $O/b_$w.json | cut -c1-140)"
done
for b in 40 4096 65536; do
  timeout -k 10 300 python bench.py --workload ar354 --batch $b --steps 20 --warmup 3 --no-cpu-baseline --parity-rows 64 > $O/f_$b.json 2> $O/f_$b.err || { echo "fused $b failed"; tail -5 $O/f_$b.err; exit 1; }
  echo "ar354 fused $b: $(tail -1 $O/f_$b.json | cut -c1-140)"
done
for b in 40 4096; do
  timeout -k 10 300 python bench.py --workload ar354 --batch $b --steps 5 --warmup 2 --unfused --no-cpu-baseline --parity-rows 64 > $O/u_$b.json 2> $O/u_$b.err || { echo "unfused $b failed"; tail -5 $O/u_$b.err; exit 1; }
  echo "ar354 unfused $b: $(tail -1 $O/u_$b.json | cut -c1-140)"
done
for b in 40 4096; do
  bash tools/pmc_passes.sh r4t_ar354_$b "k_fused_ar" --workload ar354 --batch $b || exit $?
  python tools/pmc_summary.py gpurun_out/r4t_ar354_$b --json gpurun_out/r4t_ar354_$b/summary.json > gpurun_out/r4t_ar354_$b/summary.txt
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4t_train -o train -- python3 tools/bench_train.py --batch 1048576 --steps 3 --warmup 1 --no-torch > $O/train.log 2>&1 || { tail -5 $O/train.log; exit 1; }
tail -2 $O/train.log
echo done

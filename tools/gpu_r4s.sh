#!/bin/bash
# Round 4: the fused NSF_AR forward's column split (small batches) -- bitwise vs unsplit, and
# ar354 speed fused vs per-column at the applications' batch (40) and 4096 / 65536
set -u
O=gpurun_out/r4s; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_nsfar_fused.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for b in 40 4096 65536; do
  for g in on off; do
    timeout -k 10 300 python bench.py --workload ar354 --batch $b --steps 20 --warmup 3 --graph $g --no-cpu-baseline --parity-rows 64 > $O/f_${b}_$g.json 2> $O/f_${b}_$g.err || { echo "fused $b failed"; tail -5 $O/f_${b}_$g.err; exit 1; }
    echo "fused $b graph $g: $(tail -1 $O/f_${b}_$g.json | cut -c1-120)"
  done
done
for b in 40 4096; do
  timeout -k 10 300 python bench.py --workload ar354 --batch $b --steps 5 --warmup 2 --graph on --unfused --no-cpu-baseline --parity-rows 64 > $O/u_$b.json 2> $O/u_$b.err || { echo "unfused $b failed"; tail -5 $O/u_$b.err; exit 1; }
  echo "unfused $b: $(tail -1 $O/u_$b.json | cut -c1-120)"
done
for b in 40 4096; do
  bash tools/pmc_passes.sh r4s_ar354_$b "k_fused_ar" --workload ar354 --batch $b || exit $?
  python tools/pmc_summary.py gpurun_out/r4s_ar354_$b --json gpurun_out/r4s_ar354_$b/summary.json > gpurun_out/r4s_ar354_$b/summary.txt
done
echo done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4s_train -o train -- python3 tools/bench_train.py --batch 1048576 --steps 3 --warmup 1 --no-torch > gpurun_out/r4s_train.log 2>&1 || { tail -5 gpurun_out/r4s_train.log; exit 1; }
tail -2 gpurun_out/r4s_train.log
echo done2

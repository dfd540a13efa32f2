#!/bin/bash
# Round 4: [lower | 1] gather for the first Linear's weight+bias gradient (train step), the
# NSF_AR host fast path (ar354 at the applications' batch): tests, train bench, ar354 benches
set -u
O=gpurun_out/r4u; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_chain.py tests/test_gpu_vjp.py tests/test_gpu_grad.py tests/test_gpu_nsfar_fused.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python tools/bench_train.py --batch 1048576 --steps 5 --warmup 2 --no-torch > $O/train.json 2> $O/train.err || { tail -5 $O/train.err; exit 1; }
tail -3 $O/train.json
for b in 40 50 4096; do
  timeout -k 10 300 python bench.py --workload ar354 --batch $b --steps 20 --warmup 3 --no-cpu-baseline --parity-rows 40 > $O/f_$b.json 2> $O/f_$b.err || { echo "fused $b failed"; tail -5 $O/f_$b.err; exit 1; }
  echo "ar354 fused $b: $(tail -1 $O/f_$b.json | cut -c1-140)"
done
timeout -k 10 300 python bench.py --workload ar354 --batch 50 --steps 5 --warmup 2 --unfused --no-cpu-baseline --parity-rows 40 > $O/u_50.json 2> $O/u_50.err || { echo "unfused failed"; tail -5 $O/u_50.err; exit 1; }
echo "ar354 unfused 50: $(tail -1 $O/u_50.json | cut -c1-140)"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4u_train -o train -- python3 tools/bench_train.py --batch 1048576 --steps 3 --warmup 1 --no-torch > $O/train_prof.log 2>&1 || { tail -5 $O/train_prof.log; exit 1; }
echo done

#!/bin/bash
# Round-end rehearsal: GPU tests, smoke, c3/c2/c5 bench lines, rocprofv3 stats of
# the c3 bench, c3/c2 train steps.  Each step time-limited; stops at the first failure.
set -u
O=gpurun_out/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { tail -5 $O/bench_c3.err; exit 1; }
echo "c3: $(python3 tools/bench_line.py $O/bench_c3.json)"
for w in c2 c5; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || { tail -5 $O/bench_$w.err; exit 1; }
  echo "$w: $(python3 tools/bench_line.py $O/bench_$w.json)"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o trace -- python3 bench.py --no-cpu-baseline --parity-rows 0 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
grep '^{' $O/prof.log > $O/prof_bench.json || true
for w in c3 c2; do
  timeout -k 10 300 python tools/bench_train.py --workload $w --batch 1048576 --steps 5 --warmup 2 --no-torch > $O/train_$w.json 2> $O/train_$w.err || { tail -5 $O/train_$w.err; exit 1; }
  echo "train $w: $(tail -1 $O/train_$w.json | cut -c1-250)"
done

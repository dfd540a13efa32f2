#!/bin/bash
# Round 6 (d): training re-timed on this build (c3 at 2^20, ar354 at 40 rows)
# with a rocprof summary of the c3 step; NSF_AR sampling at the applications'
# batches; the rnvp2048 bench line
set -u
O=gpurun_out/r6d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_train.py --workload c3 --batch 1048576 --steps 10 --no-torch > $O/train_c3.json 2> $O/train_c3.err || { tail -5 $O/train_c3.err; exit 1; }
cat $O/train_c3.json
timeout -k 10 300 python -u tools/bench_train.py --workload ar354 --batch 40 --steps 20 > $O/train_ar354.json 2> $O/train_ar354.err || { tail -5 $O/train_ar354.err; exit 1; }
cat $O/train_ar354.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_train_c3 -o run -- python3 tools/bench_train.py --workload c3 --batch 1048576 --steps 5 --warmup 1 --no-torch > $O/prof_train_c3.log 2>&1 || { tail -5 $O/prof_train_c3.log; exit 1; }
timeout -k 10 400 python -u tools/time_ar_sample.py > $O/ar_sample.json 2> $O/ar_sample.err || { tail -5 $O/ar_sample.err; exit 1; }
cat $O/ar_sample.json
timeout -k 10 300 python bench.py --workload rnvp2048 --no-cpu-baseline > $O/rnvp2048.json 2> $O/rnvp2048.err || { tail -5 $O/rnvp2048.err; exit 1; }
cat $O/rnvp2048.json
echo done

#!/bin/bash
# c2 training step A/B: FCNN forward/backward kernels vs library GEMMs, then a kernel trace
set -u
O=gpurun_out/trainc2; mkdir -p $O
for v in fwd dh lib; do
  f=""; [ $v = dh ] && f="--no-fcnn-fwd"; [ $v = lib ] && f="--no-fcnn-fwd --no-fcnn-dh"
  timeout -k 10 300 python tools/bench_train.py --workload c2 --batch 1048576 --steps 5 --warmup 2 --no-torch $f > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  echo "$v: $(tail -1 $O/$v.json | cut -c150-320)"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o trace -- python3 tools/bench_train.py --workload c2 --batch 1048576 --steps 2 --warmup 1 --no-torch > $O/prof.log 2>&1 || exit 1

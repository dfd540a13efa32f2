#!/bin/bash
# grad tests, then the c3 train step with and without nfk_fcnn_dh (alternating),
# then a kernel-stats profile of the dh variant
set -u
O=gpurun_out/traindh; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fcnn_dh.py tests/test_gpu_vjp.py tests/test_gpu_grad.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for v in dh lib; do
    f=""; [ $v = lib ] && f="--no-fcnn-dh"
    timeout -k 10 300 python tools/bench_train.py --batch 1048576 --steps 5 --warmup 2 --no-torch $f > $O/$v-$r.json 2> $O/$v-$r.err || { echo "train $v failed"; tail -5 $O/$v-$r.err; exit 1; }
    echo "$v $r: $(tail -1 $O/$v-$r.json | cut -c100-260)"
  done
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o trace -- python3 tools/bench_train.py --batch 1048576 --steps 2 --warmup 1 --no-torch > $O/prof.log 2>&1 || exit 1

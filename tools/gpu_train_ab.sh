#!/bin/bash
# c3 train step (tools/bench_train.py, B = 2^20) for the working tree and build_ab/$1..., alternating
set -u
O=gpurun_out/trainab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_vjp.py tests/test_gpu_grad.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for v in cur "$@"; do
    if [ $v = cur ]; then unset NFK_LIBRARY; else export NFK_LIBRARY=build_ab/$v/libnfk.so; fi
    timeout -k 10 300 python tools/bench_train.py --batch 1048576 --steps 5 --warmup 2 --no-torch > $O/$v-$r.json 2> $O/$v-$r.err || { echo "train $v failed"; tail -5 $O/$v-$r.err; exit 1; }
    echo "$v $r: $(tail -1 $O/$v-$r.json | cut -c1-200)"
  done
done

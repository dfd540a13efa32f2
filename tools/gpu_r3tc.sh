#!/bin/bash
# Training forward as one saved-input chain launch: GPU tests (new + the grad suite), then the
# c3 train step at 2^20 with and without the chain, alternated on one box.
set -u
O=gpurun_out/r3tc; mkdir -p $O
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; tail -2 $O/$n.log | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
run pytest_tc 600 python -u -m pytest tests/test_gpu_train_chain.py tests/test_gpu_grad.py tests/test_gpu_chain.py -x -v --timeout 200 --timeout-method thread
for i in 1 2; do
  run train_chain_$i 300 python tools/bench_train.py --batch 1048576 --steps 5 --warmup 2 --no-torch
  run train_layer_$i 300 python tools/bench_train.py --batch 1048576 --steps 5 --warmup 2 --no-torch --no-train-chain
done

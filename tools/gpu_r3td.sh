#!/bin/bash
# Fused VJP with global loads only while no LDS-DMA is in flight (determinism fix) + the training-forward chain:
# determinism diagnostic, the VJP / train-chain / grad / chain GPU tests, then the c3 train
# step at 2^20 with and without the training chain.
set -u
O=gpurun_out/r3td; mkdir -p $O
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; tail -3 $O/$n.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
export PYTHONPATH=.
run vjp_det 200 python tools/dbg_vjp_det.py
run pytest_tc 900 python -u -m pytest tests/test_gpu_vjp.py tests/test_gpu_train_chain.py tests/test_gpu_grad.py tests/test_gpu_chain.py -x -v --timeout 200 --timeout-method thread
run train_chain 300 python tools/bench_train.py --batch 1048576 --steps 5 --warmup 2 --no-torch
run train_layer 300 python tools/bench_train.py --batch 1048576 --steps 5 --warmup 2 --no-torch --no-train-chain

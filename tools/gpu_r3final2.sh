#!/bin/bash
# Round 3 closing run 2: the fused VJP gated to <= config.FUSED_VJP_MAX_ROWS rows (larger
# batches on the reproducible unfused backward): training GPU tests, smoke, the c3 train step.
set -u
O=gpurun_out/r3final2; mkdir -p $O
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; tail -3 $O/$n.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
export PYTHONPATH=.
run pytest_train 600 python -u -m pytest tests/test_gpu_vjp.py tests/test_gpu_grad.py tests/test_gpu_train_chain.py -q -rf --timeout 300 --timeout-method thread
run smoke 150 python -c "import __graft_entry__ as g; g.smoke()"
run train_chain 300 python tools/bench_train.py --batch 1048576 --steps 5 --warmup 2 --no-torch

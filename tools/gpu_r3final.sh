#!/bin/bash
# Round 3 closing run of the committed tree: VJP determinism (fused / unfused), the GPU suite
# and smoke, the c3 bench line + rocprofv3 kernel stats, and the c3 train step with and
# without the training-forward chain.
set -u
O=gpurun_out/r3final; mkdir -p $O
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; tail -3 $O/$n.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
export PYTHONPATH=.
DBG_ROWS=262144,1048576 NFK_LIBRARY=$PWD/build_ab/tailnop/libnfk.so run vjp_tailnop 240 python tools/dbg_vjp_det.py
run vjp_unfused 240 python tools/dbg_vjp_unfused.py
run pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
run smoke 150 python -c "import __graft_entry__ as g; g.smoke()"
run bench_c3 300 python bench.py
export TMPDIR=/tmp
run prof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o trace -- python3 bench.py --no-cpu-baseline
run train_chain 300 python tools/bench_train.py --batch 1048576 --steps 5 --warmup 2 --no-torch
run train_layer 300 python tools/bench_train.py --batch 1048576 --steps 5 --warmup 2 --no-torch --no-train-chain

#!/bin/bash
# Round 3 session s (validation of the tuned kernels), part 1: the GPU suite and smoke.
set -u
O=gpurun_out/r3s; mkdir -p $O
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; tail -2 $O/$n.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
run pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
run smoke 150 python -c "import __graft_entry__ as g; g.smoke()"

#!/bin/bash
# A/B session: GPU parity tests, then bench.py under each environment setting given.
# usage: bash tools/gpu_ab.sh TAG "ENV=.. ENV2=.." "ENV=.." ...   (bench args via BENCH_ARGS)
set -u
TAG=${1:-ab}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread \
      > "$OUT/pytest_gpu.log" 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -4 "$OUT/pytest_gpu.log"
  [ $rc -ne 0 ] && exit $rc
fi
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err"; rc=$?
  echo "[$envs] rc=$rc"; python -c "import json;d=json.load(open('$OUT/bench_$i.json'));print(d['value']/1e6,'M/s',d['roofline']['mean_ms'],'ms',d['kernels'])" 2>/dev/null || tail -3 "$OUT/bench_$i.err"
  [ $rc -ne 0 ] && exit $rc
done
exit 0

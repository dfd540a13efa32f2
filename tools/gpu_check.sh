#!/bin/bash
# One GPU-box session: parity tests -> smoke -> bench -> rocprofv3 kernel trace.
# Each GPU step has its own time limit; a fault/abort/timeout ends the script.
# usage: bash tools/gpu_check.sh TAG [bench args...]
set -u
TAG=${1:-run}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
fatal() { case $1 in 0|1) return 1;; *) echo "FATAL rc=$1 in $2"; exit $1;; esac; }

timeout -k 10 900 python -m pytest tests -m gpu -q -rfs > "$OUT/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"; fatal $rc smoke
timeout -k 10 300 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"; fatal $rc bench
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o trace \
    -- python3 "$ROOT/bench.py" --no-cpu-baseline "$@" \
    > "$OUT/prof.log" 2>&1; rc=$?
grep '^{' "$OUT/prof.log" > "$OUT/prof_bench.json" || true   # the bench line of the profiled run
echo "rocprof rc=$rc"; tail -3 "$OUT/prof.log"; fatal $rc rocprof
find "$OUT/prof" -name "*stats*" | head
if [ -n "${EXTRA_BENCH:-}" ]; then
  timeout -k 10 300 python bench.py $EXTRA_BENCH > "$OUT/bench_extra.json" 2> "$OUT/bench_extra.err"; rc=$?
  echo "bench_extra rc=$rc"; cat "$OUT/bench_extra.json"; fatal $rc bench_extra
fi
exit 0

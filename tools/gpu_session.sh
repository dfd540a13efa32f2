#!/bin/bash
# One GPU-box session: GPU tests -> smoke -> bench lines (each step under its
# own time limit; a fault/abort/timeout ends the script) -> optional rocprof.
# usage: bash tools/gpu_session.sh TAG [--no-tests] [--prof] [--pmc-insts] -- [extra bench arg sets separated by ';']
set -u
TAG=${1:-run}; shift || true
TESTS=1; PROF=0; PMCI=0
while [ $# -gt 0 ] && [ "$1" != "--" ]; do
  case $1 in --no-tests) TESTS=0;; --prof) PROF=1;; --pmc-insts) PMCI=1;; esac; shift
done
[ "${1:-}" = "--" ] && shift
EXTRA="${*:-}"
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
fatal() { case $1 in 0|1) return 1;; *) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
if [ $TESTS = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
      > "$OUT/pytest_gpu.log" 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -8 "$OUT/pytest_gpu.log"; [ $rc = 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; [ $rc = 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"; [ $rc = 0 ] || exit $rc
i=0
IFS=';' read -ra SETS <<< "$EXTRA"
for a in "${SETS[@]}"; do
  [ -z "${a// }" ] && continue
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu-baseline $a > "$OUT/bench_x$i.json" 2> "$OUT/bench_x$i.err"; rc=$?
  echo "bench_x$i ($a) rc=$rc"; cat "$OUT/bench_x$i.json"; [ $rc = 0 ] || { tail -3 "$OUT/bench_x$i.err"; exit $rc; }
done
export TMPDIR=/tmp
if [ $PROF = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o trace \
      -- python3 "$ROOT/bench.py" --no-cpu-baseline --parity-rows 0 > "$OUT/prof.log" 2>&1; rc=$?
  grep '^{' "$OUT/prof.log" > "$OUT/prof_bench.json" || true
  echo "rocprof rc=$rc"; [ $rc = 0 ] || { tail -3 "$OUT/prof.log"; exit $rc; }
fi
if [ $PMCI = 1 ]; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS \
      --kernel-include-regex k_fused --output-format csv -d "$OUT/pmci" -o pmc \
      -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-timer --parity-rows 0 \
      > "$OUT/pmci.log" 2>&1; rc=$?
  echo "pmc insts rc=$rc"; [ $rc = 0 ] || { tail -3 "$OUT/pmci.log"; exit $rc; }
fi
exit 0

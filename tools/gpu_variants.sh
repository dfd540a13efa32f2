#!/bin/bash
# Bench several library variants back to back on one box (no tests).
# usage: bash tools/gpu_variants.sh TAG lib1 [lib2 ...]   (libs relative to normalizingflow_amd/)
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
for lib in "$@"; do
  NFK_LIBRARY=$ROOT/normalizingflow_amd/$lib timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} \
      > "$OUT/bench_$lib.json" 2> "$OUT/bench_$lib.err"; rc=$?
  echo "$lib rc=$rc"; python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['roofline'])" "$OUT/bench_$lib.json"
  case $rc in 0) ;; *) echo "FATAL $rc"; tail -5 "$OUT/bench_$lib.err"; exit $rc;; esac
done

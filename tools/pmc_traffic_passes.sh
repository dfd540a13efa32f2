#!/bin/bash
# HBM traffic only: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes
# over a short bench run, restricted to the kernels matching REGEX.
# usage: bash tools/pmc_traffic_passes.sh TAG REGEX [bench args...]
set -u
TAG=$1; REGEX=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
i=3
for p in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $p --kernel-include-regex "$REGEX" --output-format csv \
      -d "$OUT/pmc$i" -o pmc -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-timer --parity-rows 0 "$@" \
      > "$OUT/pmc$i.log" 2>&1; rc=$?
  echo "pass $p rc=$rc"
  case $rc in 0) ;; *) tail -5 "$OUT/pmc$i.log"; exit $rc;; esac
done

#!/bin/bash
# A/B of library variants on one box: bench.py alternated over the variants
# ROUNDS times (c3 by default), then a one-line summary per variant.
# usage: bash tools/gpu_abv.sh TAG ROUNDS "name=path-to-libnfk.so" ... (bench args via BENCH_ARGS)
set -u
TAG=$1; ROUNDS=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    n=${v%%=*}; lib=${v#*=}
    NFK_LIBRARY=$ROOT/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --parity-rows 2048 ${BENCH_ARGS:-} \
        > "$OUT/${n}_$r.json" 2> "$OUT/${n}_$r.err"; rc=$?
    [ $rc -ne 0 ] && { echo "$n round $r rc=$rc"; tail -5 "$OUT/${n}_$r.err"; exit $rc; }
  done
done
python - "$OUT" "$@" <<'PY'
import json, sys, glob, statistics
out = sys.argv[1]
for v in sys.argv[2:]:
    n = v.split("=")[0]
    d = [json.load(open(f)) for f in sorted(glob.glob("%s/%s_*.json" % (out, n)))]
    k = [x["roofline"]["mean_ms"] for x in d]
    print("%-12s value %7.2f M/s (runs %s)  kernel %.4f ms (min %.4f)  parity %s" % (
        n, statistics.median(x["value"] for x in d) / 1e6, " ".join("%.1f" % (x["value"] / 1e6) for x in d),
        statistics.median(k), min(k), all(x["parity"]["pass"] for x in d)))
PY

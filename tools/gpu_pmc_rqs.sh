#!/bin/bash
# PMC passes (HBM bytes, SQ activity) of nfk_rqs_coupling under tools/bench_rqs.py
set -u
TAG=${1:-pmcrqs}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
PASSES=(
 "FETCH_SIZE"
 "WRITE_SIZE"
 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
 "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum GRBM_GUI_ACTIVE GRBM_COUNT"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $p --kernel-include-regex "k_rqs_(coupling|stream)" --output-format csv \
      -d "$OUT/pmc$i" -o pmc -- python3 "$ROOT/tools/bench_rqs.py" --iters 3 > "$OUT/pmc$i.log" 2>&1; rc=$?
  echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/pmc$i.log"; exit $rc; }
done
python3 tools/pmc_summary.py "$OUT" --kernel "k_rqs_" > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"

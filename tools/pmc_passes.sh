#!/bin/bash
# rocprofv3 PMC passes (one counter group per pass, never combined with tracing)
# over a short bench run; restricted to the kernels matching REGEX.
# usage: bash tools/pmc_passes.sh TAG REGEX [bench args...]
set -u
TAG=$1; REGEX=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
PASSES=(
 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES"
 "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VMEM"
 "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum GRBM_GUI_ACTIVE GRBM_COUNT"
 "FETCH_SIZE"
 "WRITE_SIZE"
 "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"
 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $p --kernel-include-regex "$REGEX" --output-format csv \
      -d "$OUT/pmc$i" -o pmc -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-timer --parity-rows 0 "$@" \
      > "$OUT/pmc$i.log" 2>&1; rc=$?
  echo "pass $i rc=$rc ($p)"
  case $rc in 0) ;; *) tail -5 "$OUT/pmc$i.log"; exit $rc;; esac
done

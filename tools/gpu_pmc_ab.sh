#!/bin/bash
# SQ/LDS PMC passes (tools/pmc_passes.sh groups 1, 2, 7) of k_fused_nsf under
# two environment settings; one rocprofv3 run per pass.
# usage: bash tools/gpu_pmc_ab.sh TAG "ENV_A" "ENV_B"
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
export TMPDIR=/tmp
PASSES=(
 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES"
 "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VMEM"
 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU"
)
v=0
for envs in "$@"; do
  v=$((v+1)); OUT=$ROOT/gpurun_out/$TAG/v$v; mkdir -p "$OUT"; echo "$envs" > "$OUT/env.txt"
  i=0
  for p in "${PASSES[@]}"; do
    i=$((i+1))
    env $envs timeout -s KILL 120 rocprofv3 --pmc $p --kernel-include-regex k_fused_nsf --output-format csv \
        -d "$OUT/pmc$i" -o pmc -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-timer \
        > "$OUT/pmc$i.log" 2>&1; rc=$?
    echo "v$v pass $i rc=$rc"
    [ $rc -eq 0 ] || { tail -5 "$OUT/pmc$i.log"; exit $rc; }
  done
  python3 tools/pmc_summary.py "$OUT" --kernel k_fused_nsf > "$OUT/summary.txt" 2>&1
  cat "$OUT/summary.txt"
done

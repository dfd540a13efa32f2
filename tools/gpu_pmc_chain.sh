#!/bin/bash
# rocprofv3 PMC passes (HBM FETCH_SIZE / WRITE_SIZE; PMC_FULL=1 adds the SQ
# utilisation groups) over a short default bench run, fused NSF kernels only.
# usage: bash tools/gpu_pmc_chain.sh [TAG]
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmcchain}; mkdir -p $OUT
PASSES=("FETCH_SIZE" "WRITE_SIZE")
[ -n "${PMC_FULL:-}" ] && PASSES+=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VMEM")
for p in "${PASSES[@]}"; do
  n=$(echo $p | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $p --kernel-include-regex "k_fused_nsf" --output-format csv -d $OUT/pmc_$n -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-timer > $OUT/pmc_$n.log 2>&1 || { echo "fail $n"; tail -5 $OUT/pmc_$n.log; exit 1; }
  echo "pass $n ok"
done
python3 tools/pmc_summary.py $OUT --kernel k_fused_nsf > $OUT/summary.txt 2>&1; cat $OUT/summary.txt | head -60

#!/bin/bash
# Round 5 (w): PMC evidence of the shipped build -- the c3 chain's seven passes, and for c2, c5,
# the Gaussian NSF_AR and ar354 the instruction-count pass + the HBM traffic passes
set -u
O=gpurun_out/r5w; mkdir -p $O
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/pmc_passes.sh r5w/pmc_c3 k_nsf_chain2 || exit 1
insts() {  # tag regex bench-args...
  local tag=$1 re=$2; shift 2
  mkdir -p $O/$tag
  timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VMEM \
      --kernel-include-regex "$re" --output-format csv -d "$ROOT/$O/$tag/pmc2" -o pmc -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-timer --parity-rows 0 "$@" \
      > "$ROOT/$O/$tag/pmc2.log" 2>&1; rc=$?
  echo "$tag insts rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$ROOT/$O/$tag/pmc2.log"; exit $rc; }
  timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES \
      --kernel-include-regex "$re" --output-format csv -d "$ROOT/$O/$tag/pmc1" -o pmc -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-timer --parity-rows 0 "$@" \
      > "$ROOT/$O/$tag/pmc1.log" 2>&1; rc=$?
  echo "$tag waves rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$ROOT/$O/$tag/pmc1.log"; exit $rc; }
  bash tools/pmc_traffic_passes.sh r5w/$tag "$re" "$@" || exit 1
}
insts pmc_c2 k_rnvp_chain --workload c2
insts pmc_c5 k_fused_nsf_wide --workload c5
insts pmc_ar k_fused_ar --workload ar
insts pmc_ar354 k_fused_ar --workload ar354
echo done

#!/bin/bash
# s1w4 timeline + first two PMC passes for the default and s1w4 builds
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; mkdir -p gpurun_out/s1b
NFK_LIBRARY=$ROOT/normalizingflow_amd/libnfk_s1w4_trace.so timeout -k 10 200 python tools/trace_wide.py --c3 --slots1 > gpurun_out/s1b/trace.txt 2>&1; rc=$?
cat gpurun_out/s1b/trace.txt; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
for lib in libnfk libnfk_s1w4; do
for i in 1 2; do
  P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES"
  P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VMEM"
  [ $i = 1 ] && P=$P1 || P=$P2
  NFK_LIBRARY=$ROOT/normalizingflow_amd/$lib.so timeout -k 10 240 rocprofv3 --pmc $P --kernel-include-regex k_fused_nsf --output-format csv \
      -d gpurun_out/s1b/${lib}_pmc$i -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-timer \
      > gpurun_out/s1b/${lib}_pmc$i.log 2>&1; rc=$?
  echo "$lib pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done; done

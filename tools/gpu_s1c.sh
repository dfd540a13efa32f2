#!/bin/bash
# parity (default + s1w4 builds), bench both, VALU/MFMA instruction counts of s1w4
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; mkdir -p gpurun_out/s1c
for V in libnfk libnfk_s1w4; do
NFK_LIBRARY=$ROOT/normalizingflow_amd/$V.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
   -k "c3 or golden or dim3 or large_n_up or ragged" > gpurun_out/s1c/pytest_$V.log 2>&1; rc=$?
echo "$V parity rc=$rc"; tail -2 gpurun_out/s1c/pytest_$V.log; [ $rc -eq 0 ] || exit $rc
done
bash tools/gpu_variants.sh s1c libnfk.so libnfk_s1w4.so || exit $?
export TMPDIR=/tmp
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VMEM"
NFK_LIBRARY=$ROOT/normalizingflow_amd/libnfk_s1w4.so timeout -k 10 240 rocprofv3 --pmc $P2 --kernel-include-regex k_fused_nsf --output-format csv \
      -d gpurun_out/s1c/pmc2 -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-timer > gpurun_out/s1c/pmc2.log 2>&1; rc=$?
echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py gpurun_out/s1c 2>&1 | head -14

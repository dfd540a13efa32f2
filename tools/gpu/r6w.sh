#!/bin/bash
# Round 6 (w): counters of the fused NSF_AR inverse at the applications' 500-row
# sampling batch (Fe dim 162 and Einstein dim 96; tools/time_ar_sample.py)
set -u
O=gpurun_out/r6w; mkdir -p $O
export TMPDIR=/tmp
i=0
for p in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum GRBM_GUI_ACTIVE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $p --kernel-include-regex "k_fused_ar<11, 1, 32, (6|11), true" --output-format csv \
      -d $O/pmc$i -o pmc -- python3 tools/time_ar_sample.py > $O/pmc$i.log 2>&1 || { tail -5 $O/pmc$i.log; exit 1; }
  echo "pass $i ok"
done
python3 tools/pmc_summary.py $O 2>&1 | grep -vE "^\s*$" | head -60
echo done

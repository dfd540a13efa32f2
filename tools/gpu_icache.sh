#!/bin/bash
# instruction-cache PMC of the c3 chain kernel (two passes, no tracing)
set -u
export TMPDIR=/tmp
O=gpurun_out/icache; mkdir -p $O
i=0
for p in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ" "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $p --kernel-include-regex "k_fused_nsf" --output-format csv -d $O/pmc$i -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-timer --parity-rows 0 "$@" > $O/pmc$i.log 2>&1; rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $O/pmc$i.log; exit $rc; }
done
python3 tools/pmc_summary.py $O --kernel k_fused_nsf

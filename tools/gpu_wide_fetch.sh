#!/bin/bash
# FETCH_SIZE / TCC pass of the c5 wide kernel for the working-tree build and
# each build_ab/NAME given (one rocprofv3 --pmc pass per run, no tracing)
set -u
export TMPDIR=/tmp
O=gpurun_out/widefetch; mkdir -p $O
for v in cur "$@"; do
  if [ $v = cur ]; then unset NFK_LIBRARY; else export NFK_LIBRARY=build_ab/$v/libnfk.so; fi
  for p in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum"; do
    tag=$(echo $p | cut -d' ' -f1)
    timeout -k 10 240 rocprofv3 --pmc $p --kernel-include-regex "k_fused_nsf_wide" --output-format csv \
        -d $O/$v/pmc-$tag -o pmc -- python3 bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline --no-timer --parity-rows 0 \
        > $O/$v-$tag.log 2>&1 || { echo "pmc $v $tag failed"; tail -5 $O/$v-$tag.log; exit 1; }
  done
  python3 tools/pmc_summary.py $O/$v --kernel k_fused_nsf_wide > $O/$v.txt 2>&1 || true
  echo "== $v"; cat $O/$v.txt | head -20
done

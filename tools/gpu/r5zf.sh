#!/bin/bash
# Round 5 (zf): c5 wide kernel, the x tile gathers (the rows' last read) non-temporal
# (NFK_WIDE_X_NT=1, build_ab/wnt) vs HEAD: time A/B/A/B, FETCH/WRITE passes
set -u
O=gpurun_out/r5zf; mkdir -p $O
export TMPDIR=/tmp
run() {  # workload variant rep steps
  if [ $2 = cur ]; then unset NFK_LIBRARY; else export NFK_LIBRARY=build_ab/$2/libnfk.so; fi
  timeout -k 10 300 python bench.py --workload $1 --steps $4 --warmup 2 --no-cpu-baseline > $O/$1-$2-$3.json 2> $O/$1-$2-$3.err || { echo "bench $1 $2 failed"; tail -5 $O/$1-$2-$3.err; exit 1; }
  echo "$1 $2 $3: $(python3 tools/bench_line.py $O/$1-$2-$3.json) $(python3 -c "import json;d=json.load(open('$O/$1-$2-$3.json'));r=d['roofline'];p=d['parity'];print(r['kernel'],r['mean_ms'],'maxrel',p['max_rel_dlog_prob'])")"
}
for r in 1 2; do for v in cur wnt; do run c5 $v $r 5; done; done
unset NFK_LIBRARY
bash tools/pmc_traffic_passes.sh r5zf/pmc_cur k_fused_nsf_wide --workload c5 || exit 1
export NFK_LIBRARY=build_ab/wnt/libnfk.so
bash tools/pmc_traffic_passes.sh r5zf/pmc_wnt k_fused_nsf_wide --workload c5 || exit 1
unset NFK_LIBRARY
for v in cur wnt; do echo "== $v"; python3 tools/pmc_summary.py gpurun_out/r5zf/pmc_$v --kernel k_fused_nsf_wide | grep -E "FETCH|WRITE|hbm" ; done
echo done

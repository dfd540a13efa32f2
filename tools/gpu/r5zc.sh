#!/bin/bash
# Round 5 (zc): x rows of the c3 chain loaded with the non-temporal policy (NFK_X_NT=1,
# build_ab/xnt) vs HEAD: c3 time A/B/A/B, then FETCH/WRITE passes of each
set -u
O=gpurun_out/r5zc; mkdir -p $O
export TMPDIR=/tmp
run() {  # workload variant rep steps
  if [ $2 = cur ]; then unset NFK_LIBRARY; else export NFK_LIBRARY=build_ab/$2/libnfk.so; fi
  timeout -k 10 300 python bench.py --workload $1 --steps $4 --warmup 3 --no-cpu-baseline > $O/$1-$2-$3.json 2> $O/$1-$2-$3.err || { echo "bench $1 $2 failed"; tail -5 $O/$1-$2-$3.err; exit 1; }
  echo "$1 $2 $3: $(python3 tools/bench_line.py $O/$1-$2-$3.json) $(python3 -c "import json;d=json.load(open('$O/$1-$2-$3.json'));r=d['roofline'];p=d['parity'];print(r['kernel'],r['mean_ms'],'maxrel',p['max_rel_dlog_prob'])")"
}
for r in 1 2 3; do for v in cur xnt; do run c3 $v $r 20; done; done
unset NFK_LIBRARY
bash tools/pmc_traffic_passes.sh r5zc/pmc_cur k_nsf_chain2 || exit 1
export NFK_LIBRARY=build_ab/xnt/libnfk.so
bash tools/pmc_traffic_passes.sh r5zc/pmc_xnt k_nsf_chain2 || exit 1
unset NFK_LIBRARY
for v in cur xnt; do echo "== $v"; python3 tools/pmc_summary.py gpurun_out/r5zc/pmc_$v --kernel k_nsf_chain2 | grep -E "FETCH|WRITE|HBM|bytes" ; done
echo done

#!/bin/bash
# Round 5 (zd): x rows of the c2 RealNVP chain by non-temporal loads (NFK_X_NT=1,
# build_ab/xnt, which also covers the c3 chain) vs HEAD: c2 time A/B/A/B, FETCH/WRITE passes
set -u
O=gpurun_out/r5zd; mkdir -p $O
export TMPDIR=/tmp
run() {  # workload variant rep steps
  if [ $2 = cur ]; then unset NFK_LIBRARY; else export NFK_LIBRARY=build_ab/$2/libnfk.so; fi
  timeout -k 10 300 python bench.py --workload $1 --steps $4 --warmup 3 --no-cpu-baseline > $O/$1-$2-$3.json 2> $O/$1-$2-$3.err || { echo "bench $1 $2 failed"; tail -5 $O/$1-$2-$3.err; exit 1; }
  echo "$1 $2 $3: $(python3 tools/bench_line.py $O/$1-$2-$3.json) $(python3 -c "import json;d=json.load(open('$O/$1-$2-$3.json'));r=d['roofline'];p=d['parity'];print(r['kernel'],r['mean_ms'],'maxrel',p['max_rel_dlog_prob'])")"
}
for r in 1 2 3; do for v in cur xnt; do run c2 $v $r 20; done; done
unset NFK_LIBRARY
bash tools/pmc_traffic_passes.sh r5zd/pmc_cur k_rnvp_chain --workload c2 || exit 1
export NFK_LIBRARY=build_ab/xnt/libnfk.so
bash tools/pmc_traffic_passes.sh r5zd/pmc_xnt k_rnvp_chain --workload c2 || exit 1
unset NFK_LIBRARY
for v in cur xnt; do echo "== $v"; python3 tools/pmc_summary.py gpurun_out/r5zd/pmc_$v --kernel k_rnvp_chain | grep -E "FETCH|WRITE|hbm" ; done
echo done

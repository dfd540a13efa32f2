#!/bin/bash
# Round 5 (z): wave priority by phase in the c3 chain (NFK_C2_PRIO: p1 = GEMM
# sub-records at priority 1, p2 = epilogues at priority 1) vs HEAD, c3 A/B/A/B
set -u
O=gpurun_out/r5z; mkdir -p $O
export TMPDIR=/tmp
run() {  # workload variant rep steps
  if [ $2 = cur ]; then unset NFK_LIBRARY; else export NFK_LIBRARY=build_ab/$2/libnfk.so; fi
  timeout -k 10 300 python bench.py --workload $1 --steps $4 --warmup 3 --no-cpu-baseline > $O/$1-$2-$3.json 2> $O/$1-$2-$3.err || { echo "bench $1 $2 failed"; tail -5 $O/$1-$2-$3.err; exit 1; }
  echo "$1 $2 $3: $(python3 tools/bench_line.py $O/$1-$2-$3.json) $(python3 -c "import json;d=json.load(open('$O/$1-$2-$3.json'));r=d['roofline'];p=d['parity'];print(r['kernel'],r['mean_ms'],'maxrel',p['max_rel_dlog_prob'])")"
}
for r in 1 2 3; do for v in cur p1 p2; do run c3 $v $r 20; done; done
unset NFK_LIBRARY
echo done

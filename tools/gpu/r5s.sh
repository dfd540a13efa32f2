#!/bin/bash
# Round 5 (s): tanh variants A/B -- HEAD (7 VALU), tanh6 (6), tanh5 (5: signed x, no |x| or
# copysign), tanh5c (tanh5 + -ffp-contract=fast in the fused units)
# copysign) on c3, c2 (3 rounds), c5 and the Gaussian NSF_AR (1 round); parity each run
set -u
O=gpurun_out/r5s; mkdir -p $O
export TMPDIR=/tmp
run() {  # workload variant rep steps
  if [ $2 = cur ]; then unset NFK_LIBRARY; else export NFK_LIBRARY=build_ab/$2/libnfk.so; fi
  timeout -k 10 300 python bench.py --workload $1 --steps $4 --warmup 3 --no-cpu-baseline > $O/$1-$2-$3.json 2> $O/$1-$2-$3.err || { echo "bench $1 $2 failed"; tail -5 $O/$1-$2-$3.err; exit 1; }
  echo "$1 $2 $3: $(python3 tools/bench_line.py $O/$1-$2-$3.json) $(python3 -c "import json;d=json.load(open('$O/$1-$2-$3.json'));r=d['roofline'];p=d['parity'];print(r['kernel'],r['mean_ms'],'maxrel',p['max_rel_dlog_prob'])")"
}
for w in c3 c2; do for r in 1 2 3; do for v in cur tanh6 tanh5 tanh5c; do run $w $v $r 20; done; done; done
for w in c5 ar; do for v in cur tanh5 tanh5c; do run $w $v 1 5; done; done
unset NFK_LIBRARY
echo done

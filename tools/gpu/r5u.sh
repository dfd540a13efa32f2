#!/bin/bash
# Round 5 (u): the fp16 residual by v_fma_mix (NFK_SPLIT_MIX, with the 6-VALU tanh): its
# bitwise check, the full GPU suite + smoke, then A/B vs the plain residual (nomix) on
# c3 / c2 (3 rounds), c5 / ar (1 round)
set -u
O=gpurun_out/r5u; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 ./tools/ubench_split_mix > $O/split_mix.txt 2>&1; rc=$?; cat $O/split_mix.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
[ $rc -ne 0 ] && exit $rc
run() {  # workload variant rep steps
  if [ $2 = cur ]; then unset NFK_LIBRARY; else export NFK_LIBRARY=build_ab/$2/libnfk.so; fi
  timeout -k 10 300 python bench.py --workload $1 --steps $4 --warmup 3 --no-cpu-baseline > $O/$1-$2-$3.json 2> $O/$1-$2-$3.err || { echo "bench $1 $2 failed"; tail -5 $O/$1-$2-$3.err; exit 1; }
  echo "$1 $2 $3: $(python3 tools/bench_line.py $O/$1-$2-$3.json) $(python3 -c "import json;d=json.load(open('$O/$1-$2-$3.json'));r=d['roofline'];p=d['parity'];print(r['kernel'],r['mean_ms'],'maxrel',p['max_rel_dlog_prob'])")"
}
for w in c3 c2; do for r in 1 2 3; do for v in cur nomix; do run $w $v $r 20; done; done; done
for w in c5 ar; do for v in cur nomix; do run $w $v 1 5; done; done
unset NFK_LIBRARY
echo done

#!/bin/bash
# Round 4: fused VJP without packed-fp32 VALU ops -- reproducibility at more sizes,
# the train step with the row gate lifted, and the all-objects no-packed build's forward speed
set -u
O=gpurun_out/r4b; mkdir -p $O
for v in nopk exactnopk; do
  echo "== $v"
  DBG_ROWS=32768,49152,65536,262144,1048576 DBG_REPS=4 DBG_MODELS=0 NFK_LIBRARY=$PWD/build_ab/$v/libnfk.so \
    timeout -k 10 150 python -u tools/dbg_vjp_poison.py > $O/$v.log 2>&1
  rc=$?; grep -h "vjp inv" $O/$v.log | awk '{d=0; for(i=1;i<=NF;i++) if($i=="diff" && $(i+1)+0>d) d=$(i+1)+0; print $1,$2,$3,$5, "maxdiff", d}' | sort | uniq -c; [ $rc -ne 0 ] && { tail -5 $O/$v.log; exit $rc; }
done
for v in base nopk; do
  NFK_LIBRARY=$PWD/build_ab/$v/libnfk.so timeout -k 10 200 python tools/bench_train.py --batch 1048576 --steps 5 --warmup 2 --no-torch --vjp-max-rows 100000000 > $O/train_$v.json 2> $O/train_$v.err || { echo "train $v failed"; tail -5 $O/train_$v.err; exit 1; }
  echo "train $v (gate lifted): $(tail -1 $O/train_$v.json | cut -c1-300)"
done
timeout -k 10 200 python tools/bench_train.py --batch 1048576 --steps 5 --warmup 2 --no-torch > $O/train_gated.json 2> $O/train_gated.err && echo "train gated: $(tail -1 $O/train_gated.json | cut -c1-300)"
for v in cur allnopk; do
  if [ $v = cur ]; then unset NFK_LIBRARY; else export NFK_LIBRARY=$PWD/build_ab/$v/libnfk.so; fi
  for w in c3 c5 c2 ar; do
    timeout -k 10 200 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_${v}_$w.json 2> $O/bench_${v}_$w.err || { echo "bench $v $w failed"; tail -5 $O/bench_${v}_$w.err; exit 1; }
    echo "bench $v $w: $(python -c "import json,sys; d=json.loads(open('$O/bench_${v}_$w.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
  done
done

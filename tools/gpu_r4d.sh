#!/bin/bash
# Round 4: VJP without packed FP32 (product build) + per-sample scaling: tests, reproducibility, train step
set -u
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_outlier.py tests/test_gpu_vjp.py -x -v --timeout 200 --timeout-method thread > $O/new.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $O/new.log | tail -30; [ $rc -ne 0 ] && { grep -B5 -A30 "Error\|assert" $O/new.log | head -80; exit $rc; }
DBG_ROWS=32768,49152,65536,262144,1048576 DBG_REPS=4 DBG_MODELS=0 timeout -k 10 150 python -u tools/dbg_vjp_poison.py > $O/vjp_det.log 2>&1
rc=$?; grep -h "vjp inv" $O/vjp_det.log | awk '{d=0; for(i=1;i<=NF;i++) if($i=="diff" && $(i+1)+0>d) d=$(i+1)+0; print $1,$2,$3, "maxdiff", d}' | sort | uniq -c; [ $rc -ne 0 ] && { tail -5 $O/vjp_det.log; exit $rc; }
for v in cur; do
  if [ $v = cur ]; then unset NFK_LIBRARY; else export NFK_LIBRARY=$PWD/build_ab/$v/libnfk.so; fi
  timeout -k 10 200 python tools/bench_train.py --batch 1048576 --steps 5 --warmup 2 --no-torch > $O/train_$v.json 2> $O/train_$v.err || { echo "train $v failed"; tail -5 $O/train_$v.err; exit 1; }
  echo "train $v: $(tail -1 $O/train_$v.json | cut -c1-300)"
done
unset NFK_LIBRARY
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -ne 0 ] && { grep -B5 -A40 "^____\|Error" $O/suite.log | head -80; exit $rc; }
exit 0

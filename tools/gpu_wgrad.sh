# nfk_wgrad: tests, then the c3 train step with and without it (2^20 rows)
set -u
O=gpurun_out/wgrad; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wgrad.py -rs > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -12 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in on off on off on off; do
  f=""; [ $v = off ] && f="--no-wgrad-mfma"
  timeout -k 10 300 python tools/bench_train.py --batch 1048576 --steps 5 --warmup 2 --no-torch $f > $O/train_$v.json 2> $O/train_$v.err; rc=$?
  echo "train $v rc=$rc: $(cat $O/train_$v.json)"; [ $rc -eq 0 ] || { tail -5 $O/train_$v.err; exit $rc; }
done
exit 0

#!/bin/bash
# Round 5 (f): NSF_AR + chain tests after the column-order log|det| sum rewrite and the
# branch-free chain2 map reads; bench lines c3, ar354, fe162, poly2048; then the VJP
# discriminating variants: reload (element backward on re-read inputs) and twice (two evaluations)
set -u
O=gpurun_out/r5f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_nsfar_fused.py tests/test_gpu_chain.py -q -rf -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|fe162|poly2048" $O/pytest.log | tail -6
[ $rc -ne 0 ] && exit $rc
for w in c3 ar354 fe162 poly2048; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$w.json'));r=d['roofline'];print('$w', d['value'], 'samples/s', d['ms_per_step'], 'ms/step', r['kernel'], r['mean_ms'], 'ms', r['bound'], r['frac'], d['parity']['pass'])"
done
for v in fastre reload twice; do
  echo "== $v"
  DBG_ROWS=262144 DBG_REPS=3 NFK_LIBRARY=$PWD/build_ab/$v/libnfk.so \
    timeout -k 10 240 python -u tools/dbg_vjp_save.py > $O/vjp_$v.log 2>&1
  rc=$?; grep -h "inv=\|twice" $O/vjp_$v.log | head -24; [ $rc -ne 0 ] && { tail -5 $O/vjp_$v.log; exit $rc; }
done
echo done

#!/bin/bash
# Round 5 (m): nfk_fused_ar.hip built without packed FP32 as a unit (the 512-register
# instances take it back per kernel): the AR / CL tests, bench lines, and the streamed
# form's sub-record ring A/B at Polymer's 40 rows
set -u
O=gpurun_out/r5m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_nsfar_fused.py tests/test_gpu_cl_wide.py tests/test_gpu_parity.py tests/test_gpu_forward_repro.py -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for w in ar ar354 fe162; do
  timeout -k 10 300 python bench.py --workload $w --steps 30 --no-cpu-baseline --parity-rows 1024 > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  echo "$w: $(python3 tools/bench_line.py $O/$w.json) $(python3 -c "import json;d=json.load(open('$O/$w.json'));r=d['roofline'];print(r['kernel'],r['mean_ms'],r['frac'])")"
done
NFK_LIBRARY=build_ab/ars4k1/libnfk.so timeout -k 10 300 python -u -m pytest tests/test_gpu_nsfar_fused.py -k "streamed or polymer" -q -rf --timeout 200 --timeout-method thread > $O/pytest_ars4k1.log 2>&1; rc=$?; echo "pytest ars4k1 rc=$rc"; tail -2 $O/pytest_ars4k1.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in cur ars2k1 ars4k1; do
    if [ $v = cur ]; then unset NFK_LIBRARY; else export NFK_LIBRARY=build_ab/$v/libnfk.so; fi
    timeout -k 10 300 python bench.py --workload poly2048 --steps 30 --warmup 3 --no-cpu-baseline --parity-rows 40 > $O/poly-$v-$r.json 2> $O/poly-$v-$r.err || { echo "bench $v failed"; tail -5 $O/poly-$v-$r.err; exit 1; }
    echo "poly2048 $v $r: $(python3 tools/bench_line.py $O/poly-$v-$r.json) $(python3 -c "import json;d=json.load(open('$O/poly-$v-$r.json'));r=d['roofline'];print(r['kernel'],r['mean_ms'],r['frac'])")"
  done
done
unset NFK_LIBRARY
echo done

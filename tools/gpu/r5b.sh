#!/bin/bash
# Round 5 (b): the NSF_AR tests (Fe dim 162, Polymer goldens), the packed-FP32 read-after-write microbenchmark (tools/ubench_pk_raw.hip), then
# an A/B of the product build vs one without packed-FP32 VALU code anywhere (build_ab/nopkall)
set -u
O=gpurun_out/r5b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_nsfar_fused.py -q -rf -s --timeout 200 --timeout-method thread > $O/pytest_ar.log 2>&1; echo "pytest_ar rc=$?"; grep -E "passed|failed|fe162" $O/pytest_ar.log | tail -5
timeout -k 10 120 ./tools/ubench_pk_raw > $O/ubench_pk_raw.txt 2>&1 || { tail -5 $O/ubench_pk_raw.txt; exit 1; }
cat $O/ubench_pk_raw.txt
for w in c3 c5 c2 ar; do
  for v in base nopkall; do
    L=""; [ $v = nopkall ] && L="NFK_LIBRARY=$PWD/build_ab/nopkall/libnfk.so"
    env $L timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --parity-rows 2048 > $O/${w}_$v.json 2> $O/${w}_$v.err || { tail -5 $O/${w}_$v.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${w}_$v.json'));print('$w $v', round(d['value']/1e6,2),'M/s', d['roofline']['mean_ms'],'ms', 'parity', d['parity']['pass'])"
  done
done
echo done

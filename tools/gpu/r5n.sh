#!/bin/bash
# Round 5 (n): waves whose rows all lie past the batch skip their MFMAs (AR register and
# streamed forms, the wide CL kernel): AR / CL tests, bench lines at the applications' batches
set -u
O=gpurun_out/r5n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_nsfar_fused.py tests/test_gpu_cl_wide.py tests/test_gpu_parity.py tests/test_gpu_outlier.py -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for w in ar354 fe162 poly2048; do
  timeout -k 10 300 python bench.py --workload $w --steps 50 --no-cpu-baseline --parity-rows 1024 > $O/$w-$r.json 2> $O/$w-$r.err || { tail -5 $O/$w-$r.err; exit 1; }
  echo "$w $r: $(python3 tools/bench_line.py $O/$w-$r.json) $(python3 -c "import json;d=json.load(open('$O/$w-$r.json'));r=d['roofline'];print(r['kernel'],r['mean_ms'],r['frac'])")"
done
done
timeout -k 10 300 python tools/time_cl354.py > $O/cl354.txt 2>&1 || { tail -5 $O/cl354.txt; exit 1; }
tail -6 $O/cl354.txt
echo done

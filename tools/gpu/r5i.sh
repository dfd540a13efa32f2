#!/bin/bash
# Round 5 (i): NSF_AR golden parity (dim-scaled log|det| slack), host profile of the NSF_AR
# workloads with the C++ cache-key helper, bench lines (with the CPU leg) for ar354/fe162/poly2048,
# a kernel-trace summary and the HBM-traffic passes of fe162 and poly2048
set -u
O=gpurun_out/r5i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k nsfar -q -rf --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for w in ar354 fe162 poly2048; do
  timeout -k 10 200 python -u tools/prof_host_ar.py $w > $O/host_$w.txt 2>&1 || { tail -5 $O/host_$w.txt; exit 1; }
  grep -m1 "ms per step" $O/host_$w.txt
done
for w in ar354 fe162 poly2048; do
  timeout -k 10 300 python bench.py --workload $w > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$w.json'));r=d['roofline'];print('$w', d['value'], 'samples/s', d['ms_per_step'], 'ms/step', r['kernel'], r['mean_ms'], 'ms', r['bound'], r['frac'], d['parity']['pass'], 'cpu', d['cpu_baseline']['value'])"
done
for w in fe162 poly2048; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run -- python3 bench.py --workload $w --steps 10 --no-cpu-baseline --no-timer > $O/prof_$w.log 2>&1 || { tail -5 $O/prof_$w.log; exit 1; }
  bash tools/pmc_traffic_passes.sh r5i/pmc_$w k_fused_ar --workload $w || exit 1
done
echo done

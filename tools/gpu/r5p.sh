#!/bin/bash
# Round 5 (p): full GPU suite + smoke; c5 with the serpentine chunk order vs without
# (NFK_WIDE_SERP=0): bench A/B and HBM traffic passes of both; the c3 line with its CPU leg,
# its rocprofv3 kernel-trace summary and PMC passes; NSF_AR lines
set -u
O=gpurun_out/r5p; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in serp noserp; do
    if [ $v = noserp ]; then export NFK_WIDE_SERP=0; else unset NFK_WIDE_SERP; fi
    timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline --parity-rows 1024 > $O/c5-$v-$r.json 2> $O/c5-$v-$r.err || { tail -5 $O/c5-$v-$r.err; exit 1; }
    echo "c5 $v $r: $(python3 tools/bench_line.py $O/c5-$v-$r.json) $(python3 -c "import json;d=json.load(open('$O/c5-$v-$r.json'));r=d['roofline'];print(r['kernel'],r['mean_ms'],r['frac'])")"
  done
done
unset NFK_WIDE_SERP
bash tools/pmc_traffic_passes.sh r5p/pmc_c5_serp k_fused_nsf_wide --workload c5 || exit 1
NFK_WIDE_SERP=0 bash tools/pmc_traffic_passes.sh r5p/pmc_c5_noserp k_fused_nsf_wide --workload c5 || exit 1
timeout -k 10 400 python bench.py > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
echo "c3: $(python3 tools/bench_line.py $O/c3.json)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 bench.py --no-cpu-baseline > $O/prof_c3.log 2>&1 || { tail -5 $O/prof_c3.log; exit 1; }
bash tools/pmc_passes.sh r5p/pmc_c3 k_nsf_chain2 || exit 1
for w in ar354 fe162 poly2048 c2; do
  timeout -k 10 300 python bench.py --workload $w --steps 30 > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  echo "$w: $(python3 tools/bench_line.py $O/$w.json) $(python3 -c "import json;d=json.load(open('$O/$w.json'));r=d['roofline'];print(r['kernel'],r['mean_ms'],r['frac'])")"
done
echo done

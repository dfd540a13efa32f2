#!/bin/bash
# Round 5 (zg): the closing build (x rows non-temporal in the c3 and c2 chains) -- full GPU suite + smoke, every bench line (c3 with its CPU
# leg), the c3 rocprofv3 kernel-trace summary
set -u
O=gpurun_out/r5zg; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
echo "c3: $(python3 tools/bench_line.py $O/c3.json)"
for w in c2 c5 ar ar354 fe162 poly2048; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  echo "$w: $(python3 tools/bench_line.py $O/$w.json) $(python3 -c "import json;d=json.load(open('$O/$w.json'));r=d['roofline'];print(r['kernel'],r['mean_ms'],r['frac'],r['floors'].get('valu_issue_frac'))")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 bench.py --no-cpu-baseline > $O/prof_c3.log 2>&1 || { tail -5 $O/prof_c3.log; exit 1; }
echo done

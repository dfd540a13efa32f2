#!/bin/bash
# Round 5 (v): the prefix max as a v_max3 tree (NFK_MAX3_ASM): full GPU suite + smoke, c3 / c2
# lines with the CPU leg, c3 rocprofv3 summary
set -u
O=gpurun_out/r5v; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
[ $rc -ne 0 ] && exit $rc
for w in c3 c2 c5 ar; do
  timeout -k 10 400 python bench.py --workload $w > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  echo "$w: $(python3 tools/bench_line.py $O/$w.json) $(python3 -c "import json;d=json.load(open('$O/$w.json'));r=d['roofline'];print(r['kernel'],r['mean_ms'],r['frac'],r['floors'].get('valu_issue_frac'))")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 bench.py --no-cpu-baseline > $O/prof_c3.log 2>&1 || { tail -5 $O/prof_c3.log; exit 1; }
echo done

#!/bin/bash
# Round 5 (o): the full GPU suite and smoke on the committed build, the c3 bench line with its CPU leg, a
# rocprofv3 kernel-trace summary of the same command, the c3 chain's PMC passes (instruction
# counts, HBM traffic) on this round's build, NSF_AR bench lines
set -u
O=gpurun_out/r5o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
echo "c3: $(python3 tools/bench_line.py $O/c3.json)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 bench.py --no-cpu-baseline > $O/prof_c3.log 2>&1 || { tail -5 $O/prof_c3.log; exit 1; }
bash tools/pmc_passes.sh r5o/pmc_c3 k_nsf_chain2 || exit 1
for w in ar354 fe162 poly2048; do
  timeout -k 10 300 python bench.py --workload $w --steps 50 > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  echo "$w: $(python3 tools/bench_line.py $O/$w.json) $(python3 -c "import json;d=json.load(open('$O/$w.json'));r=d['roofline'];print(r['kernel'],r['mean_ms'],r['frac'])")"
done
echo done

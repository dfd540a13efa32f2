#!/bin/bash
# Round 5 (j): the NSF_AR tests after the ld-sum rewrite (1024-thread, double-buffered) and
# the C++ pack watch; NSF_AR bench lines (100 steps); kernel stats (csv) for poly2048/fe162;
# the element-backward twice microbenchmark; c3 A/B of three epilogue/ISA variants
set -u
O=gpurun_out/r5j; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_nsfar_fused.py tests/test_gpu_parity.py -k "nsfar or ar_ or fused_ar or streamed or polymer or fe162" -q -rf --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for w in ar354 fe162 poly2048; do
  timeout -k 10 300 python bench.py --workload $w --steps 100 --no-cpu-baseline > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$w.json'));r=d['roofline'];print('$w', d['value'], 'samples/s', d['ms_per_step'], 'ms/step', r['kernel'], r['mean_ms'], 'ms', r['bound'], r['frac'], d['parity']['pass'])"
done
for w in fe162 poly2048; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python3 bench.py --workload $w --steps 20 --no-cpu-baseline --no-timer > $O/prof_$w.log 2>&1 || { tail -5 $O/prof_$w.log; exit 1; }
done
echo "== element backward twice (packed build, then without packed FP32)"
timeout -k 10 120 ./tools/ubench_elem_twice 4 16 > $O/ubench_elem_twice.txt 2>&1 || { tail -5 $O/ubench_elem_twice.txt; exit 1; }
cat $O/ubench_elem_twice.txt
timeout -k 10 120 ./tools/ubench_elem_twice_nopk 4 16 > $O/ubench_elem_twice_nopk.txt 2>&1 || { tail -5 $O/ubench_elem_twice_nopk.txt; exit 1; }
cat $O/ubench_elem_twice_nopk.txt
echo "== c3 A/B"
for r in 1 2; do
  for v in cur lut2 lut0 nopk; do
    if [ $v = cur ]; then unset NFK_LIBRARY; else export NFK_LIBRARY=build_ab/$v/libnfk.so; fi
    timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline --parity-rows 4096 > $O/c3-$v-$r.json 2> $O/c3-$v-$r.err || { echo "bench c3 $v failed"; tail -5 $O/c3-$v-$r.err; exit 1; }
    echo "c3 $v $r: $(python3 tools/bench_line.py $O/c3-$v-$r.json)"
  done
done
unset NFK_LIBRARY
echo done

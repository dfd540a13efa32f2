#!/bin/bash
# Round 5 (k): the element-backward microbenchmark with per-evaluation verdicts against a
# reference launch (which of the two evaluations goes wrong, under which burst), packed and
# non-packed builds; bench A/B of the whole library built without packed FP32 (nopk) vs HEAD
set -u
O=gpurun_out/r5k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 ./tools/ubench_elem_twice 2 64 > $O/ubench_elem.txt 2>&1 || { tail -5 $O/ubench_elem.txt; exit 1; }
cat $O/ubench_elem.txt
timeout -k 10 200 ./tools/ubench_elem_twice_nopk 2 64 > $O/ubench_elem_nopk.txt 2>&1 || { tail -5 $O/ubench_elem_nopk.txt; exit 1; }
cat $O/ubench_elem_nopk.txt
for w in c2 c5 ar ar354 fe162; do
  for r in 1 2; do
    for v in cur nopk; do
      if [ $v = cur ]; then unset NFK_LIBRARY; else export NFK_LIBRARY=build_ab/$v/libnfk.so; fi
      timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --parity-rows 1024 > $O/$w-$v-$r.json 2> $O/$w-$v-$r.err || { echo "bench $w $v failed"; tail -5 $O/$w-$v-$r.err; exit 1; }
      echo "$w $v $r: $(python3 tools/bench_line.py $O/$w-$v-$r.json) $(python3 -c "import json;d=json.load(open('$O/$w-$v-$r.json'));r=d['roofline'];print(r['kernel'],r['mean_ms'])")"
    done
  done
done
unset NFK_LIBRARY
echo done

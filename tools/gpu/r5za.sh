#!/bin/bash
# Round 5 (za): c5 wide kernel workgroup shape -- w4f32 = 4-wave workgroups with
# 32-block frames (two workgroups per CU, so the two waves sharing a SIMD come from
# different workgroups and need not be in the same phase), w8f32 = the default
# 8-wave workgroup with 32-block frames (control) -- vs HEAD, A/B/A/B
set -u
O=gpurun_out/r5za; mkdir -p $O
export TMPDIR=/tmp
run() {  # workload variant rep steps
  if [ $2 = cur ]; then unset NFK_LIBRARY; else export NFK_LIBRARY=build_ab/$2/libnfk.so; fi
  timeout -k 10 300 python bench.py --workload $1 --steps $4 --warmup 2 --no-cpu-baseline > $O/$1-$2-$3.json 2> $O/$1-$2-$3.err || { echo "bench $1 $2 failed"; tail -5 $O/$1-$2-$3.err; exit 1; }
  echo "$1 $2 $3: $(python3 tools/bench_line.py $O/$1-$2-$3.json) $(python3 -c "import json;d=json.load(open('$O/$1-$2-$3.json'));r=d['roofline'];p=d['parity'];print(r['kernel'],r['mean_ms'],'maxrel',p['max_rel_dlog_prob'])")"
}
for r in 1 2; do for v in cur w4f32 w8f32; do run c5 $v $r 5; done; done
unset NFK_LIBRARY
echo done

#!/bin/bash
# Round 4: uniform-address (saddr) weight DMA A/B on the c5 wide kernel and the fused NSF_AR
set -u
O=gpurun_out/r4z; mkdir -p $O
for pass in 1 2; do
  for v in base c5saddr; do
    if [ $v = base ]; then L=$PWD/normalizingflow_amd/libnfk.so; else L=$PWD/build_ab/$v/libnfk.so; fi
    NFK_LIBRARY=$L timeout -k 10 200 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline --parity-rows 1024 > $O/c5_$v.$pass.json 2> $O/c5_$v.$pass.err || { echo "$v failed"; tail -5 $O/c5_$v.$pass.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/c5_$v.$pass.json').read().strip().splitlines()[-1]); print('c5 $pass $v', round(d['roofline']['mean_ms'],4), round(d['value']/1e6,3), 'parity', d['parity']['pass'])"
  done
  for v in base arsaddr; do
    if [ $v = base ]; then L=$PWD/normalizingflow_amd/libnfk.so; else L=$PWD/build_ab/$v/libnfk.so; fi
    NFK_LIBRARY=$L timeout -k 10 200 python bench.py --workload ar --steps 10 --warmup 2 --no-cpu-baseline --parity-rows 1024 > $O/ar_$v.$pass.json 2> $O/ar_$v.$pass.err || { echo "$v failed"; tail -5 $O/ar_$v.$pass.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/ar_$v.$pass.json').read().strip().splitlines()[-1]); print('ar $pass $v', round(d['roofline']['mean_ms'],4), round(d['value']/1e6,3), 'parity', d['parity']['pass'])"
  done
done

#!/bin/bash
# Round 4: c3 chain kernel A/B -- LLVM scheduler strategies, packed knot prefixes, the
# uniform-address DMA -- each a libnfk.so differing only in nfk_fused_chain2.o; two passes
set -u
O=gpurun_out/r4v; mkdir -p $O
for pass in 1 2; do
  for v in base c3ilp c3memcl c3itilp c3pk2 c3nosaddr; do
    if [ $v = base ]; then L=$PWD/normalizingflow_amd/libnfk.so; else L=$PWD/build_ab/$v/libnfk.so; fi
    NFK_LIBRARY=$L timeout -k 10 120 python bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline --parity-rows 2048 > $O/$v.$pass.json 2> $O/$v.$pass.err || { echo "$v failed"; tail -5 $O/$v.$pass.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/$v.$pass.json').read().strip().splitlines()[-1]); print('$pass $v', round(d['roofline']['mean_ms'],4), 'parity', d['parity']['pass'])"
  done
done

#!/bin/bash
# Round 6 (s): c3 chain built under three AMDGPU scheduler strategies (A/B)
set -u
O=gpurun_out/r6s; mkdir -p $O
export TMPDIR=/tmp
run() {  # name, library
    NFK_LIBRARY=$2 timeout -k 10 180 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { tail -3 $O/$1.err; return 1; }
    python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', round(d['value']/1e6,2), 'M/s', d['ms_per_step'], 'ms', 'parity', d['parity']['pass'])"
}
L=normalizingflow_amd/libnfk.so
run base0 $L &&
run max_ilp build_ab/c3_max-ilp/libnfk.so &&
run iter_ilp build_ab/c3_iterative-ilp/libnfk.so &&
run mem_clause build_ab/c3_max-memory-clause/libnfk.so &&
run base1 $L &&
run max_ilp_2 build_ab/c3_max-ilp/libnfk.so &&
run iter_ilp_2 build_ab/c3_iterative-ilp/libnfk.so
echo done

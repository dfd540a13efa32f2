#!/bin/bash
# Round 6 (ac): c3 chain A/B -- s_setprio 1 around the GEMM clusters (NFK_C2_PRIO)
set -u
O=gpurun_out/r6ac; mkdir -p $O
export TMPDIR=/tmp
run() {
    NFK_LIBRARY=$2 timeout -k 10 180 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { tail -3 $O/$1.err; return 1; }
    python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', round(d['value']/1e6,2), 'M/s', d['ms_per_step'], 'ms', 'parity', d['parity']['pass'])"
}
L=normalizingflow_amd/libnfk.so; P=build_ab/c3_prio/libnfk.so
run base0 $L && run prio0 $P && run base1 $L && run prio1 $P && run base2 $L && run prio2 $P
echo done

#!/bin/bash
# c3 chain kernel: pre-RA scheduler variants (whole-library builds under build_ab/), A/B/A/B on one box
set -u
O=gpurun_out/r3sched; mkdir -p $O
for i in 1 2; do
  for v in base bd mb; do
    lib=normalizingflow_amd/libnfk.so; [ $v != base ] && lib=build_ab/$v/libnfk.so
    NFK_LIBRARY=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --parity-rows 4096 > $O/c3_${v}_$i.json 2> $O/c3_${v}_$i.err; rc=$?
    echo "$v $i rc=$rc $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['value'], d['roofline']['mean_ms'], d['parity']['pass'] if isinstance(d.get('parity'),dict) else d.get('parity'))" $O/c3_${v}_$i.json 2>&1 | tail -1)"
    [ $rc -eq 0 ] || exit $rc
  done
done

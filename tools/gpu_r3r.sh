#!/bin/bash
# Round 3 session r: fused AR inverse, HEAD vs tree (LDS-DMA spline inputs).
set -u
O=gpurun_out/r3r; mkdir -p $O
for r in 1 2; do
  NFK_LIBRARY=build_ab/head/libnfk.so timeout -k 10 200 python tools/diag/ar_inverse_time.py > $O/head_$r.log 2>&1 || exit $?
  timeout -k 10 200 python tools/diag/ar_inverse_time.py > $O/tree_$r.log 2>&1 || exit $?
done
for f in $O/*.log; do echo "$f $(tail -1 $f)"; done

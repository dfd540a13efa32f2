#!/bin/bash
# Round 4: the wide fused NSF_AR (H = 354) parity failure -- diagnostic variants
set -u
O=gpurun_out/r4f; mkdir -p $O
for v in cur arpad arpostnop artailnop arboth; do
  if [ $v = cur ]; then unset NFK_LIBRARY; else export NFK_LIBRARY=$PWD/build_ab/$v/libnfk.so; fi
  timeout -k 10 200 python -u -m pytest tests/test_gpu_nsfar_fused.py -q -k "golden" --timeout 100 --timeout-method thread > $O/$v.log 2>&1
  rc=$?; echo "== $v rc=$rc: $(tail -1 $O/$v.log)"; grep -h "^FAILED\|Greatest absolute" $O/$v.log | head -8
  case $rc in 0|1) ;; *) exit $rc;; esac
done
exit 0

#!/bin/bash
# Round 3 session d: fused NSF_AR sub-record width (NS) x workgroup size (NW) A/B, tests.
set -u
O=gpurun_out/r3d; mkdir -p $O
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; grep -h '^{' $O/$n.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); r=d.get('roofline') or {}; print('  value %.1f M/s  ms/step %.4f  kernel %s %.4f ms  frac %s  parity %s' % (d['value']/1e6, d['ms_per_step'], r.get('kernel'), r.get('mean_ms', 0), r.get('frac'), (d.get('parity') or {}).get('pass')))" 2>/dev/null || tail -3 $O/$n.log
  [ $rc -eq 0 ] || exit $rc
}
run ar_tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_nsfar_fused.py
run wide_tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wide.py
run bench_c5 300 python bench.py --workload c5 --no-cpu-baseline
for r in 1 2; do
  for nw in 4 8; do
    NFK_AR_WAVES=$nw run ar_ns3_w${nw}_$r 300 python bench.py --workload ar --no-cpu-baseline --parity-rows 4096
    NFK_LIBRARY=build_ab/arns2/libnfk.so NFK_AR_WAVES=$nw run ar_ns2_w${nw}_$r 300 python bench.py --workload ar --no-cpu-baseline --parity-rows 4096
  done
done

#!/bin/bash
# Round 6 (t): rnvp2048 with the hidden layers' GEMM + activation fused (k_wl_gemm_act)
set -u
O=gpurun_out/r6t; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rnvp_polymer.py -m gpu -v -rP --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error" $O/pytest.log | tail -5
[ $rc -ne 0 ] && exit $rc
for f in 1 0 1; do
  NFK_WL_FUSED=$f timeout -k 10 240 python3 bench.py --workload rnvp2048 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_f$f.json 2> $O/bench_f$f.err || { tail -5 $O/bench_f$f.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_f$f.json').read().strip().splitlines()[-1]); print('fused=$f', d['value'], d['ms_per_step'], 'ms', 'frac', d['roofline']['frac'], 'layer', d['roofline']['mean_ms'], 'parity', d['parity']['pass'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --workload rnvp2048 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
cut -d, -f1-4 $O/prof/run_kernel_stats.csv | grep -E "k_wl" | head
echo done

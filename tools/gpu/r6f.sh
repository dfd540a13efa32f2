#!/bin/bash
# Round 6 (f): sequential NSF_AR inverse with batched staging (one launch per
# column); weight-stream RealNVP GEMM shapes A/B (NFK_WL_CFG 0/1/2)
set -u
O=gpurun_out/r6f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_nsfar_fused.py tests/test_gpu_rnvp_polymer.py -m gpu -v -rP --timeout 300 --timeout-method thread -k "seqinv or polymer2048 or rnvp or wide" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error|poly2048" $O/pytest.log | tail -8
[ $rc -ne 0 ] && exit $rc
for c in 0 1 2; do
  NFK_WL_CFG=$c timeout -k 10 300 python bench.py --workload rnvp2048 --no-cpu-baseline --parity-rows 0 > $O/rnvp_cfg$c.json 2> $O/rnvp_cfg$c.err || { tail -5 $O/rnvp_cfg$c.err; exit 1; }
  echo "cfg $c: $(python3 -c "import json;d=json.load(open('$O/rnvp_cfg$c.json'));print(d['ms_per_step'], d['roofline']['mean_ms'], d['roofline']['frac'])")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_seqinv -o run -- python3 tools/time_ar_sample.py > $O/prof_seqinv.log 2>&1 || { tail -5 $O/prof_seqinv.log; exit 1; }
tail -25 $O/prof_seqinv.log
echo done

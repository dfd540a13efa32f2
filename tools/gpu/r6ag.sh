#!/bin/bash
# Round 6 (ag): sequential NSF_AR inverse -- chunk halves, one staging round trip,
# prefetch workgroups; tests, phase clocks, kernel trace
set -u
O=gpurun_out/r6ag; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_nsfar_fused.py -m gpu -v -rP --timeout 300 --timeout-method thread  > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error|poly2048" $O/pytest.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u tools/sq_phase_timing.py > $O/phases.json 2> $O/phases.err || { tail -5 $O/phases.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/phases.json')); print({k: v.get('median', v) for k, v in d.items()})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_seqinv -o run -- python3 tools/time_ar_sample.py > $O/prof_seqinv.log 2>&1 || { tail -5 $O/prof_seqinv.log; exit 1; }
grep polymer2048 $O/prof_seqinv.log | head -2
python3 tools/sq_trace_stats.py $O/prof_seqinv/run_kernel_trace.csv
echo done

#!/bin/bash
# Round 6 (e): NSF_AR column-loop inverse from the library (nfk_ar_seqinv):
# parity, Polymer inverse timing; the ar354 training step's host and kernel profile
set -u
O=gpurun_out/r6e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_nsfar_fused.py -m gpu -v -rP --timeout 300 --timeout-method thread -k "seqinv or polymer2048" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error|poly2048" $O/pytest.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/time_ar_sample.py > $O/ar_sample.json 2> $O/ar_sample.err || { tail -5 $O/ar_sample.err; exit 1; }
cat $O/ar_sample.json
timeout -k 10 300 python -u tools/prof_host_ar354_train.py > $O/host_ar354_train.txt 2>&1 || { tail -5 $O/host_ar354_train.txt; exit 1; }
head -45 $O/host_ar354_train.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_train_ar354 -o run -- python3 tools/bench_train.py --workload ar354 --batch 40 --steps 10 --no-torch > $O/prof_train_ar354.log 2>&1 || { tail -5 $O/prof_train_ar354.log; exit 1; }
echo done
timeout -k 10 300 python -u tools/time_rnvp2048.py > $O/time_rnvp2048.json 2> $O/time_rnvp2048.err || { tail -5 $O/time_rnvp2048.err; exit 1; }
head -12 $O/time_rnvp2048.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_rnvp -o run -- python3 bench.py --workload rnvp2048 --no-cpu-baseline --steps 10 > $O/prof_rnvp.log 2>&1 || { tail -5 $O/prof_rnvp.log; exit 1; }
echo done2

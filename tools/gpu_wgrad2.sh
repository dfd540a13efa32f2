set -u
O=gpurun_out/wgrad2; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wgrad.py -rs > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -12 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ubench_wgrad_mfma.py > $O/ub.txt 2>&1; rc=$?; cat $O/ub.txt; [ $rc -eq 0 ] || exit $rc
exit 0

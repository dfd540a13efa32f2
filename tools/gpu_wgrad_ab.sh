set -u
timeout -k 10 300 python tools/ubench_wgrad_mfma.py > gpurun_out/wg_ub_tm2.txt 2>&1 || exit 1
NFK_LIBRARY=build_ab/tm4/libnfk.so timeout -k 10 300 python tools/ubench_wgrad_mfma.py > gpurun_out/wg_ub_tm4.txt 2>&1 || exit 1
cat gpurun_out/wg_ub_tm2.txt; echo ---; cat gpurun_out/wg_ub_tm4.txt

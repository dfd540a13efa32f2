#!/bin/bash
# Round 4: fused NSF_CL with the applications' wide conditioner (k_fused_cl): its tests, the
# applications' NSF_CL branch model test, timing of that branch; the ar354 host profile
set -u
O=gpurun_out/r4x; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_cl_wide.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_cl.log 2>&1 || { tail -40 $O/pytest_cl.log; exit 1; }
tail -3 $O/pytest_cl.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k applications --timeout 180 --timeout-method thread > $O/pt_app.log 2>&1 || { tail -30 $O/pt_app.log; exit 1; }
tail -2 $O/pt_app.log
timeout -k 10 200 python tools/time_cl354.py > $O/cl354.txt 2>&1 || { tail -5 $O/cl354.txt; exit 1; }
cat $O/cl354.txt
timeout -k 10 200 python -c "
import normalizingflow_amd.config as c; c.USE_FUSED=False
import runpy, sys; sys.argv=['t']; runpy.run_path('tools/time_cl354.py', run_name='__main__')" > $O/cl354_unfused.txt 2>&1 || { tail -5 $O/cl354_unfused.txt; exit 1; }
sed 's/^/unfused /' $O/cl354_unfused.txt
timeout -k 10 200 python tools/prof_host_ar354.py > $O/prof.txt 2>&1 || { tail -5 $O/prof.txt; exit 1; }
head -30 $O/prof.txt

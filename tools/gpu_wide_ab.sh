#!/bin/bash
# wide-kernel A/B: tests on the working-tree build, then c5 log_prob with the
# working tree and with build_ab/$1 (NFK_LIBRARY)
set -o pipefail
O=gpurun_out/wideab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for v in cur "$@"; do
  if [ $v = cur ]; then unset NFK_LIBRARY; else export NFK_LIBRARY=build_ab/$v/libnfk.so; fi
  timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { tail -5 $O/bench_$v.err; exit 1; }
  echo "$v: $(python -c "import json,sys;d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'])")"
done

#!/bin/bash
# Round 4: forced column-split A/B of the fused NSF_AR forward at large batches (ar354, 65536 rows)
set -u
O=gpurun_out/r4af; mkdir -p $O
for cs in 0 8 32 0 8 32; do
  NFK_AR_CSPLIT=$cs timeout -k 10 200 python bench.py --workload ar354 --batch 65536 --steps 5 --warmup 2 --no-cpu-baseline --parity-rows 64 > $O/cs$cs.json 2> $O/cs$cs.err || { echo "cs $cs failed"; tail -5 $O/cs$cs.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/cs$cs.json').read().strip().splitlines()[-1]); print('csplit $cs', d['ms_per_step'], round(d['value']/1e6,3), 'parity', d['parity']['pass'])"
done

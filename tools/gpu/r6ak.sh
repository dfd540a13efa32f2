#!/bin/bash
# Round 6 (ak): sequential NSF_AR inverse with and without the prefetch workgroups (A/B)
set -u
O=gpurun_out/r6ak; mkdir -p $O
export TMPDIR=/tmp
for v in 1 0 1 0; do
  NFK_SQ_PREFETCH=$v timeout -k 10 300 python3 -u tools/sq_phase_timing.py > $O/phases_$v.json 2> $O/phases_$v.err || { tail -5 $O/phases_$v.err; exit 1; }
  NFK_SQ_PREFETCH=$v timeout -k 10 300 python3 tools/time_ar_sample.py > $O/sample_$v.json 2> $O/sample_$v.err || { tail -5 $O/sample_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/phases_$v.json')); print('prefetch=$v stage', d['stage']['median'], 'finish', d['finish_total']['median'])"
  grep polymer2048 $O/sample_$v.err
done
echo done

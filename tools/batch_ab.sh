#!/bin/bash
# A/B of the launch batch size, interleaved so that box-level drift hits both
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in ${REPS_AB:-1 2}; do
  for b in ${BATCHES:-64 96}; do
    timeout -k 10 200 python bench.py --no-cpu --batch $b --steps 3 > gpurun_out/ab_${b}_${rep}.log 2>&1 || exit 1
    python -c "
import json;d=json.loads(open('gpurun_out/ab_${b}_${rep}.log').read().strip().splitlines()[-1])
print('batch $b rep $rep', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['checks']['reads_decoded'])"
  done
done

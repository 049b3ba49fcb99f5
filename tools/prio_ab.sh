#!/bin/bash
# A/B of the field-chain stream priority (LDG_PRIO), interleaved
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for p in 0 1; do
    LDG_PRIO=$p timeout -k 10 200 python bench.py --no-cpu --steps 3 > gpurun_out/pab_${p}_${rep}.log 2>&1 || exit 1
    python -c "
import json;d=json.loads(open('gpurun_out/pab_${p}_${rep}.log').read().strip().splitlines()[-1])
print('prio $p rep $rep', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done

#!/bin/bash
# A/B of the number of field-chain sub-streams (LDG_DECODE_STREAMS), interleaved
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in ${REPS_AB:-1 2}; do
  for ns in ${NSTREAMS:-2 4 8}; do
    LDG_DECODE_STREAMS=$ns timeout -k 10 200 python bench.py --no-cpu --steps 3 > gpurun_out/sab_${ns}_${rep}.log 2>&1 || exit 1
    python -c "
import json;d=json.loads(open('gpurun_out/sab_${ns}_${rep}.log').read().strip().splitlines()[-1])
print('streams $ns rep $rep', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done

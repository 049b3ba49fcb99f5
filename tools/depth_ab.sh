#!/bin/bash
# A/B of the pipeline depth (LDG_DEPTH), interleaved so that box-level drift hits both
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for d in ${DEPTHS:-2 3}; do
    LDG_DEPTH=$d timeout -k 10 200 python bench.py --no-cpu --steps 3 > gpurun_out/dab_${d}_${rep}.log 2>&1 || exit 1
    python -c "
import json;d=json.loads(open('gpurun_out/dab_${d}_${rep}.log').read().strip().splitlines()[-1])
print('depth $d rep $rep', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['checks']['reads_decoded'], d['checks']['host_s'])"
  done
done

#!/bin/bash
# LDG_DEPTH A/B of the default bench, interleaved on one box: tools/depth_ab.sh TAG STEPS D1 D2 ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=$1; STEPS=$2; shift 2
for rep in 1 2; do
  for d in "$@"; do
    LDG_DEPTH=$d timeout -k 10 300 python bench.py --steps $STEPS --warmup 3 --no-cpu > gpurun_out/${TAG}_d${d}_r${rep}.json 2> gpurun_out/${TAG}_d${d}_r${rep}.err || exit 1
    python -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_d${d}_r${rep}.json').read().strip().splitlines()[-1]); print('depth $d rep $rep', d['value'], d['ms_per_step'], max(d['checks']['step_ms']))" >> gpurun_out/${TAG}_summary.txt
  done
done

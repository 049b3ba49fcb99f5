#!/bin/bash
# interleaved A/B of the planner's wide bootstrap (LDG_BOOT_WIDE) on the 60 s bench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in $(seq 1 ${1:-3}); do
  for b in 0 1; do
    echo -n "boot_wide=$b "
    LDG_BOOT_WIDE=$b timeout -k 10 200 python3 bench.py --no-cpu --steps 3 > gpurun_out/bw.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/bw.json').read().splitlines()[-1]);c=d['checks'];print(d['value'],d['ms_per_step'],c['reads_decoded'],c['batches'])"
  done
done

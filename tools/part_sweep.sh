#!/bin/bash
# CU partition sweep (LDG_CHAIN_CUS = CUs per XCD for the non-demod streams):
# steady-state launch period (stage_trace) and the 60 s bench per setting.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for k in ${PARTS:-0 4 6 8}; do
  echo -n "chain_cus=$k stage_trace: "
  LDG_CHAIN_CUS=$k BATCH=96 LDG_DEPTH=3 LDG_STAGES=7 REPS=20 timeout -k 10 60 python3 tools/stage_trace.py 2>&1 | tail -1
  echo -n "chain_cus=$k bench: "
  LDG_CHAIN_CUS=$k timeout -k 10 200 python3 bench.py --no-cpu --steps 3 > gpurun_out/part_$k.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/part_$k.json').read().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"
done

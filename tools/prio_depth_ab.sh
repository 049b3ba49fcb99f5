#!/bin/bash
# Interleaved A/B with two demod streams: field-chain stream priority (LDG_PRIO) x pipeline depth (LDG_DEPTH)
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python bench.py --no-cpu > /dev/null 2>&1
for i in 1 2 3; do
  for cfg in "0 3" "1 3" "0 4" "1 4"; do
    set -- $cfg
    echo -n "prio $1 depth $2: "; LDG_PRIO=$1 LDG_DEPTH=$2 timeout -k 10 200 python bench.py --no-cpu 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['demod_busy_ms_per_launch'])"
  done
done

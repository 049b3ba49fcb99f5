#!/bin/bash
# Interleaved A/B of pipeline depth (LDG_DEPTH) x launch batch on the 60 s bench (two demod streams)
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  for cfg in "3 96" "4 96" "3 128" "4 128" "3 64"; do
    set -- $cfg
    echo -n "depth $1 batch $2: "; LDG_DEPTH=$1 timeout -k 10 200 python bench.py --no-cpu --batch $2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['demod_busy_ms_per_launch'])"
  done
done

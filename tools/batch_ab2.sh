#!/bin/bash
# Interleaved A/B of the launch batch (depth 3, two demod streams), after one discarded run
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python bench.py --no-cpu > /dev/null 2>&1
for i in 1 2 3; do
  for b in 96 128 160; do
    echo -n "batch $b: "; timeout -k 10 200 python bench.py --no-cpu --batch $b 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['demod_busy_ms_per_launch'])"
  done
done

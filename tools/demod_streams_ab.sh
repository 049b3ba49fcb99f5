#!/bin/bash
# Interleaved A/B of one vs two demod streams (LDG_DEMOD_STREAMS): pipeline period and the 60 s bench
cd "$GRAFT_REPO_ROOT"
for i in 1 2 3; do
  for d in 1 2; do
    echo -n "streams $d: "; LDG_DEMOD_STREAMS=$d REPS=30 BATCH=96 LDG_DEPTH=3 timeout -k 10 60 python tools/stage_trace.py 2>&1 | tail -1
  done
done
for i in 1 2; do
  for d in 1 2; do
    echo -n "bench streams $d: "; LDG_DEMOD_STREAMS=$d timeout -k 10 200 python bench.py --no-cpu 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done

#!/bin/bash
# A/B: demod as one launch per call vs group by group (LDG_DEMOD_SPLIT), interleaved
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  for sp in 0 1; do
    echo -n "split $sp: "
    LDG_DEMOD_SPLIT=$sp REPS=30 timeout -k 10 60 python3 tools/stage_trace.py > gpurun_out/split_one.log 2>&1 || { cat gpurun_out/split_one.log; exit 1; }
    tail -1 gpurun_out/split_one.log
  done
done
for rep in 1 2; do
  for sp in 0 1; do
    LDG_DEMOD_SPLIT=$sp timeout -k 10 200 python bench.py --no-cpu > gpurun_out/split_b.log 2>&1 || exit 1
    python -c "
import json;d=json.loads(open('gpurun_out/split_b.log').read().strip().splitlines()[-1])
print('bench split $sp', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done

#!/bin/bash
# Interleaved A/B: wait for the launch holding the missed read (LDG_MISS_DRAIN=1) or not (0)
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python bench.py --no-cpu > /dev/null 2>&1
for i in 1 2 3; do
  for d in 1 0; do
    echo -n "drain $d: "; LDG_MISS_DRAIN=$d timeout -k 10 200 python bench.py --no-cpu 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['checks']; print(d['value'], d['ms_per_step'], d['roofline']['demod_busy_ms_per_launch'], c['drain_waits'], c['misses'], c['batches'], c['reads_decoded'])"
  done
done
LDG_MISS_DRAIN=0 LDG_SPANDUMP=gpurun_out/s54_spans.txt timeout -k 10 200 python bench.py --no-cpu > /dev/null 2>&1 && python tools/span_gaps.py gpurun_out/s54_spans.txt

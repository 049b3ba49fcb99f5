#!/bin/bash
# Interleaved A/B: the next launch planned before the wait (LDG_PREPLAN=1) or after it (0)
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python bench.py --no-cpu > /dev/null 2>&1
for i in 1 2 3; do
  for d in 1 0; do
    echo -n "preplan $d: "; LDG_PREPLAN=$d timeout -k 10 200 python bench.py --no-cpu 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['checks']; print(d['value'], d['ms_per_step'], d['roofline']['demod_busy_ms_per_launch'], c['misses'], c['batches'], c['reads_decoded'], c['reads_used'])"
  done
done
LDG_HOSTTRACE=gpurun_out/s57_host.txt LDG_SPANDUMP=gpurun_out/s57_spans.txt timeout -k 10 200 python bench.py --no-cpu > /dev/null 2>&1 && python tools/span_gaps.py gpurun_out/s57_spans.txt

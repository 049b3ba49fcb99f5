#!/bin/bash
# Interleaved A/B of the field-chain sub-stream count (LDG_DECODE_STREAMS) with two demod streams
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python bench.py --no-cpu > /dev/null 2>&1
for i in 1 2 3; do
  for n in 2 3 4; do
    echo -n "chain streams $n: "; LDG_DECODE_STREAMS=$n timeout -k 10 200 python bench.py --no-cpu 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['demod_busy_ms_per_launch'])"
  done
done

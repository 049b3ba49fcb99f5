#!/bin/bash
# Interleaved bench A/B over pipeline settings (run through gpurun):
#   tools/pipe_ab.sh REPS "ENV_A [--batch B]" "ENV_B" ...
#   e.g. tools/pipe_ab.sh 2 "LDG_DEPTH=2" "LDG_DEPTH=3 --batch 128"
# Words with '=' are environment settings, the rest bench.py arguments.
# Prints one line per run: the settings, value (RF MS/s), ms/step, demod avg launch ms, reads decoded.
set -e
REPS=$1; shift
for i in $(seq 1 $REPS); do
  for cfg in "$@"; do
    envs=(); args=()
    for w in $cfg; do case $w in *=*) envs+=("$w");; *) args+=("$w");; esac; done
    out=$(env "${envs[@]}" timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu "${args[@]}" 2>/dev/null | tail -1)
    echo "$cfg | $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["checks"]["reads_decoded"])')"
  done
done

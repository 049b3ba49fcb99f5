#!/bin/bash
# Interleaved steady-state launch periods of the decode pipeline per stage set, for
# whole trees (run through gpurun from the repo root):  TREES=". abtree" tools/stage_ab.sh REPS
set -e
REPS=$1
root=$(pwd)
for i in $(seq 1 $REPS); do
  for st in 1 3 5 7; do
    for t in $TREES; do
      out=$(cd "$root/$t" && LDG_STAGES=$st LDG_DEPTH=3 BATCH=96 REPS=30 timeout -k 10 120 python3 tools/stage_trace.py 2>&1 | tail -1)
      echo "$t stages=$st $out"
    done
  done
done

#!/bin/bash
# Interleaved A/B of whole source trees (host code + library) on one box:
#   TREES=". abtree" tools/tree_ab.sh REPS BENCH-ARGS...
# Each tree must hold its own built libldgpu.so. Prints one line per run:
# "<tree> <value> <ms_per_step>".
set -e
REPS=$1; shift
root=$(pwd)
for i in $(seq 1 $REPS); do
  for t in $TREES; do
    out=$(cd "$root/$t" && timeout -k 10 300 python bench.py "$@" 2>/dev/null | tail -1)
    echo "$t $(python -c "import json,sys; d=json.loads(sys.argv[1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" "$out")"
  done
done

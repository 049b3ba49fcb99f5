#!/bin/bash
# Interleaved A/B of whole source trees, printing each run's host-side phases:
#   TREES=". abtree" tools/tree_phases.sh REPS BENCH-ARGS...
# One line per run: "<tree> <value> <ms_per_step> <checks.phase_s> <checks.host_s>".
set -e
REPS=$1; shift
root=$(pwd)
for i in $(seq 1 $REPS); do
  for t in $TREES; do
    out=$(cd "$root/$t" && timeout -k 10 300 python bench.py "$@" 2>/dev/null | tail -1)
    echo "$t $(python -c "import json,sys; d=json.loads(sys.argv[1]); c=d['checks']; print(d['value'], d['ms_per_step'], json.dumps(c.get('phase_s')), json.dumps(c.get('host_s')))" "$out")"
  done
done

#!/bin/bash
# Interleaved A/B of an environment setting on one box (run through gpurun):
#   tools/env_ab.sh REPS "A_ENV" "B_ENV" CMD...   e.g.
#   tools/env_ab.sh 3 LDG_COMB_3K=1 LDG_COMB_3K=0 python bench.py --steps 10 --warmup 3 --no-cpu
# Each run's last output line is printed prefixed with its setting.
set -e
REPS=$1; A=$2; B=$3; shift 3
for i in $(seq 1 $REPS); do
  for e in "$A" "$B"; do
    out=$(env $e timeout -k 10 300 "$@" 2>&1 | tail -1)
    echo "$e $out"
  done
done

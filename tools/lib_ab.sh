#!/bin/bash
# Interleaved A/B of library builds under this tree's host code (LDGPU_LIB):
#   LIBS="a.so b.so" tools/lib_ab.sh REPS BENCH-ARGS...
# One line per run: "<lib> <RF MS/s> <ms/step> <isolated demod ms per launch>".
set -e
REPS=$1; shift
for i in $(seq 1 $REPS); do
  for lib in $LIBS; do
    out=$(LDGPU_LIB=$lib timeout -k 10 300 python bench.py "$@" 2>/dev/null | tail -1)
    echo "$(basename $lib) $(python -c "import json,sys; d=json.loads(sys.argv[1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" "$out")"
  done
done

#!/bin/bash
# Interleaved A/B/... of builds of libldgpu on one box (run through gpurun):
#   LIBS="a.so b.so" tools/ab_lib.sh REPS CMD...   e.g.
#   LIBS="ld-decode_amd/ldgpu/libldgpu_base.so ld-decode_amd/ldgpu/libldgpu.so" \
#       tools/ab_lib.sh 3 env LDG_STAGES=1 BATCH=96 python tools/stage_trace.py
# Each run's last output line is printed prefixed with the library's basename.
set -e
REPS=$1; shift
for i in $(seq 1 $REPS); do
  for lib in $LIBS; do
    out=$(LDGPU_LIB=$lib timeout -k 10 300 "$@" 2>&1 | tail -1)
    echo "$(basename $lib) $out"
  done
done

#!/bin/bash
# Interleaved A/B of two builds of libldgpu on one box (run through gpurun):
#   tools/ab_lib.sh LIB_A LIB_B REPS CMD...   e.g.  tools/ab_lib.sh ld-decode_amd/ldgpu/libldgpu_base.so \
#       ld-decode_amd/ldgpu/libldgpu.so 3 env LDG_STAGES=1 BATCH=96 python tools/stage_trace.py
# Each run's output line is prefixed with A or B.
set -e
A=$1; B=$2; REPS=$3; shift 3
for i in $(seq 1 $REPS); do
  for tag in A B; do
    lib=$A; [ $tag = B ] && lib=$B
    out=$(LDGPU_LIB=$lib timeout -k 10 300 "$@" 2>&1 | tail -1)
    echo "$tag $out"
  done
done

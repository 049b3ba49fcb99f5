#!/bin/bash
# A/B of library builds: field chains alone (tools/chain_alone.py, stages 4 wall)
# and the steady-state pipeline period (tools/stage_trace.py, everything).
#   LIBS="a.so b.so" tools/chain_ab.sh REPS
cd "$GRAFT_REPO_ROOT"
for i in $(seq 1 ${1:-2}); do
  for lib in $LIBS; do
    a=$(LDGPU_LIB=$lib BATCH=96 REPS=10 timeout -k 10 120 python3 tools/chain_alone.py 2>&1 | grep "stages 4" || echo fail)
    b=$(LDGPU_LIB=$lib BATCH=96 LDG_DEPTH=3 LDG_STAGES=7 REPS=20 timeout -k 10 120 python3 tools/stage_trace.py 2>&1 | tail -1)
    echo "$(basename $lib) | $a | $b"
  done
done

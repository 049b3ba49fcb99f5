#!/bin/bash
# steady-state launch period of tools/stage_trace.py per pipeline depth and LDG_STAGES (no profiler)
cd "$GRAFT_REPO_ROOT"
for d in 2 3; do
  for st in 1 3 5 7; do
    REPS=30 LDG_DEPTH=$d LDG_STAGES=$st timeout -k 10 60 python3 tools/stage_trace.py || exit 1
  done
done

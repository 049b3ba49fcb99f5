#!/bin/bash
# steady-state launch period of tools/stage_trace.py per stream-priority setting (LDG_PRIO)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {
  echo -n "$1: "
  shift
  env "$@" REPS=30 timeout -k 10 60 python3 tools/stage_trace.py > gpurun_out/cu_sweep_one.log 2>&1
  rc=$?
  tail -3 gpurun_out/cu_sweep_one.log
  [ $rc -eq 0 ] || { echo "rc $rc"; exit 1; }
}
for p in 0 1 2; do
  for st in 5 7; do
    run "prio $p" LDG_PRIO=$p LDG_STAGES=$st
  done
done

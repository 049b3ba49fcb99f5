#!/bin/bash
# marginal cost of each field-chain kernel: steady-state launch period with it not
# launched (LDG_SKIP bit; downstream results are garbage -- timing probe only)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {
  echo -n "$1: "
  shift
  env "$@" REPS=30 timeout -k 10 60 python3 tools/stage_trace.py > gpurun_out/skip_one.log 2>&1
  rc=$?
  tail -1 gpurun_out/skip_one.log
  [ $rc -eq 0 ] || { echo "rc $rc"; exit 1; }
}
run "demod only" LDG_STAGES=1
run "demod+audio" LDG_STAGES=3
run "demod+fields" LDG_STAGES=5
run "all" LDG_STAGES=7
i=0
for k in sync_walk sync linelocs hsync_lines hsync_field philips burst_lines burst_field final_lines; do
  run "skip $k" LDG_STAGES=7 LDG_SKIP=$((1 << i))
  i=$((i+1))
done
run "skip all but sync_walk+sync" LDG_STAGES=7 LDG_SKIP=$((511 - 3))

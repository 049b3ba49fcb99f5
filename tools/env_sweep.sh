#!/bin/bash
# Interleaved bench runs per environment setting ("-" = none; settings joined by ","):
#   tools/env_sweep.sh REPS "- LDG_DEPTH=4 LDG_PRIO=1,LDG_DEPTH=4" BENCH-ARGS...
set -e
REPS=$1; SETS=$2; shift 2
for i in $(seq 1 $REPS); do
  for e in $SETS; do
    envs=(); [ "$e" != "-" ] && IFS=, read -ra envs <<< "$e"
    mkdir -p gpurun_out
    out=$(env "${envs[@]}" timeout -k 10 600 python bench.py "$@" 2>>gpurun_out/env_sweep.err | tail -1)
    echo "$e $(python -c "import json,sys; d=json.loads(sys.argv[1]); c=d.get('checks', {}); i = c.get('demod_issue') or {}; print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], c.get('reads_decoded'), c.get('vcut_redo'), 'host_late', i.get('host_late'), 'idle_ms', i.get('idle_ms'))" "$out")"
  done
done

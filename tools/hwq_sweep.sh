#!/bin/bash
# Interleaved sweep of the HIP runtime's hardware queues per process (GPU_MAX_HW_QUEUES,
# HIP's default 4) on one box, through gpurun:
#   tools/hwq_sweep.sh TAG REPS "Q1 Q2 ..." BENCH_ARGS...
# One line per run: queues, RF MS/s, ms per step, host-late demod launches.
set -e
TAG=$1; REPS=$2; QS=$3; shift 3
mkdir -p gpurun_out
for i in $(seq 1 $REPS); do
  for q in $QS; do
    f=gpurun_out/${TAG}_q${q}_r${i}.json
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py "$@" > $f 2> ${f%.json}.err
    python -c "
import json; d = json.load(open('$f')); c = d['checks']; i = c.get('demod_issue') or {}
print('queues $q rep $i', d['value'], d['ms_per_step'], 'host_late', i.get('host_late'), '/', i.get('launches'), 'idle_ms', i.get('idle_ms'))
" | tee -a gpurun_out/${TAG}_summary.txt
  done
done

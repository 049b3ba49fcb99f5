#!/bin/bash
# Interleaved same-box A/B of two environment settings on the 60 s bench (STEPS steps each):
#   bash tools/envab.sh TAG PAIRS STEPS "A_ENV" "B_ENV" [bench args]
TAG=$1; PAIRS=$2; STEPS=$3; A=$4; B=$5; shift 5
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in $(seq 1 $PAIRS); do
  for v in A B; do
    if [ $v = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 300 python bench.py --steps $STEPS --warmup 2 --no-cpu "$@" > gpurun_out/${TAG}_${v}${i}.json 2> gpurun_out/${TAG}_${v}${i}.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_${v}${i}.json')); c=d['checks']; print('$v$i %8.3f ms/step %9.1f MS/s reads %d batches %d idle_ms %.1f' % (d['ms_per_step'], d['value'], c['reads_decoded'], c['batches'], c['demod_issue']['idle_ms'] if c['demod_issue'] else -1))" >> gpurun_out/${TAG}_summary.txt
  done
done
cat gpurun_out/${TAG}_summary.txt

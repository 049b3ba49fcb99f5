#!/bin/bash
# GPU-box profiling recipe (run through gpurun from the repo root):
#   1. kernel trace + stats of a bench run           -> gpurun_out/prof/<tag>/trace
#   2. PMC passes (no trace domains), one per group  -> gpurun_out/prof/<tag>/pmcN
# usage: tools/profile.sh TAG "BENCH ARGS" [pmc groups...]
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
ARGS=$1; shift
OUT=gpurun_out/prof/$TAG
mkdir -p $OUT
if [ "$1" = notrace ]; then
  shift
else
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
fi
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py $ARGS > $OUT/pmc$i.log 2>&1
done
echo done

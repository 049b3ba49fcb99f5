#!/bin/bash
# Marginal step cost of stages: the 60 s bench (5 steps) with one stage left out
# (timing probes only: a skipped kernel's outputs are garbage).  usage: bash tools/marginal.sh TAG
TAG=${1:-marg}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu $EXTRA > gpurun_out/${TAG}_${name}.json 2> gpurun_out/${TAG}_${name}.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_${name}.json')); print('%-12s %8.3f ms/step %9.1f MS/s' % ('$name', d['ms_per_step'], d['value']))" >> gpurun_out/${TAG}_summary.txt
}
run base
EXTRA=--no-comb run nocomb
run nofinal LDG_SKIP=256
run noaudio2 LDG_STAGES=5
run base2
cat gpurun_out/${TAG}_summary.txt

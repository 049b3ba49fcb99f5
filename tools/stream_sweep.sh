#!/bin/bash
# bench.py under several decode sub-stream settings (LDG_DECODE_STREAMS / LDG_SPLIT_DEMOD)
set -e
mkdir -p gpurun_out
SECS=${SECS:-20}
for cfg in "1 1" "2 1" "4 1" "4 0" "8 1"; do
  set -- $cfg
  LDG_DECODE_STREAMS=$1 LDG_SPLIT_DEMOD=$2 timeout -k 10 300 python bench.py --seconds $SECS --steps 2 --warmup 1 --no-cpu \
    > gpurun_out/sweep_$1_$2.json 2> gpurun_out/sweep_$1_$2.err
  echo "streams=$1 split=$2 $(python -c "import json,sys;d=json.loads(open('gpurun_out/sweep_$1_$2.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'])")"
done

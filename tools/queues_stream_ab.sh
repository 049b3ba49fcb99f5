#!/bin/bash
# A/B: hardware queues 12 (the default raise) vs 16 for the streamed-from-file bench
# (the context's ten streams plus the stream's four copy streams) and the resident bench.
#   bash tools/queues_stream_ab.sh TAG
set -e
TAG=${1:-qab}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  for q in 12 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu \
        --stream-file /tmp/ldg_cap60.u8 > gpurun_out/${TAG}_stream_q${q}_${rep}.json 2> /dev/null
  done
done
for q in 12 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu \
      > gpurun_out/${TAG}_resident_q${q}.json 2> /dev/null
done
rm -f /tmp/ldg_cap60.u8

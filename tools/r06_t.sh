#!/bin/bash
# Streamed-from-file bench A/B (round 6): the copy-stream count, then the default.
#   bash tools/r06_t.sh TAG "1 2 4"
set -e
TAG=${1:-r06_t}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for c in ${2:-1 2 4}; do
  LDG_STREAM_COPIES=$c timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --stream-file /tmp/ldg_cap60.u8 \
      > gpurun_out/${TAG}_stream_c$c.json 2> gpurun_out/${TAG}_stream_c$c.err
done
rm -f /tmp/ldg_cap60.u8

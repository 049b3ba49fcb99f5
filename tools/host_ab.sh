#!/bin/bash
# Same-box A/B of a host-side (Python) change: abtmp/ holds the previous commit's
# bench.py and ldgpu package (git archive), run against the same libldgpu.so.
#   bash tools/host_ab.sh TAG
set -e
TAG=${1:-hab}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export LDG_SYNTH_CACHE=/tmp/ldg_synth
LIB=$GRAFT_REPO_ROOT/ld-decode_amd/ldgpu/libldgpu.so
for rep in 1 2; do
  for v in new old; do
    B=bench.py; [ $v = old ] && B=abtmp/bench.py
    LDGPU_LIB=$LIB timeout -k 10 300 python $B --steps 10 --warmup 2 --no-cpu > gpurun_out/${TAG}_ntsc_${v}_${rep}.json 2> /dev/null
    LDGPU_LIB=$LIB timeout -k 10 400 python $B --system PAL --steps 10 --warmup 2 --no-cpu > gpurun_out/${TAG}_pal_${v}_${rep}.json 2> gpurun_out/${TAG}_pal_${v}_${rep}.err
  done
done

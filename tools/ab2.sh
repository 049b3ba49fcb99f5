#!/bin/bash
# Same-box A/B of two library builds on the 60 s bench: B = the tree's libldgpu.so,
# A = LIB_A (another build of the library, e.g. the previous commit's), interleaved
# pairs of STEPS-step runs.  usage: LIB_A=path bash tools/ab2.sh TAG [pairs] [steps]
TAG=${1:-ab}; PAIRS=${2:-3}; STEPS=${3:-10}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in $(seq 1 $PAIRS); do
  for v in A B; do
    if [ $v = A ]; then L=$LIB_A; else L=ld-decode_amd/ldgpu/libldgpu.so; fi
    LDGPU_LIB=$L timeout -k 10 300 python bench.py --steps $STEPS --warmup 2 --no-cpu > gpurun_out/${TAG}_${v}${i}.json 2> gpurun_out/${TAG}_${v}${i}.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_${v}${i}.json')); print('$v$i %8.3f ms/step %9.1f MS/s iso %.4f' % (d['ms_per_step'], d['value'], d['roofline']['avg_launch_ms']))" >> gpurun_out/${TAG}_summary.txt
  done
done
cat gpurun_out/${TAG}_summary.txt

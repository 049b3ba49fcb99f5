set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=ld-decode_amd/ldgpu
LIBS="$L/libldgpu_base.so $L/libldgpu_skew5.so $L/libldgpu_skew10.so" bash tools/ab_lib.sh 3 env LDG_STAGES=1 BATCH=96 python tools/stage_trace.py > gpurun_out/s87_stage.txt 2>&1
LIBS="$L/libldgpu_base.so $L/libldgpu_skew5.so $L/libldgpu_skew10.so" bash tools/ab_lib.sh 3 python bench.py --no-cpu > gpurun_out/s87_bench.txt 2>&1

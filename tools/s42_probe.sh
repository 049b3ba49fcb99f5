set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python tools/demod_stamps.py > gpurun_out/s42_stamps.txt 2>&1
L=ld-decode_amd/ldgpu
LIBS="$L/libldgpu_base.so $L/libldgpu.so $L/libldgpu_t1.so" bash tools/ab_lib.sh 3 env REPS=30 BATCH=96 LDG_DEPTH=3 LDG_STAGES=1 python tools/stage_trace.py > gpurun_out/s42_ab.txt 2>&1
LIBS="$L/libldgpu_base.so $L/libldgpu.so $L/libldgpu_t1.so" bash tools/ab_lib.sh 2 env REPS=30 BATCH=96 LDG_DEPTH=3 python tools/stage_trace.py >> gpurun_out/s42_ab.txt 2>&1

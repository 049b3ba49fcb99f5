set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s43_tests.txt 2>&1
L=ld-decode_amd/ldgpu
LIBS="$L/libldgpu_base.so $L/libldgpu.so" bash tools/ab_lib.sh 3 env REPS=30 BATCH=96 LDG_DEPTH=3 LDG_STAGES=3 python tools/stage_trace.py > gpurun_out/s43_ab.txt 2>&1
LIBS="$L/libldgpu_base.so $L/libldgpu.so" bash tools/ab_lib.sh 3 env REPS=30 BATCH=96 LDG_DEPTH=3 python tools/stage_trace.py >> gpurun_out/s43_ab.txt 2>&1

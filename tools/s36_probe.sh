set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s36_tests.txt 2>&1
LIBS="ld-decode_amd/ldgpu/libldgpu_base.so ld-decode_amd/ldgpu/libldgpu.so" bash tools/ab_lib.sh 3 env REPS=30 BATCH=96 LDG_DEPTH=3 python tools/stage_trace.py > gpurun_out/s36_ab.txt 2>&1
LIBS="ld-decode_amd/ldgpu/libldgpu_base.so ld-decode_amd/ldgpu/libldgpu.so" bash tools/ab_lib.sh 1 env BATCH=96 REPS=10 python tools/chain_alone.py > gpurun_out/s36_alone.txt 2>&1 || true

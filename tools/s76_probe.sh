set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s76_tests.txt 2>&1
L=ld-decode_amd/ldgpu
LIBS="$L/libldgpu_base.so $L/libldgpu.so" bash tools/ab_lib.sh 3 env LDG_STAGES=1 BATCH=96 python tools/stage_trace.py > gpurun_out/s76_stage.txt 2>&1
LIBS="$L/libldgpu_base.so $L/libldgpu.so" bash tools/ab_lib.sh 3 python bench.py --no-cpu > gpurun_out/s76_bench.txt 2>&1

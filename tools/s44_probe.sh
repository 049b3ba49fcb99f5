set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s44_tests.txt 2>&1
L=ld-decode_amd/ldgpu
LIBS="$L/libldgpu_base.so $L/libldgpu_w5.so $L/libldgpu.so" bash tools/ab_lib.sh 3 env REPS=30 BATCH=96 LDG_DEPTH=3 python tools/stage_trace.py > gpurun_out/s44_ab.txt 2>&1
for lib in libldgpu_base.so libldgpu.so; do echo "== $lib" >> gpurun_out/s44_alone.txt; LDGPU_LIB=$L/$lib BATCH=96 REPS=10 timeout -k 10 120 python tools/chain_alone.py >> gpurun_out/s44_alone.txt 2>&1; done

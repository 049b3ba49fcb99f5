set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s89_tests.txt 2>&1
L=ld-decode_amd/ldgpu
LIBS="$L/libldgpu_base.so $L/libldgpu.so" bash tools/ab_lib.sh 4 python bench.py --no-cpu > gpurun_out/s89_bench.txt 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/s89_bench20.json 2> /dev/null

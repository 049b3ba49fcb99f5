set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_comb.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s71_tests.txt 2>&1
LIBS="ld-decode_amd/ldgpu/libldgpu_base.so ld-decode_amd/ldgpu/libldgpu.so" bash tools/ab_lib.sh 3 python bench.py --no-cpu > gpurun_out/s71_ab.txt 2>&1

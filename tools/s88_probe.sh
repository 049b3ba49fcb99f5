set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=ld-decode_amd/ldgpu
LIBS="$L/libldgpu_base.so $L/libldgpu_skew10.so $L/libldgpu_skew15.so" bash tools/ab_lib.sh 4 python bench.py --no-cpu > gpurun_out/s88_bench.txt 2>&1

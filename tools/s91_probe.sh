set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=ld-decode_amd/ldgpu
LIBS="$L/libldgpu_noilp.so $L/libldgpu.so" bash tools/ab_lib.sh 3 python bench.py --no-cpu --steps 20 --warmup 5 > gpurun_out/s91_bench.txt 2>&1

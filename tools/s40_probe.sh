set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in p2048 p4096; do
  sed "s|libldgpu_stamps.so|libldgpu_stamps_$v.so|" tools/demod_stamps.py > tools/_ds_$v.py
  timeout -k 10 120 python tools/_ds_$v.py > gpurun_out/s40_stamps_$v.txt 2>&1
done
L=ld-decode_amd/ldgpu
LIBS="$L/libldgpu_base.so $L/libldgpu_p2048.so $L/libldgpu_p4096.so" bash tools/ab_lib.sh 2 env REPS=30 BATCH=96 LDG_DEPTH=3 LDG_STAGES=1 python tools/stage_trace.py > gpurun_out/s40_ab.txt 2>&1
LIBS="$L/libldgpu_base.so $L/libldgpu_p2048.so $L/libldgpu_p4096.so" bash tools/ab_lib.sh 2 env REPS=30 BATCH=96 LDG_DEPTH=3 python tools/stage_trace.py >> gpurun_out/s40_ab.txt 2>&1

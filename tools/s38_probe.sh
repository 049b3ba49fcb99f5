set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python tools/demod_stamps.py > gpurun_out/s38_stamps.txt 2>&1
sed -i 's|libldgpu_stamps.so|libldgpu_stamps_ns.so|' tools/demod_stamps.py
timeout -k 10 120 python tools/demod_stamps.py > gpurun_out/s38_stamps_nostore.txt 2>&1

set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in p256 p512 p1024; do
  sed "s|libldgpu_stamps.so|libldgpu_stamps_$v.so|" tools/demod_stamps.py > /tmp/ds_$v.py
  cp /tmp/ds_$v.py tools/_ds_$v.py
  timeout -k 10 120 python tools/_ds_$v.py > gpurun_out/s39_stamps_$v.txt 2>&1
done

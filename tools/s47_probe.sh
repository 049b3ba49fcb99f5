cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python tools/long_probe.py 240 > gpurun_out/s47_cav240.txt 2>&1
timeout -k 10 120 python tools/long_probe.py 240 --clv > gpurun_out/s47_clv240.txt 2>&1

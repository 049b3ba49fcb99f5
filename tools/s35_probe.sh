set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
BATCH=96 LDG_DEPTH=3 bash tools/skip_sweep.sh > gpurun_out/s35_skip.txt 2>&1
BATCH=96 REPS=10 timeout -k 10 120 python tools/chain_alone.py > gpurun_out/s35_chain_alone.txt 2>&1

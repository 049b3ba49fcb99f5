set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s49_tests.txt 2>&1
bash tools/demod_streams_ab.sh > gpurun_out/s49_ab.txt 2>&1

set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_comb.py tests/test_cli.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s80_tests.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/s80/trace -o run -- python3 bench.py --no-cpu > gpurun_out/s80_trace.log 2>&1

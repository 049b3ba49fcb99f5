set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s94_tests.txt 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s94_smoke.txt 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/s94_bench20.json 2> /dev/null

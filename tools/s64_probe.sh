set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s64_tests.txt 2>&1
timeout -k 10 300 python tools/pal_waste.py --seconds 4 > gpurun_out/s64_pal_waste.txt 2>&1
timeout -k 10 600 python tools/pal_bench.py --seconds 10 --steps 3 > gpurun_out/s64_pal.json 2> gpurun_out/s64_pal.err
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/s64_bench.json 2> /dev/null

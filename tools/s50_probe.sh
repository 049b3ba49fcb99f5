set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s50_tests.txt 2>&1
timeout -k 10 200 python bench.py > gpurun_out/s50_bench.json 2> gpurun_out/s50_bench.err
bash tools/profile.sh s50 "--no-cpu" "FETCH_SIZE" "WRITE_SIZE" > gpurun_out/s50_prof.log 2>&1

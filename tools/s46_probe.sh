set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s46_tests.txt 2>&1
# config C5's per-capture work on one GPU: a 1-hour CLV capture resident in HBM (144 GB u8)
timeout -k 10 500 python bench.py --seconds 3600 --clv --steps 1 --warmup 0 --no-cpu > gpurun_out/s46_bench_1h.json 2> gpurun_out/s46_bench_1h.err

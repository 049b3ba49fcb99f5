set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python tools/long_probe.py 240 > gpurun_out/s48_cav240.txt 2>&1
timeout -k 10 120 python tools/long_probe.py 240 --clv > gpurun_out/s48_clv240.txt 2>&1
timeout -k 10 200 python bench.py > gpurun_out/s48_bench.json 2> gpurun_out/s48_bench.err
timeout -k 10 500 python bench.py --seconds 3600 --clv --steps 1 --warmup 0 --no-cpu > gpurun_out/s48_bench_1h.json 2> gpurun_out/s48_bench_1h.err

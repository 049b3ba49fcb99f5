set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
# config C4: 10-bit packed captures (.r30 = ddpack, .lds), unpacked inside the demod
timeout -k 10 200 python bench.py --fmt 2 --no-cpu > gpurun_out/s45_bench_r30.json 2> gpurun_out/s45_bench_r30.err
timeout -k 10 200 python bench.py --fmt 3 --no-cpu > gpurun_out/s45_bench_lds.json 2> gpurun_out/s45_bench_lds.err
# config C5's per-capture work on one GPU: a 1-hour CLV capture resident in HBM (144 GB u8)
timeout -k 10 400 python bench.py --seconds 3600 --clv --steps 1 --warmup 0 --no-cpu > gpurun_out/s45_bench_1h.json 2> gpurun_out/s45_bench_1h.err

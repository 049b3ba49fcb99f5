set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s79_smoke.txt 2>&1
timeout -k 10 300 python bench.py > gpurun_out/s79_bench.json 2> gpurun_out/s79_bench.err
timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 5 > gpurun_out/s79_bench20.json 2> /dev/null
bash tools/profile.sh s79 "--no-cpu" "FETCH_SIZE" "WRITE_SIZE" > gpurun_out/s79_prof.log 2>&1

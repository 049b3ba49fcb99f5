set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s86_smoke.txt 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/s86_bench20.json 2> gpurun_out/s86_bench20.err
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/s86_bench.json 2> /dev/null
bash tools/profile.sh s86 "--no-cpu" "FETCH_SIZE" "WRITE_SIZE" > gpurun_out/s86_prof.log 2>&1

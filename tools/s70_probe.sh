set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s70_tests.txt 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s70_smoke.txt 2>&1
timeout -k 10 200 python bench.py > gpurun_out/s70_bench.json 2> gpurun_out/s70_bench.err
bash tools/profile.sh s70 "--no-cpu" "FETCH_SIZE" "WRITE_SIZE" > gpurun_out/s70_prof.log 2>&1
bash tools/demod_pmc.sh s70d > gpurun_out/s70_dpmc.log 2>&1

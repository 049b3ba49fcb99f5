set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s34_tests.txt 2>&1
timeout -k 10 200 python bench.py > gpurun_out/s34_bench.json 2> gpurun_out/s34_bench.err
for st in 1 3 5 7 1 3 5 7; do
  REPS=30 BATCH=96 LDG_DEPTH=3 LDG_STAGES=$st timeout -k 10 60 python3 tools/stage_trace.py >> gpurun_out/s34_stages.txt 2>&1
done

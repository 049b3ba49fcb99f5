set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2 3; do
  for b in 96 128 112; do
    echo -n "batch $b " >> gpurun_out/s93_batch.txt
    timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 5 --batch $b 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" >> gpurun_out/s93_batch.txt
  done
done

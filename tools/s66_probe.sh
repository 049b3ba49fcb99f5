set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for b in 48 96 64; do
  echo -n "batch $b: " >> gpurun_out/s66_pal_batch.txt
  timeout -k 10 400 python tools/pal_bench.py --seconds 10 --steps 3 --batch $b 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['realtime_x'], d['reads_decoded_total'], d['reads_used_total'], d['batches'])" >> gpurun_out/s66_pal_batch.txt
done

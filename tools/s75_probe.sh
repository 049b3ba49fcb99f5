set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2 3; do
  for b in 0 1; do
    echo -n "boot_now=$b " >> gpurun_out/s75_ab.txt
    LDG_BOOT_NOW=$b timeout -k 10 200 python bench.py --no-cpu 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['checks']['batches'], d['checks']['reads_decoded'])" >> gpurun_out/s75_ab.txt
  done
done
for i in 1 2; do
  for b in 0 1; do
    echo -n "PAL boot_now=$b " >> gpurun_out/s75_ab.txt
    LDG_BOOT_NOW=$b timeout -k 10 400 python tools/pal_bench.py --seconds 10 --steps 3 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['realtime_x'], d['reads_decoded_total'], d['reads_used_total'], d['batches'])" >> gpurun_out/s75_ab.txt
  done
done

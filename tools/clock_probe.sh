#!/bin/bash
# bench runs back to back with the GPU's clocks / power / temperature logged before each
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2 3 4; do
  timeout -k 5 20 rocm-smi --showclocks --showpower --showtemp > gpurun_out/smi_$rep.txt 2>&1
  grep -E "sclk|Power|Temperature \(Sensor junction\)|mclk" gpurun_out/smi_$rep.txt | head -6
  timeout -k 10 200 python bench.py --no-cpu --steps 3 > gpurun_out/clk_$rep.log 2>&1 || exit 1
  python -c "
import json;d=json.loads(open('gpurun_out/clk_$rep.log').read().strip().splitlines()[-1])
print('rep $rep', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done

#!/bin/bash
# Round-end extras on one GPU box (through gpurun), beside tools/final_check.sh:
#   the streamed-from-file bench (4 copy streams), the end-to-end CLI (tools/cli_e2e.sh),
#   and the N = 2 launch rehearsed on the one GPU (two ranks sharing it, gloo).
#   bash tools/final_extras.sh TAG
set -e
TAG=${1:-extras}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/r06_t.sh ${TAG} 4
bash tools/cli_e2e.sh ${TAG}
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --seconds 240 --no-cpu \
    > gpurun_out/${TAG}_bench_sharded_240s_2rank_1gpu.json 2> gpurun_out/${TAG}_bench_sharded_2rank.err
echo done

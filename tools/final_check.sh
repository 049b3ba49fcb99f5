#!/bin/bash
# Round-end validation on one GPU box: GPU tests, smoke, NTSC 20-step and PAL 10-step bench lines, then
# tools/profile.sh (kernel trace + SQ / FETCH / WRITE passes).  usage (via gpurun): bash tools/final_check.sh TAG
set -e
TAG=${1:-final}
export LDG_SYNTH_CACHE=/tmp/ldg_synth
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1
timeout -k 10 500 python bench.py --steps 20 --warmup 3 > gpurun_out/${TAG}_bench_60s_20steps.json 2> gpurun_out/${TAG}_bench.err
timeout -k 10 500 python bench.py --system PAL --steps 10 --warmup 2 > gpurun_out/${TAG}_pal_bench_10s.json 2> gpurun_out/${TAG}_pal.err
bash tools/profile.sh ${TAG} "--no-cpu --steps 5 --warmup 2" SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VALU,SQ_WAIT_INST_LDS SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_VALU,SQ_INSTS_VALU_FMA_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_ADD_F64,SQ_BUSY_CU_CYCLES,GRBM_GUI_ACTIVE,GRBM_COUNT SQ_INSTS_LDS_LOAD,SQ_INSTS_LDS_LOAD_BANDWIDTH,SQ_INSTS_LDS_STORE,SQ_INSTS_LDS_STORE_BANDWIDTH,SQ_LDS_ADDR_CONFLICT,SQ_LDS_DATA_FIFO_FULL,SQ_ACTIVE_INST_SCA,SQ_INSTS_SALU FETCH_SIZE WRITE_SIZE

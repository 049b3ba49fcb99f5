#!/bin/bash
# Round-end validation on one GPU box (run through gpurun), in two calls:
#   bash tools/final_check.sh TAG check    GPU tests, smoke, NTSC 20-step and PAL 10-step bench lines
#   bash tools/final_check.sh TAG profile  tools/profile.sh: kernel trace + SQ / FETCH / WRITE passes
# then, here: python tools/pmc_summary.py gpurun_out/prof/TAG profiles/TAG gpurun_out/prof/TAGsq...
# and copy profiles/TAG_pmc_traffic.json to profiles/pmc_traffic.json (bench.py attaches it
# only to a run of the library it was taken of: its source hash).
set -e
TAG=${1:-final}
WHAT=${2:-check}
export LDG_SYNTH_CACHE=/tmp/ldg_synth
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ "$WHAT" = check ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1
  timeout -k 10 500 python bench.py --steps 20 --warmup 3 > gpurun_out/${TAG}_bench_60s_20steps.json 2> gpurun_out/${TAG}_bench.err
  timeout -k 10 500 python bench.py --system PAL --steps 10 --warmup 2 --no-cpu > gpurun_out/${TAG}_pal_bench_10s.json 2> gpurun_out/${TAG}_pal.err
else
  bash tools/profile.sh ${TAG} "--no-cpu --steps 5 --warmup 2" SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VALU,SQ_WAIT_INST_LDS SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_VALU,SQ_INSTS_VALU_FMA_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_ADD_F64,SQ_BUSY_CU_CYCLES,GRBM_GUI_ACTIVE,GRBM_COUNT SQ_INSTS_LDS_LOAD,SQ_INSTS_LDS_LOAD_BANDWIDTH,SQ_INSTS_LDS_STORE,SQ_INSTS_LDS_STORE_BANDWIDTH,SQ_LDS_ADDR_CONFLICT,SQ_LDS_DATA_FIFO_FULL,SQ_ACTIVE_INST_SCA,SQ_INSTS_SALU FETCH_SIZE WRITE_SIZE
fi
echo done

#!/bin/bash
# Demod-only PMC passes (run through gpurun from the repo root): one rocprofv3
# --pmc pass per counter group over the demod-only decode loop of
# tools/stage_trace.py; summaries -> gpurun_out/prof/<tag>/pmcN
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=$1
OUT=gpurun_out/prof/$TAG
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_LDS_UNALIGNED_STALL SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  LDG_STAGES=1 BATCH=96 REPS=6 timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python3 tools/stage_trace.py > $OUT/pmc$i.log 2>&1
done
echo done

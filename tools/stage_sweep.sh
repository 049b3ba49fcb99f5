#!/bin/bash
# kernel traces of tools/stage_trace.py per LDG_STAGES value (default: 1 7)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/prof
for st in ${@:-1 7}; do
  LDG_STAGES=$st timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof/stg$st -o run -- python3 tools/stage_trace.py > gpurun_out/stg$st.log 2>&1 || exit 1
done
echo ok

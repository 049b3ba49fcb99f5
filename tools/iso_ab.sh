#!/bin/bash
# demod iso leg A/B of library variants on one box: tools/iso_ab.sh TAG LIB1 LIB2 ...
# (LIB "default": the in-tree libldgpu.so; "old": the same with LDG_DEMOD2=0)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1; shift
for rep in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = default ]; then timeout -k 10 120 python tools/demod_iso.py 20 >> gpurun_out/${TAG}_iso.txt 2>&1 || exit 1
    elif [ "$lib" = old ]; then LDG_DEMOD2=0 timeout -k 10 120 python tools/demod_iso.py 20 >> gpurun_out/${TAG}_iso.txt 2>&1 || exit 1
    else LDGPU_LIB=$lib timeout -k 10 120 python tools/demod_iso.py 20 | sed "s#^#$lib #" >> gpurun_out/${TAG}_iso.txt 2>&1 || exit 1
    fi
  done
done

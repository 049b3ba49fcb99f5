#!/bin/bash
# End-to-end lddecode.py timing on the GPU box (file -> .tbc/.pcm/.json, and with --comb):
# a 60 s NTSC CAV u8 capture written to local storage, then the CLI run on it with
# --stats-json (read / decode / write breakdown).  usage (via gpurun): bash tools/cli_e2e.sh TAG
set -e
TAG=${1:-e2e}
cd "$GRAFT_REPO_ROOT"
D=/tmp/ldg_e2e
mkdir -p $D gpurun_out
timeout -k 10 120 python tools/make_capture_file.py $D/cap60.u8 60 > gpurun_out/${TAG}_make.txt 2>&1
lscpu > gpurun_out/${TAG}_lscpu.txt 2>&1 || true
df -h /tmp >> gpurun_out/${TAG}_lscpu.txt 2>&1 || true
run() {   # name, extra args
  local name=$1; shift
  /usr/bin/time -v timeout -k 10 300 python ld-decode_amd/lddecode.py --stats-json gpurun_out/${TAG}_${name}_stats.json "$@" \
      $D/cap60.u8 $D/out_$name > $D/${name}.stdout 2> gpurun_out/${TAG}_${name}.err
  ls -l $D/out_$name.* >> gpurun_out/${TAG}_${name}.err
  tail -2 $D/${name}.stdout >> gpurun_out/${TAG}_${name}.err
}
run stream
run stream_comb --comb
run whole --window-mb 0
cmp $D/out_stream.tbc $D/out_whole.tbc && cmp $D/out_stream.pcm $D/out_whole.pcm && cmp $D/out_stream.json $D/out_whole.json \
  && echo "stream == whole: identical .tbc .pcm .json" > gpurun_out/${TAG}_cmp.txt
rm -rf $D
echo done

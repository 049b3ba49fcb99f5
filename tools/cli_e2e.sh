#!/bin/bash
# End-to-end lddecode.py timing on the GPU box (file -> .tbc/.pcm/.json, and with --comb):
# a 60 s NTSC CAV u8 capture written to local storage, then the CLI run on it with
# --stats-json (read / decode / write breakdown).  "cold": the capture's pages dropped from
# the page cache first (posix_fadvise DONTNEED), so the reader goes to storage.
# usage (via gpurun): bash tools/cli_e2e.sh TAG
set -e
TAG=${1:-e2e}
cd "$GRAFT_REPO_ROOT"
D=/tmp/ldg_e2e
mkdir -p $D gpurun_out
timeout -k 10 120 python tools/make_capture_file.py $D/cap60.u8 60 > gpurun_out/${TAG}_make.txt 2>&1
lscpu > gpurun_out/${TAG}_lscpu.txt 2>&1 || true
df -h /tmp >> gpurun_out/${TAG}_lscpu.txt 2>&1 || true
uncache() {
  python -c "import os,sys
for p in sys.argv[1:]:
    fd = os.open(p, os.O_RDONLY); os.fsync(fd) if False else None; os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED); os.close(fd)" "$@"
}
run() {   # name, extra args
  local name=$1; shift
  rm -f $D/out_*
  sync
  local t0=$(date +%s.%N)
  timeout -k 10 300 python ld-decode_amd/lddecode.py --stats-json gpurun_out/${TAG}_${name}_stats.json "$@" \
      $D/cap60.u8 $D/out_$name > $D/${name}.stdout 2> gpurun_out/${TAG}_${name}.err
  local t1=$(date +%s.%N)
  echo "$name wall_s $(python -c "print(round($t1 - $t0, 3))") (process start to exit, python and HIP init included)" >> gpurun_out/${TAG}_walls.txt
  ls -l $D/out_$name.* >> gpurun_out/${TAG}_${name}.err
  tail -2 $D/${name}.stdout >> gpurun_out/${TAG}_${name}.err
  sha256sum $D/out_$name.tbc $D/out_$name.pcm $D/out_$name.json | sed "s|$D/out_$name||" > gpurun_out/${TAG}_${name}_sha.txt
}
run stream
uncache $D/cap60.u8
run stream_cold
run stream_comb --comb
run whole --window-mb 0
cmp gpurun_out/${TAG}_stream_sha.txt gpurun_out/${TAG}_whole_sha.txt && echo "stream == whole: identical .tbc .pcm .json" > gpurun_out/${TAG}_cmp.txt
rm -rf $D
echo done

#!/bin/bash
# A long capture through lddecode.py's streamed capture (2 GiB ring): SECONDS of NTSC
# CLV u8 written to local storage, decoded to .tbc/.pcm/.json with --stats-json.
# usage (via gpurun): bash tools/cli_long.sh TAG SECONDS
set -e
TAG=${1:-long}; SECS=${2:-600}
cd "$GRAFT_REPO_ROOT"
D=/tmp/ldg_long
mkdir -p $D gpurun_out
df -h /tmp > gpurun_out/${TAG}_df.txt
timeout -k 10 400 python tools/make_capture_file.py $D/cap.u8 $SECS 0 --clv > gpurun_out/${TAG}_make.txt 2>&1
t0=$(date +%s.%N)
timeout -k 10 600 python ld-decode_amd/lddecode.py --stats-json gpurun_out/${TAG}_stats.json $D/cap.u8 $D/out \
    > $D/stdout.txt 2> gpurun_out/${TAG}.err
t1=$(date +%s.%N)
echo "wall_s $(python -c "print(round($t1 - $t0, 3))")" > gpurun_out/${TAG}_wall.txt
ls -l $D >> gpurun_out/${TAG}_wall.txt
grep -c '^frame ' $D/stdout.txt >> gpurun_out/${TAG}_wall.txt
rm -rf $D
echo done

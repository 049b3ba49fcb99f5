set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/profile.sh s95 "--no-cpu" "FETCH_SIZE" "WRITE_SIZE" > gpurun_out/s95_prof.log 2>&1

set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof/r05_d
timeout -k 10 120 python tools/demod_iso.py 20 > gpurun_out/r05_d_iso_new.txt 2>&1
LDG_DEMOD2=0 timeout -k 10 120 python tools/demod_iso.py 20 > gpurun_out/r05_d_iso_old.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/r05_d/trace -o run -- python3 tools/demod_iso.py 20 > gpurun_out/prof/r05_d/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VALU,SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/prof/r05_d/pmc1 -o run -- python3 tools/demod_iso.py 20 > gpurun_out/prof/r05_d/pmc1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_VALU,SQ_INSTS_VALU_FMA_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_ADD_F64,SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE,GRBM_COUNT --output-format csv -d gpurun_out/prof/r05_d/pmc2 -o run -- python3 tools/demod_iso.py 20 > gpurun_out/prof/r05_d/pmc2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/r05_d/pmc3 -o run -- python3 tools/demod_iso.py 20 > gpurun_out/prof/r05_d/pmc3.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/r05_d/pmc4 -o run -- python3 tools/demod_iso.py 20 > gpurun_out/prof/r05_d/pmc4.log 2>&1
echo done

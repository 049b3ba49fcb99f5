#!/bin/bash
# One gpurun session, parameterised (replaces the per-session sNN_probe.sh wrappers):
#   gpurun -- 'bash tools/session.sh TAG STEP [STEP ...]'
# STEP (each under its own time limit, chained: the first failure ends the session):
#   tests[=PYTEST-K-EXPR]   pytest -m gpu             -> gpurun_out/TAG_tests.txt
#   smoke                   __graft_entry__.smoke()   -> gpurun_out/TAG_smoke.txt
#   bench[=ARGS]            python bench.py ARGS      -> gpurun_out/TAG_bench[N].json (+ .err)
#   prof[=ARGS]             tools/profile.sh TAG "ARGS" FETCH_SIZE WRITE_SIZE -> gpurun_out/prof/TAG
#   sq[=ARGS]               SQ / GRBM counter passes (no trace) -> gpurun_out/prof/TAGsq
#   lds[=ARGS]              LDS bytes / scalar counter passes   -> gpurun_out/prof/TAGlds
#   run=CMD                 any command (bash -c)     -> gpurun_out/TAG_runN.txt
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1; shift
n=0
for step in "$@"; do
  n=$((n+1))
  name=${step%%=*}; arg=""
  [[ "$step" == *=* ]] && arg=${step#*=}
  case $name in
    tests)
      k=(); [ -n "$arg" ] && k=(-k "$arg")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" \
        > gpurun_out/${TAG}_tests.txt 2>&1 ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 ;;
    bench)
      timeout -k 10 600 python bench.py $arg > gpurun_out/${TAG}_bench$n.json 2> gpurun_out/${TAG}_bench$n.err ;;
    prof)
      bash tools/profile.sh $TAG "$arg" FETCH_SIZE WRITE_SIZE > gpurun_out/${TAG}_prof.log 2>&1 ;;
    sq)
      # the demod's issue / LDS / FP64 counters (MI355X_MICROARCH.md: <= 8 SQ, 2 GRBM per pass)
      bash tools/profile.sh ${TAG}sq "$arg" notrace \
        SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VALU,SQ_WAIT_INST_LDS \
        SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_VALU,SQ_INSTS_VALU_FMA_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_ADD_F64,SQ_BUSY_CU_CYCLES \
        GRBM_GUI_ACTIVE,GRBM_COUNT > gpurun_out/${TAG}_sq.log 2>&1 ;;
    lds)
      # LDS bytes moved and the scalar side (the LDS roofline of the demod)
      bash tools/profile.sh ${TAG}lds "$arg" notrace \
        SQ_INSTS_LDS_LOAD,SQ_INSTS_LDS_STORE,SQ_INSTS_LDS_LOAD_BANDWIDTH,SQ_INSTS_LDS_STORE_BANDWIDTH \
        SQ_ACTIVE_INST_SCA,SQ_INSTS_SALU,SQ_LDS_ADDR_CONFLICT,SQ_LDS_DATA_FIFO_FULL > gpurun_out/${TAG}_lds.log 2>&1 ;;
    run)
      timeout -k 10 600 bash -c "$arg" > gpurun_out/${TAG}_run$n.txt 2>&1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "step $n ($name) ok"
done

#!/bin/bash
# Interleaved bench runs per LDG_STREAM_ORDER (stream creation = hardware queue order):
#   tools/order_ab.sh REPS "ORDER1 ORDER2 ..." BENCH-ARGS...
set -e
REPS=$1; ORDERS=$2; shift 2
for i in $(seq 1 $REPS); do
  for o in $ORDERS; do
    out=$(LDG_STREAM_ORDER=$o timeout -k 10 300 python bench.py "$@" 2>/dev/null | tail -1)
    echo "$o $(python -c "import json,sys; d=json.loads(sys.argv[1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['checks'].get('phase_s', ''))" "$out")"
  done
done

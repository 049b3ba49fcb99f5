#!/bin/bash
# gpurun with waits while no box / slot is free (exit 3: nothing ran, nothing charged)
LOG=$1; shift
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun "$@" > $LOG 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 150
done
exit $rc

#!/bin/bash
# usage: scripts/gpr.sh LOG TIMEOUT CMD -- retries only when no box was free (exit 3: nothing ran)
LOG=$1; TO=$2; shift 2
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  if [ $rc -ne 3 ]; then echo "EXIT $rc" >> $LOG; exit $rc; fi
  echo "no box (try $i), waiting" >> $LOG.retries
  sleep 150
done
echo "EXIT 3 (gave up)" >> $LOG

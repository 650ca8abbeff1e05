#!/bin/bash
# Build-container helper: run one gpurun call, retrying only while the pool has no box or slot
# free (gpurun exit 3: nothing ran, nothing charged).  Any other outcome ends the loop.
# Usage: tools/gpurun_retry.sh OUTFILE TIMEOUT 'command'
OUT=$1; TO=$2; CMD=$3
for k in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $OUT 2>&1
  rc=$?
  echo "[retry] attempt $k rc=$rc" >> $OUT.attempts
  if [ $rc -ne 3 ] && ! grep -q "status=transient" $OUT; then exit $rc; fi
  sleep 150
done
exit 3

#!/bin/bash
# On the GPU box: run "NAME SECONDS CMD..." steps from a steps file, each under its own time
# limit, logging to OUT/NAME.log.  A step that fails normally (a test failure, exit 1) does
# not stop the list; a timeout, abort, kill or segfault (124/134/137/139) ends it there.
# Usage: tools/gpu_steps.sh OUT STEPFILE
OUT=$1; STEPS=$2
mkdir -p $OUT
while read -r name secs cmd; do
  [ -z "$name" ] && continue
  case "$name" in \#*) continue;; esac
  echo "[step $name] $cmd" >> $OUT/steps.log
  # heartbeat: a step that prints nothing for minutes (a long oracle check) still writes here
  ( while true; do sleep 60; echo "[$(date +%T)] $name running" >> $OUT/heartbeat.log; done ) &
  hb=$!
  timeout -k 10 $secs bash -c "$cmd" > $OUT/$name.log 2>&1
  rc=$?
  kill $hb 2>/dev/null; wait $hb 2>/dev/null
  echo "[step $name] rc=$rc" >> $OUT/steps.log
  case $rc in 124|134|137|139) echo "stopping after $name (rc=$rc)" >> $OUT/steps.log; exit $rc;; esac
done < $STEPS

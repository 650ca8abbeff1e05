#!/bin/bash
# On the GPU box (gpurun): selected GPU tests, then the default two-stream bench without the
# CPU leg (A/B of a change).  Usage: tools/gpu_ab.sh OUTDIR [pytest selection...]
OUT=${1:-gpurun_out/ab}
shift
mkdir -p $OUT
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> $OUT/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python3 -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err

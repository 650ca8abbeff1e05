#!/bin/bash
# On the GPU box (gpurun): GPU tests, then a kernel-trace profile of one bench step
# (cold run included; one mapping stream, so kernel durations are not inflated by the other
# stream's kernels).  Usage: [NOTEST=1] tools/gpu_iter.sh OUTDIR [pytest selection...]
OUT=${1:-gpurun_out/iter}
shift
SEL=${@:-tests}
mkdir -p $OUT
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> $OUT/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --map-streams 1 > $OUT/bench.json 2> $OUT/bench.err

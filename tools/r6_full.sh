#!/bin/bash
# round 6: GPU tests (the ones named, or the whole suite), then the C5 (CAMI-high) bench
# without the CPU leg; a heartbeat file keeps the silent stretches (C5 data generation, the
# oracle's mapping on the host cores) visible
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r6_full
mkdir -p $OUT
(while true; do date >> $OUT/heartbeat; sleep 50; done) &
HB=$!
trap "kill $HB" EXIT
SEL=${TESTS:-tests}
timeout -k 10 1800 python -u -m pytest $SEL -m gpu -x -v --timeout 1500 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
[ -n "$NOC5" ] || timeout -k 10 900 python3 bench.py --workload cami-high --steps 2 --warmup 1 --no-cpu > $OUT/c5_bench.json 2> $OUT/c5_bench.err

#!/bin/bash
# round 6 head: C5 one-stream kernel trace (regions wave kernel after the set_parent change)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r6_c5one
mkdir -p $OUT
(while true; do date >> $OUT/heartbeat; sleep 50; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace1 -o run -- python3 bench.py --workload cami-high --steps 1 --warmup 1 --no-cpu --map-streams 1 > $OUT/trace1_bench.json 2> $OUT/trace1_bench.err || exit $?
python3 tools/lastrun.py $OUT/trace1 40 > $OUT/laststep_1.txt
gzip -f $OUT/trace1/*kernel_trace.csv

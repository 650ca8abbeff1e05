#!/bin/bash
# round 6: chaining work-prefetch A/B on the C4 dump + one-stream kernel trace of the bench
set -eo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
NOTEST=1 LONG=1 AB_OUT=r6_ab1 bash tools/chain_ab.sh chain_prof chain_prof_wpf0 chain_prof_gt chain_prof_gt0
OUT=gpurun_out/r6_ab1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace1 -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu --map-streams 1 > $OUT/trace1_bench.json 2> $OUT/trace1_bench.err
python3 tools/lastrun.py $OUT/trace1 60 > $OUT/onestream_laststep.txt
find $OUT -name '*.csv' -size +20M -delete
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace2 -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu > $OUT/trace2_bench.json 2> $OUT/trace2_bench.err
python3 tools/lastrun.py $OUT/trace2 60 > $OUT/twostream_laststep.txt
python3 tools/busy_union.py $OUT/trace1 > $OUT/busy_onestream.txt
python3 tools/busy_union.py $OUT/trace2 > $OUT/busy_twostream.txt
find $OUT -name '*.csv' -size +20M -delete

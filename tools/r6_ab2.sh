#!/bin/bash
# round 6: t cleared in the chaining kernels (default) vs a fill (tools/var/tz0): chain_prof on
# the C4 dumps, one-stream kernel traces and two-stream benches of both libraries
set -eo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
NOTEST=1 LONG=1 AB_OUT=r6_ab2 bash tools/chain_ab.sh chain_prof chain_prof_tz0
OUT=gpurun_out/r6_ab2
for v in def tz0; do
  unset HYMET_LIB; [ $v = tz0 ] && export HYMET_LIB=tools/var/tz0/libhymet_gpu.so
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace1_$v -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu --map-streams 1 > $OUT/trace1_$v.json 2> $OUT/trace1_$v.err
  python3 tools/lastrun.py $OUT/trace1_$v 30 > $OUT/onestream_$v.txt
  python3 tools/busy_union.py $OUT/trace1_$v >> $OUT/onestream_$v.txt
  timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 --no-cpu > $OUT/bench_$v.json 2> $OUT/bench_$v.err
done
find $OUT -name '*.csv' -size +20M -delete

#!/bin/bash
# round 6 final measurements: the default bench line (CPU leg), the rocprofv3 kernel-trace
# stats of the same command, C5 and Zymo-backbone benches, the emulated N = 8 step
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r6_final
mkdir -p $OUT
(while true; do date >> $OUT/heartbeat; sleep 50; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python3 bench.py > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit $?
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace2 -o run -- python3 bench.py --no-cpu > $OUT/trace2_bench.json 2> $OUT/trace2_bench.err || exit $?
python3 tools/lastrun.py $OUT/trace2 60 > $OUT/twostream_laststep.txt
python3 tools/busy_union.py $OUT/trace2 >> $OUT/twostream_laststep.txt
gzip -f $OUT/trace2/*kernel_trace.csv
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace1 -o run -- python3 bench.py --no-cpu --map-streams 1 --steps 3 --warmup 1 > $OUT/trace1_bench.json 2> $OUT/trace1_bench.err || exit $?
python3 tools/lastrun.py $OUT/trace1 60 > $OUT/onestream_laststep.txt
python3 tools/busy_union.py $OUT/trace1 >> $OUT/onestream_laststep.txt
gzip -f $OUT/trace1/*kernel_trace.csv
timeout -k 10 900 python3 bench.py --workload cami-medium-zymo > $OUT/bench_zymo.json 2> $OUT/bench_zymo.err || exit $?
timeout -k 10 900 python3 bench.py --emulate-rank 0,7/8 --steps 3 --warmup 2 > $OUT/emulate_c4.json 2> $OUT/emulate_c4.err || exit $?
timeout -k 10 1100 python3 bench.py --workload cami-high --steps 2 --warmup 1 > $OUT/bench_c5.json 2> $OUT/bench_c5.err

#!/bin/bash
# round 6: two-stream kernel trace of the bench (per-kernel concurrency), then PC sampling
# (stochastic, beta) of the chaining kernel on the C4 first-batch dump
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r6_pcs
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace2 -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu > $OUT/trace2_bench.json 2> $OUT/trace2_bench.err || exit $?
python3 tools/lastrun.py $OUT/trace2 40 > $OUT/twostream_laststep.txt
python3 tools/busy_union.py $OUT/trace2 >> $OUT/twostream_laststep.txt
python3 tools/overlap.py $OUT/trace2 16 > $OUT/twostream_overlap.txt
gzip -f $OUT/trace2/*kernel_trace.csv
timeout -k 10 60 rocprofv3 -L > $OUT/list_avail.txt 2>&1
HYMET_DUMP_MAX=300000000 HYMET_DUMP_ANCHORS=/tmp/anchors.bin timeout -k 10 400 python3 bench.py --steps 1 --warmup 0 --no-cpu --contig-gbp 0.1 > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -s KILL 120 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 262144 --output-format csv -d $OUT/pcs -o run -- tools/chain_prof /tmp/anchors.bin 1000 > $OUT/pcs_stdout.txt 2> $OUT/pcs_stderr.txt
echo "pcs rc=$?" >> $OUT/pcs_stderr.txt
ls -laR $OUT/pcs >> $OUT/pcs_stderr.txt 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ztrace1 -o run -- python3 bench.py --workload cami-medium-zymo --steps 1 --warmup 1 --no-cpu --map-streams 1 > $OUT/ztrace1_bench.json 2> $OUT/ztrace1_bench.err
python3 tools/lastrun.py $OUT/ztrace1 40 > $OUT/zymo_onestream_laststep.txt
gzip -f $OUT/ztrace1/*kernel_trace.csv

#!/bin/bash
# round 6: PC sampling (stochastic, beta) of the chaining kernel on the C4 first-batch dump
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r6_pcs
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/list_avail.txt 2>&1
HYMET_DUMP_MAX=300000000 HYMET_DUMP_ANCHORS=/tmp/anchors.bin timeout -k 10 400 python3 bench.py --steps 1 --warmup 0 --no-cpu --contig-gbp 0.1 > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -s KILL 120 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 262144 --output-format csv -d $OUT/pcs -o run -- tools/chain_prof /tmp/anchors.bin 1000 > $OUT/pcs_stdout.txt 2> $OUT/pcs_stderr.txt
echo "pcs rc=$?" >> $OUT/pcs_stderr.txt
ls -laR $OUT/pcs >> $OUT/pcs_stderr.txt 2>&1
find $OUT -name '*.csv' -size +60M -delete

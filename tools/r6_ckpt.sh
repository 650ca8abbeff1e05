#!/bin/bash
# round 6 checkpoint: the emulated N = 8 step (ranks 0 and 7), then the default bench line with
# its CPU leg
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r6_ckpt
mkdir -p $OUT
(while true; do date >> $OUT/heartbeat; sleep 50; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python3 bench.py --emulate-rank 0,7/8 --steps 3 --warmup 2 > $OUT/emulate_c4.json 2> $OUT/emulate_c4.err || exit $?
timeout -k 10 900 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err

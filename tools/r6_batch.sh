#!/bin/bash
# round 6: mapping batch size (C4 60 / 75 / 90 Mbp, C5 40 / 50 Mbp) with a larger scratch cap
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r6_batch
mkdir -p $OUT
(while true; do date >> $OUT/heartbeat; sleep 50; done) &
HB=$!
trap "kill $HB" EXIT
export HYMET_SCRATCH_CAP_GB=230
for b in 60 75 90; do
  timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 --no-cpu --batch-mbp $b > $OUT/c4_b$b.json 2> $OUT/c4_b$b.err || exit $?
done
for b in 40 50; do
  timeout -k 10 900 python3 bench.py --workload cami-high --steps 2 --warmup 1 --no-cpu --batch-mbp $b > $OUT/c5_b$b.json 2> $OUT/c5_b$b.err || exit $?
done

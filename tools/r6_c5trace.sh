#!/bin/bash
# round 6: three mapping streams on C4 (benches), then C5 kernel traces (two mapping streams:
# GPU busy union; one stream: per-kernel totals)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r6_c5trace
mkdir -p $OUT
(while true; do date >> $OUT/heartbeat; sleep 50; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python3 bench.py --steps 4 --warmup 2 --no-cpu --map-streams 3 --batch-mbp 40 > $OUT/c4_s3_b40.json 2> $OUT/c4_s3_b40.err
HYMET_SCRATCH_CAP_GB=230 timeout -k 10 400 python3 bench.py --steps 4 --warmup 2 --no-cpu --map-streams 3 > $OUT/c4_s3_b60.json 2> $OUT/c4_s3_b60.err
for s in 2 1; do
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace$s -o run -- python3 bench.py --workload cami-high --steps 1 --warmup 1 --no-cpu --map-streams $s > $OUT/trace${s}_bench.json 2> $OUT/trace${s}_bench.err || exit $?
  python3 tools/lastrun.py $OUT/trace$s 40 > $OUT/laststep_$s.txt
  python3 tools/busy_union.py $OUT/trace$s >> $OUT/laststep_$s.txt
  gzip -f $OUT/trace$s/*kernel_trace.csv
done

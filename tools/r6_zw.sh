#!/bin/bash
# round 6: z-order wave kernel loading 64 groups' bounds per round -- mapping tests, C4
# one-stream kernel trace, C4 and C5 benches (no CPU leg)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r6_zw
mkdir -p $OUT
(while true; do date >> $OUT/heartbeat; sleep 50; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 1200 python -u -m pytest ${TESTS:-tests/test_mm_map_gpu.py tests/test_zymo_real_gpu.py tests/test_configs_gpu.py} -m gpu -x -v --timeout 1100 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace1 -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu --map-streams 1 > $OUT/trace1_bench.json 2> $OUT/trace1_bench.err || exit $?
python3 tools/lastrun.py $OUT/trace1 40 > $OUT/onestream_laststep.txt
gzip -f $OUT/trace1/*kernel_trace.csv
timeout -k 10 600 python3 bench.py --steps 5 --warmup 2 --no-cpu > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit $?
[ -n "$NOC5" ] || timeout -k 10 900 python3 bench.py --workload cami-high --steps 2 --warmup 1 --no-cpu > $OUT/bench_c5.json 2> $OUT/bench_c5.err

#!/bin/bash
# round 6: lane-kernel chaining with the group's anchor loads issued together -- chaining and
# mapping tests, C4 and Zymo one-stream kernel traces, the C5 bench (no CPU leg)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r6_cs
mkdir -p $OUT
(while true; do date >> $OUT/heartbeat; sleep 50; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 1200 python -u -m pytest tests/test_chain_gpu.py tests/test_mm_map_gpu.py tests/test_zymo_real_gpu.py tests/test_configs_gpu.py -m gpu -x -v --timeout 1100 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace1 -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu --map-streams 1 > $OUT/trace1_bench.json 2> $OUT/trace1_bench.err || exit $?
python3 tools/lastrun.py $OUT/trace1 40 > $OUT/onestream_laststep.txt
gzip -f $OUT/trace1/*kernel_trace.csv
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ztrace1 -o run -- python3 bench.py --workload cami-medium-zymo --steps 1 --warmup 1 --no-cpu --map-streams 1 > $OUT/ztrace1_bench.json 2> $OUT/ztrace1_bench.err || exit $?
python3 tools/lastrun.py $OUT/ztrace1 40 > $OUT/zymo_onestream_laststep.txt
gzip -f $OUT/ztrace1/*kernel_trace.csv
timeout -k 10 900 python3 bench.py --workload cami-high --steps 2 --warmup 1 --no-cpu > $OUT/bench_c5.json 2> $OUT/bench_c5.err

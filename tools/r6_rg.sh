#!/bin/bash
# round 6: regions sorts with loads batched per pass -- mapping tests, then the Zymo-backbone bench and its
# one-stream kernel trace (regions_wave_kernel per launch)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r6_rg
mkdir -p $OUT
(while true; do date >> $OUT/heartbeat; sleep 50; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 1200 python -u -m pytest ${TESTS:-tests/test_zymo_real_gpu.py tests/test_mm_map_gpu.py tests/test_configs_gpu.py} -m gpu -x -v --timeout 1100 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ztrace1 -o run -- python3 bench.py --workload cami-medium-zymo --steps 1 --warmup 1 --no-cpu --map-streams 1 > $OUT/ztrace1_bench.json 2> $OUT/ztrace1_bench.err || exit $?
python3 tools/lastrun.py $OUT/ztrace1 40 > $OUT/zymo_onestream_laststep.txt
gzip -f $OUT/ztrace1/*kernel_trace.csv
timeout -k 10 600 python3 bench.py --workload cami-medium-zymo --steps 3 --warmup 1 --no-cpu > $OUT/zymo_bench.json 2> $OUT/zymo_bench.err
HYMET_REG_PROF=1 timeout -k 10 600 python3 bench.py --workload cami-medium-zymo --steps 1 --warmup 0 --no-cpu --map-streams 1 > $OUT/regprof_bench.json 2> $OUT/regprof_bench.err

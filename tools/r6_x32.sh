#!/bin/bash
# round 6: x's low words as their own array for the chaining kernels -- mapping tests, the dump
# timing, FETCH/WRITE of the chaining kernels, one-stream trace and a two-stream bench
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r6_x32
mkdir -p $OUT
(while true; do date >> $OUT/heartbeat; sleep 50; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_chain_gpu.py tests/test_mm_map_gpu.py tests/test_zymo_real_gpu.py tests/test_configs_gpu.py tests/test_pipeline_gpu.py > $OUT/tests.log 2>&1 || exit $?
NOTEST=1 LONG=1 AB_OUT=r6_x32/dump bash tools/chain_ab.sh chain_prof || exit $?
RE='chain_groups_kernel|tile_scatter_kernel|mark_compact_kernel|block_seg_sort'
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-include-regex "$RE" --output-format csv -d $OUT/$c -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $OUT/${c}_bench.json 2> $OUT/${c}_bench.err || exit $?
done
python3 tools/pmc_summary.py $OUT/pmc_traffic_c4.json $OUT/FETCH_SIZE $OUT/WRITE_SIZE > $OUT/pmc_summary.txt
find $OUT -name '*.csv' -size +20M -delete
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace1 -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu --map-streams 1 > $OUT/trace1.json 2> $OUT/trace1.err || exit $?
python3 tools/lastrun.py $OUT/trace1 60 > $OUT/onestream_laststep.txt
python3 tools/busy_union.py $OUT/trace1 >> $OUT/onestream_laststep.txt
gzip -f $OUT/trace1/*kernel_trace.csv
timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 --no-cpu > $OUT/bench.json 2> $OUT/bench.err

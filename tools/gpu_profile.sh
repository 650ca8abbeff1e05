#!/bin/bash
# On the GPU box (gpurun): rocprofv3 kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes of the
# bench's hot kernels, summarised into gpurun_out/prof_TAG/.  Usage: tools/gpu_profile.sh TAG
set -eo pipefail
TAG=${1:-run}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS="--steps 1 --warmup 1 --no-cpu"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace_bench.json 2> $OUT/trace_bench.err
RE='chain_groups_kernel|backtrack_groups_kernel|write_anchor_keys_kernel|screen_count_kernel|tile_scatter_kernel|scan_down_kernel'
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RE" --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch_bench.json 2> $OUT/fetch_bench.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RE" --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write_bench.json 2> $OUT/write_bench.err
python3 tools/pmc_summary.py $OUT/pmc_traffic.json $OUT/fetch $OUT/write > $OUT/pmc_summary.txt
find $OUT -name '*.csv' -size +20M -delete

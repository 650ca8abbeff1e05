#!/bin/bash
# round 6 (HEAD): FETCH_SIZE / WRITE_SIZE passes of the C4 bench's hot kernels (verdict item 6),
# then the chaining kernel's SQ issue counters on the C4 first-batch dump
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r6_pmc
mkdir -p $OUT
(while true; do date >> $OUT/heartbeat; sleep 50; done) &
HB=$!
trap "kill $HB" EXIT
RE='chain_groups_kernel|write_anchor_keys_kernel|backtrack_long_kernel|chain_stats_flat_kernel|tile_scatter_kernel|mark_compact_kernel|group_heads_'
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-include-regex "$RE" --output-format csv -d $OUT/$c -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $OUT/${c}_bench.json 2> $OUT/${c}_bench.err || exit $?
done
python3 tools/pmc_summary.py $OUT/pmc_traffic_c4.json $OUT/FETCH_SIZE $OUT/WRITE_SIZE > $OUT/pmc_summary.txt
find $OUT -name '*.csv' -size +20M -delete
NOTEST=1 AB_OUT=r6_pmc/dump bash tools/chain_ab.sh chain_prof || exit $?
PMC_OUT=r6_pmc/sq bash tools/chain_pmc2.sh chain_prof

#!/bin/bash
# On the GPU box: dump the first mapping batch's real anchors (bench cold run on a 0.1 Gbp
# pool against the full C4 candidate set), then the chaining profile of the builds named
# (LONG=1: also on the long-join re-chain's anchors, bw 100k).
REPO=$(cd "$(dirname "$0")/.." && pwd)
OUT=$REPO/gpurun_out/${AB_OUT:-chain_ab}
mkdir -p $OUT
cd $REPO
HYMET_DUMP_MAX=${DUMP_MAX:-300000000} HYMET_DUMP_ANCHORS=/tmp/anchors.bin HYMET_DUMP_ANCHORS2=/tmp/anchors2.bin timeout -k 10 400 python3 bench.py --workload ${WORKLOAD:-cami-medium} --steps 1 --warmup 0 --no-cpu --contig-gbp 0.1 > $OUT/bench.json 2> $OUT/bench.err || exit $?
for b in "$@"; do
  timeout -k 10 200 tools/$b /tmp/anchors.bin 1000 > $OUT/$b.txt 2>&1 || exit $?
  [ -z "$LONG" ] || timeout -k 10 200 tools/$b /tmp/anchors2.bin 100000 > $OUT/$b.long.txt 2>&1 || exit $?
done
[ -n "$NOTEST" ] || timeout -k 10 400 python -u -m pytest tests/test_chain_gpu.py -x -q --timeout 300 > $OUT/chain_tests.log 2>&1

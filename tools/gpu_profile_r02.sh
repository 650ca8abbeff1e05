#!/bin/bash
# On the GPU box: world-2 test, rocprofv3 kernel stats of the bench, a host-side cProfile
# of one step, and the chaining section profile on the bench's real anchors.
REPO=$(cd "$(dirname "$0")/.." && pwd)
OUT=$REPO/gpurun_out/r02
mkdir -p $OUT
cd $REPO
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py -v --timeout 300 -k world2 > $OUT/w2test.log 2>&1
echo "w2 rc=$?" >> $OUT/w2test.log
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $REPO/bench.py --steps 2 --warmup 1 --no-cpu > $OUT/trace_bench.json 2> $OUT/trace_bench.err || exit $?
cd $REPO
HYMET_BENCH_PYPROF=1 HYMET_DUMP_ANCHORS=/tmp/anchors.bin timeout -k 10 500 python3 bench.py --steps 1 --warmup 1 --no-cpu > $OUT/pyprof.json 2> $OUT/pyprof.err || exit $?
timeout -k 10 300 tools/chain_prof /tmp/anchors.bin 1000 > $OUT/chain_prof.txt 2>&1
find $OUT -name '*.csv' -size +20M -delete

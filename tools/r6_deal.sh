#!/bin/bash
# round 6: mapping tasks pulled from a queue vs dealt round-robin (HYMET_MAP_DEAL=rr), alternating
cd "$(dirname "$0")/.."
OUT=gpurun_out/r6_deal
mkdir -p $OUT
(while true; do date >> $OUT/heartbeat; sleep 50; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_pipeline_gpu.py -k "map_streams or world2_pipeline_equals_world1 and loader-halves" > $OUT/tests.log 2>&1 || exit $?
for r in 1 2; do
  for v in q rr; do
    unset HYMET_MAP_DEAL; [ $v = rr ] && export HYMET_MAP_DEAL=rr
    timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu > $OUT/bench_${v}_$r.json 2> $OUT/bench_${v}_$r.err || exit $?
  done
done

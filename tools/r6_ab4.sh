#!/bin/bash
# round 6: mid-group inner-walk skip (HYMET_CHAIN_MIDSKIP) on the C4 and Zymo-backbone dumps
set -eo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
(while true; do date >> gpurun_out/r6_ab4.heartbeat; sleep 50; done) &
HB=$!
trap "kill $HB" EXIT
NOTEST=1 AB_OUT=r6_ab4/c4 bash tools/chain_ab.sh chain_prof chain_prof_ms0 chain_prof_gt chain_prof_gt0
NOTEST=1 WORKLOAD=cami-medium-zymo AB_OUT=r6_ab4/zy bash tools/chain_ab.sh chain_prof chain_prof_ms0 chain_prof_gt chain_prof_gt0

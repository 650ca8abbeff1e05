#!/bin/bash
# round 6: head-block prefetch (HYMET_CHAIN_HCPF 1 / 2) on the C4 dumps
set -eo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
NOTEST=1 LONG=1 AB_OUT=r6_ab3 bash tools/chain_ab.sh chain_prof chain_prof_hc1 chain_prof_hc2

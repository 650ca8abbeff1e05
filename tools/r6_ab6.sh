#!/bin/bash
# round 6: argmin reductions on integer priority images (HYMET_CHAIN_OKEY=1) vs better()'s
# double compares, on the C4 and Zymo-backbone first-batch dumps (timing builds, NOPROF=1)
set -eo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
NOTEST=1 LONG=1 AB_OUT=r6_ab6 bash tools/chain_ab.sh chain_prof chain_prof_okey
NOTEST=1 AB_OUT=r6_ab6z WORKLOAD=cami-medium-zymo bash tools/chain_ab.sh chain_prof chain_prof_okey

#!/bin/bash
# round 6: wave-uniform state in VGPRs (HYMET_CHAIN_UNI=0) vs SGPRs on the C4 dump
set -eo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
NOTEST=1 LONG=1 AB_OUT=r6_ab5 bash tools/chain_ab.sh chain_prof chain_prof_uni0 chain_prof chain_prof_uni0

#!/bin/bash
# Build the chain section profiler (see tools/chain_prof.hip): the default kernel and the
# variants named on the command line as NAME=-DFLAG=VALUE (NOPROF=1: timing builds without the
# section counters, which change register allocation).
#   tools/chain_prof.sh pf3=-DHYMET_CHAIN_PF3=1
set -e
cd "$(dirname "$0")/.."
CXX="hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -I include"
[ -n "$NOPROF" ] || CXX="$CXX -DHYMET_CHAIN_PROF"
$CXX tools/chain_prof.hip hymet_amd/csrc/ctx.cpp -o tools/chain_prof
for v in "$@"; do
  $CXX ${v#*=} tools/chain_prof.hip hymet_amd/csrc/ctx.cpp -o tools/chain_prof_${v%%=*}
done

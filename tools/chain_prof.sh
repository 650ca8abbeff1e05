#!/bin/bash
# Build the chain section profiler (see tools/chain_prof.hip) and run it on a dumped group.
set -e
cd "$(dirname "$0")/.."
hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -DHYMET_CHAIN_PROF -I include \
    tools/chain_prof.hip hymet_amd/csrc/ctx.cpp -o tools/chain_prof
hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -DHYMET_CHAIN_PROF -DHYMET_CHAIN_STIN_FAST=0 -I include \
    tools/chain_prof.hip hymet_amd/csrc/ctx.cpp -o tools/chain_prof_base

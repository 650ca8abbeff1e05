#!/bin/bash
# On the GPU box: dump real first-pass anchors (as tools/chain_ab.sh), then SQ counter passes
# of the chaining kernel on them (tools/chain_prof_np: the timing build).  One rocprofv3 pass
# per counter set, each under its own time limit.
REPO=$(cd "$(dirname "$0")/.." && pwd)
OUT=$REPO/gpurun_out/chain_pmc
mkdir -p $OUT
cd $REPO
HYMET_DUMP_ANCHORS=/tmp/anchors.bin timeout -k 10 400 python3 bench.py --steps 1 --warmup 0 --no-cpu --contig-gbp 0.1 > $OUT/bench.json 2> $OUT/bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
n=0
for P in "$P1" "$P2"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex chain_groups --output-format csv -d $OUT/p$n -o run -- $REPO/tools/chain_prof_np /tmp/anchors.bin 1000 > $OUT/p$n.log 2>&1 || exit $?
done

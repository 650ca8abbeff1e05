#!/bin/bash
# On the GPU box, after tools/chain_ab.sh (which leaves the real first-batch anchors in
# /tmp/anchors.bin): SQ counter passes of the chaining kernel for each chain_prof build named,
# one rocprofv3 pass per counter set, each under its own time limit.
REPO=$(cd "$(dirname "$0")/.." && pwd)
OUT=$REPO/gpurun_out/${PMC_OUT:-chain_pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
for b in "$@"; do
  n=0
  for P in "$P1" "$P2"; do
    n=$((n+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex chain_groups --output-format csv -d $OUT/${b}_p$n -o run -- $REPO/tools/$b /tmp/anchors.bin 1000 > $OUT/${b}_p$n.log 2>&1 || exit $?
  done
  # busy cycles of the shader engines (the issue roofline's denominator); optional
  timeout -s KILL 60 rocprofv3 --pmc SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex chain_groups --output-format csv -d $OUT/${b}_p3 -o run -- $REPO/tools/$b /tmp/anchors.bin 1000 > $OUT/${b}_p3.log 2>&1
done

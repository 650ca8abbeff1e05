#!/bin/bash
# Drop-in for HYMET scripts/minimap2.sh: INPUT_DIR REFERENCE_FASTA INDEX_PATH PAF_OUT.
# Index build and asm10 mapping run on the GPU, equivalent to
#   minimap2 -d INDEX_PATH -I2g REFERENCE_FASTA ; minimap2 -x asm10 INDEX_PATH INPUT_DIR/*.fna   (-I from $SPLIT_IDX)
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
exec env PYTHONPATH="$HERE${PYTHONPATH:+:$PYTHONPATH}" python3 -m hymet_amd.cli map "$@"

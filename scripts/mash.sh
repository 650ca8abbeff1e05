#!/bin/bash
# Drop-in for HYMET scripts/mash.sh (same 8 positional arguments, same 5 output files).
# The Mash screen runs on the GPU (libhymet_gpu.so); selection follows mash.sh:15-55.
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
exec env PYTHONPATH="$HERE${PYTHONPATH:+:$PYTHONPATH}" python3 -m hymet_amd.cli screen "$@"

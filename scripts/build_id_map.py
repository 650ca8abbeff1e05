#!/usr/bin/env python3
"""Drop-in for HYMET tools/build_id_map.py (same argv, output bytes and messages; the classification
fallback of run_hymet_cami.sh:183-205)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hymet_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(["build-id-map"] + sys.argv[1:]))

#!/usr/bin/env python3
"""Drop-in for HYMET tools/eval_cami.py (CAMI profile + contig metrics; host only; taxonkit
restated from the taxdump)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hymet_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(["eval-cami"] + sys.argv[1:]))

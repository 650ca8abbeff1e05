#!/usr/bin/env python3
"""Drop-in for HYMET tools/hymet2cami.py (classified TSV -> CAMI profile; host only)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hymet_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(["hymet2cami"] + sys.argv[1:]))

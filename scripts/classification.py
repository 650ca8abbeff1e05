#!/usr/bin/env python3
"""Drop-in for HYMET scripts/classification.py (same flags, same output bytes); runs on the GPU."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hymet_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(["classify-legacy"] + sys.argv[1:]))

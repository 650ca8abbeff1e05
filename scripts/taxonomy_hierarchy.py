#!/usr/bin/env python3
"""Drop-in for HYMET scripts/taxonomy_hierarchy.py (taxdump -> taxonomy_hierarchy.tsv; host only)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hymet_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(["taxonomy-hierarchy"] + sys.argv[1:]))

#!/usr/bin/env python3
"""Drop-in for HYMET scripts/downloadDB.py, offline: detailed_taxonomy.tsv and
combined_genomes.fasta from the genomes already in <output_dir> and the assembly summaries
cached in <cache_dir> (no network; host only)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hymet_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(["download-db"] + sys.argv[1:]))

#!/usr/bin/env python3
"""Copy the reference's real Zymo genomes into tests/golden/zymo/ (build container only).

    python tests/golden/make_zymo_fixture.py [--ref /root/reference]

The reference ships 25 real genomes (case/truth/zymo_refs/genomes/*/*.fna.gz, 63
sequences, 107.5 Mbp; the Cryptococcus genome is a missing large blob) next to a real
minimap2 PAF of the Zymo mock-community contigs against them
(case/truth/zymo_mc/zymo_mc_vs_refs.paf, already committed as tests/golden/classify/zymo.paf).
Those two are the only evidence in the image of what the real minimap2 does on this path
(scripts/minimap2.sh:12,23), so the genomes travel with the tests as data: the gzip files
are copied unchanged, one directory per species, and a manifest records their sizes and
sha256.  No reference code is run.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import shutil
from pathlib import Path

HERE = Path(__file__).resolve().parent


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    a = ap.parse_args()
    src = Path(a.ref) / "case/truth/zymo_refs/genomes"
    out = HERE / "zymo" / "genomes"
    out.mkdir(parents=True, exist_ok=True)
    man = []
    for f in sorted(src.glob("*/*.fna.gz")):
        d = out / f.parent.name
        d.mkdir(exist_ok=True)
        shutil.copyfile(f, d / f.name)
        data = f.read_bytes()
        man.append({"species": f.parent.name, "file": f.name, "bytes": len(data),
                    "sha256": hashlib.sha256(data).hexdigest()})
    shutil.copyfile(Path(a.ref) / "case/truth/zymo_refs/seqid2taxid.tsv", HERE / "zymo" / "seqid2taxid.tsv")
    (HERE / "zymo" / "manifest.json").write_text(json.dumps(man, indent=1) + "\n")
    print(f"{len(man)} genome files -> {out}")


if __name__ == "__main__":
    main()

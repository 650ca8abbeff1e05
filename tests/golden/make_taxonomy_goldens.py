#!/usr/bin/env python3
"""Generate tests/golden/taxonomy/ by running the REFERENCE scripts themselves (importable
in the build container only; never on the GPU box):

    python tests/golden/make_taxonomy_goldens.py  [--ref /root/reference]

  names.dmp, nodes.dmp         a small synthetic NCBI taxdump with the edge cases the
                               builder meets: synonyms, a taxon without a scientific name, a
                               node whose parent is missing, a duplicated node row, 'no rank'
                               strains, 2025-style 'domain' and older 'superkingdom' tops
  expect_hierarchy.tsv         scripts/taxonomy_hierarchy.py generate_taxonomy_hierarchy on them
  classified.tsv               a classified_sequences.tsv with aliased / unknown / partial lineages
  cami_inputs.json             the taxonkit answers hymet2cami consumes (name -> taxid, taxid ->
                               (names path, ids path)), written here as fixed inputs
  expect_cami.txt              tools/hymet2cami.py load_records + accumulate + emit_cami on them
"""
from __future__ import annotations

import argparse
import contextlib
import importlib.util
import io
import json
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent


def load_module(path: Path, name: str):
    spec = importlib.util.spec_from_file_location(name, str(path))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


NODES = [  # taxid, parent, rank, division
    ("1", "1", "no rank", "8"), ("131567", "1", "no rank", "8"),
    ("2", "131567", "domain", "0"), ("2157", "131567", "superkingdom", "0"),
    ("1783272", "2", "kingdom", "0"), ("1239", "1783272", "phylum", "0"), ("91061", "1239", "class", "0"),
    ("1385", "91061", "order", "0"), ("186817", "1385", "family", "0"), ("1386", "186817", "genus", "0"),
    ("1423", "1386", "species", "0"), ("224308", "1423", "strain", "0"), ("999001", "1423", "no rank", "0"),
    ("1224", "2", "phylum", "0"), ("1236", "1224", "class", "0"), ("91347", "1236", "order", "0"),
    ("543", "91347", "family", "0"), ("561", "543", "genus", "0"), ("562", "561", "species", "0"),
    ("511145", "562", "no rank", "0"), ("83333", "562", "strain", "0"),
    ("28890", "2157", "phylum", "0"), ("183925", "28890", "class", "0"), ("2158", "183925", "order", "0"),
    ("2159", "2158", "family", "0"), ("2172", "2159", "genus", "0"), ("2173", "2172", "species", "0"),
    ("777777", "555555", "species", "0"),       # parent missing from nodes.dmp
    ("888888", "1386", "species", "0"),         # no scientific name row
    ("1423", "1386", "species", "0"),           # duplicated row (same content)
    ("12908", "1", "no rank", "8"), ("408169", "12908", "species", "8"),
]
NAMES = [  # taxid, name, unique, class
    ("1", "root", "", "scientific name"), ("131567", "cellular organisms", "", "scientific name"),
    ("2", "Bacteria", "Bacteria <bacteria>", "scientific name"), ("2", "eubacteria", "", "genbank common name"),
    ("2157", "Archaea", "", "scientific name"), ("1783272", "Bacillati", "", "scientific name"),
    ("1239", "Bacillota", "", "scientific name"), ("1239", "Firmicutes", "", "synonym"),
    ("91061", "Bacilli", "", "scientific name"), ("1385", "Bacillales", "", "scientific name"),
    ("186817", "Bacillaceae", "", "scientific name"), ("1386", "Bacillus", "Bacillus <bacterium>", "scientific name"),
    ("1423", "Bacillus subtilis", "", "scientific name"), ("224308", "Bacillus subtilis subsp. subtilis str. 168", "",
                                                        "scientific name"),
    ("999001", "Bacillus subtilis strain X", "", "scientific name"),
    ("1224", "Pseudomonadota", "", "scientific name"), ("1224", "Proteobacteria", "", "synonym"),
    ("1236", "Gammaproteobacteria", "", "scientific name"), ("91347", "Enterobacterales", "", "scientific name"),
    ("543", "Enterobacteriaceae", "", "scientific name"), ("561", "Escherichia", "", "scientific name"),
    ("562", "Escherichia coli", "", "scientific name"), ("562", "Bacterium coli", "", "synonym"),
    ("511145", "Escherichia coli str. K-12 substr. MG1655", "", "scientific name"),
    ("83333", "Escherichia coli K-12", "", "scientific name"),
    ("28890", "Methanobacteriota", "", "scientific name"), ("183925", "Methanobacteria", "", "scientific name"),
    ("2158", "Methanobacteriales", "", "scientific name"), ("2159", "Methanobacteriaceae", "", "scientific name"),
    ("2172", "Methanobrevibacter", "", "scientific name"), ("2173", "Methanobrevibacter smithii", "", "scientific name"),
    ("777777", "Orphanus incertus", "", "scientific name"),
    ("12908", "unclassified sequences", "", "scientific name"), ("408169", "metagenome", "", "scientific name"),
]

CLASSIFIED = [
    ("Query", "Lineage", "Taxonomic Level", "Confidence"),
    ("c1", "superkingdom:Bacteria; phylum:Bacillota; class:Bacilli; order:Bacillales; family:Bacillaceae; "
           "genus:Bacillus; species:Bacillus subtilis", "species", "0.9100"),
    ("c2", "superkingdom:Bacteria; phylum:Bacillota; class:Bacilli", "class", "0.5000"),
    ("c3", "domain:Bacteria;p:Pseudomonadota;c:Gammaproteobacteria;o:Enterobacterales;f:Enterobacteriaceae;"
           "g:Escherichia;s:Escherichia coli", "species", "1.0000"),
    ("c4", "Unknown", "root", "0.0000"),
    ("c5", "superkingdom:Archaea; phylum:Methanobacteriota; genus:Methanobrevibacter; species:Methanobrevibacter smithii",
     "species", "0.7700"),
    ("c6", "sk:Bacteria; k:Bacillati; phylum:Firmicutes; strain:Bacillus subtilis subsp. subtilis str. 168", "strain",
     "0.8800"),
    ("c7", "superkingdom:Bacteria; phylum:Bacillota; class:Bacilli; order:Bacillales; family:Bacillaceae; "
           "genus:Bacillus; species:Bacillus subtilis", "species", "0.9100"),
    ("c8", "species:Nomen nudum; genus:Escherichia", "species", "0.3000"),
    ("c9", "superkingdom:Bacteria; phylum:Pseudomonadota", "phylum", "0.6000"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    a = ap.parse_args()
    ref = Path(a.ref)
    out = HERE / "taxonomy"
    out.mkdir(exist_ok=True)
    with open(out / "nodes.dmp", "w") as f:
        for t, p, r, d in NODES:
            f.write(f"{t}\t|\t{p}\t|\t{r}\t|\t\t|\t{d}\t|\t0\t|\t1\t|\t0\t|\t0\t|\t0\t|\t0\t|\t0\t|\t\t|\n")
    with open(out / "names.dmp", "w") as f:
        for t, n, u, c in NAMES:
            f.write(f"{t}\t|\t{n}\t|\t{u}\t|\t{c}\t|\n")
    th = load_module(ref / "scripts" / "taxonomy_hierarchy.py", "ref_taxonomy_hierarchy")
    with contextlib.redirect_stdout(io.StringIO()):
        th.generate_taxonomy_hierarchy(str(out / "names.dmp"), str(out / "nodes.dmp"), str(out / "expect_hierarchy.tsv"))
    with open(out / "classified.tsv", "w", newline="") as f:
        for row in CLASSIFIED:
            f.write("\t".join(row) + "\r\n")
    # taxonkit answers as fixed inputs: scientific or synonym names -> taxid; paths from the
    # dump's lineage (d|p|c|o|f|g|s, empty where absent)
    sci = {}
    for t, n, _, c in NAMES:
        sci.setdefault(n, t)
    parent = {t: p for t, p, _, _ in NODES}
    rank = {t: r for t, _, r, _ in NODES}
    name_of = {t: n for t, n, _, c in NAMES if c == "scientific name"}
    want = ["domain|superkingdom", "phylum", "class", "order", "family", "genus", "species"]

    def path(t):
        at = {}
        cur = t
        while True:
            at.setdefault(rank.get(cur, ""), cur)
            if cur == "1" or cur not in parent:
                break
            cur = parent[cur]
        ids = [next((at[r] for r in w.split("|") if r in at), "") for w in want]
        return "|".join(name_of.get(i, "") if i else "" for i in ids), "|".join(ids)

    h2c = load_module(ref / "tools" / "hymet2cami.py", "ref_hymet2cami")
    recs = h2c.load_records(out / "classified.tsv")
    names = sorted({n for p in recs for n in p.values() if n})
    n2t = {n: sci[n] for n in names if n in sci}
    counts, totals, needed = h2c.accumulate(recs, n2t)
    t2p = {t: path(t) for t in sorted(needed)}
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        h2c.emit_cami(counts, totals, t2p)
    (out / "expect_cami.txt").write_text(buf.getvalue())
    (out / "cami_inputs.json").write_text(json.dumps({"name2taxid": n2t, "taxid2path": t2p}, indent=1, sort_keys=True))
    print(f"wrote {out}")


if __name__ == "__main__":
    main()

"""NCBI taxdump tools on either side of the hot path.

* hierarchy_tsv: scripts/taxonomy_hierarchy.py (:6-61) -- names.dmp + nodes.dmp ->
  taxonomy_hierarchy.tsv (TaxID, Name, Rank, ParentTaxID, Lineage "rank:name;..." from the
  root's child down), the classifier's hierarchy input.  The reference walks every taxon to
  the root (O(N x depth) list inserts); here each lineage is its parent's lineage plus one
  part, memoised for the taxa that are parents, so the build is one pass over the nodes.
* name2taxid / reformat: the two taxonkit commands tools/hymet2cami.py runs
  (`taxonkit name2taxid --show-rank`, `taxonkit reformat -I 1 -f "{d}|{p}|...|{s}" -t`),
  restated from names.dmp / nodes.dmp.  taxonkit (bench/environment.lock.yml:179, 0.20.0)
  is absent from the image: parity unpinned for these two.
* hymet2cami: tools/hymet2cami.py (:40-149) -- classified_sequences.tsv -> CAMI profile;
  its own logic (lineage parsing, per-rank counts, output) is pinned by reference-generated
  goldens (tests/golden/taxonomy).

Host-side text work on files read once: no device code.
"""
from __future__ import annotations

import csv
import io
import sys
from collections import defaultdict
from typing import Dict, Iterable, List, Optional, Tuple

CAMI_RANKS = ["superkingdom", "phylum", "class", "order", "family", "genus", "species"]
CAMI_ALIAS = {  # tools/hymet2cami.py:15-32
    "domain": "superkingdom", "kingdom": "superkingdom", "sk": "superkingdom", "k": "superkingdom",
    "phylum": "phylum", "p": "phylum", "class": "class", "c": "class", "order": "order", "o": "order",
    "family": "family", "f": "family", "genus": "genus", "g": "genus", "species": "species", "s": "species",
}


# ---------------------------------------------------------------------- taxdump
class TaxDump:
    """names.dmp + nodes.dmp, parsed the way scripts/taxonomy_hierarchy.py parses them."""

    def __init__(self, names_dmp: str, nodes_dmp: str, all_names: bool = False):
        self.sci: Dict[str, str] = {}                 # taxid -> scientific name (last row wins)
        self.names: List[Tuple[str, str, str]] = []   # (name, taxid, class) rows (taxonkit)
        with open(names_dmp, "r", encoding="utf-8") as f:
            for line in f:
                p = line.split("\t|\t")
                tid, name, cls = p[0].strip(), p[1].strip(), p[3].strip("\t|\n")
                if cls == "scientific name":
                    self.sci[tid] = name
                if all_names:
                    self.names.append((name, tid, cls))
        self.node: Dict[str, Tuple[str, str]] = {}    # taxid -> (rank, parent), file order
        with open(nodes_dmp, "r", encoding="utf-8") as f:
            for line in f:
                p = line.split("\t|\t")
                tid, parent, rank = p[0].strip(), p[1].strip(), p[2].strip("\t|\n")
                # taxonomy_hierarchy.py:31-32 tests column 4 (the division id) for "strain"
                if rank == "no rank" and "strain" in p[4]:
                    rank = "strain"
                self.node[tid] = (rank, parent)

    def lineage_parts(self, tid: str, memo: Dict[str, str]) -> str:
        """taxonomy_hierarchy.py get_lineage: 'rank:name' parts from below the root to tid
        joined by ';' (a taxid without a node row ends the walk as (\"\", root))."""
        chain = []
        cur = tid
        seen = 0
        while cur != "1" and cur not in memo:
            chain.append(cur)
            cur = self.node.get(cur, ("", "1"))[1]
            seen += 1
            if seen > len(self.node) + 1:
                raise ValueError(f"nodes.dmp: the parent chain of {tid} never reaches the root")
        base = "" if cur == "1" else memo[cur]
        for t in reversed(chain):
            rank = self.node.get(t, ("", "1"))[0]
            part = f"{rank}:{self.sci.get(t, 'Unknown')}"
            base = part if not base else base + ";" + part
            if t in self.parents:
                memo[t] = base
        return base

    @property
    def parents(self):
        p = getattr(self, "_parents", None)
        if p is None:
            p = self._parents = {par for _, par in self.node.values()}
        return p


def hierarchy_tsv(names_dmp: str, nodes_dmp: str) -> bytes:
    """The bytes scripts/taxonomy_hierarchy.py writes to data/taxonomy_hierarchy.tsv."""
    d = TaxDump(names_dmp, nodes_dmp)
    memo: Dict[str, str] = {}
    out = io.StringIO()
    out.write("TaxID\tName\tRank\tParentTaxID\tLineage\n")
    for tid, (rank, parent) in d.node.items():
        out.write(f"{tid}\t{d.sci.get(tid, 'Unknown')}\t{rank}\t{parent}\t{d.lineage_parts(tid, memo)}\n")
    return out.getvalue().encode("utf-8")


# ------------------------------------------------------------- taxonkit restated
def name2taxid(d: TaxDump, names: Iterable[str]) -> Dict[str, str]:
    """`taxonkit name2taxid --show-rank` as hymet2cami.py:60-75 consumes it: every name of
    names.dmp (any name class) matched case-insensitively; a name shared by several taxids
    prints one line per taxid in names.dmp order and the consumer keeps the last."""
    want = {n.lower(): n for n in names if n}
    out: Dict[str, str] = {}
    for name, tid, _ in d.names:
        q = want.get(name.lower())
        if q is not None:
            out[q] = tid
    return out


def reformat(d: TaxDump, taxids: Iterable[str], fmt_ranks=("domain|superkingdom", "phylum", "class", "order", "family",
                                                            "genus", "species")) -> Dict[str, Tuple[str, str]]:
    """`taxonkit reformat -I 1 -f "{d}|{p}|{c}|{o}|{f}|{g}|{s}" -t` (hymet2cami.py:78-101):
    per taxid the names and the taxids of its ancestors (itself included) at those ranks,
    '|'-joined, empty where the lineage has no such rank; unknown taxids give no line."""
    out: Dict[str, Tuple[str, str]] = {}
    want = [set(r.split("|")) for r in fmt_ranks]
    for tid in taxids:
        if not tid or tid not in d.node:
            continue
        at: Dict[str, str] = {}
        cur, hops = tid, 0
        while True:
            rank, parent = d.node.get(cur, ("", "1"))
            at.setdefault(rank, cur)
            if cur == "1" or parent == cur or hops > len(d.node):
                break
            cur, hops = parent, hops + 1
        ids = []
        for ws in want:
            t = next((at[r] for r in ws if r in at), "")
            ids.append(t)
        out[tid] = ("|".join(d.sci.get(t, "") if t else "" for t in ids), "|".join(ids))
    return out


# -------------------------------------------------------------------- hymet2cami
def parse_lineage(lineage: str) -> Dict[str, str]:
    """hymet2cami.py:40-52."""
    out = {r: "" for r in CAMI_RANKS}
    if not lineage:
        return out
    for part in lineage.split(";"):
        part = part.strip()
        if not part or ":" not in part:
            continue
        rk, name = part.split(":", 1)
        rk = CAMI_ALIAS.get(rk.strip().lower(), rk.strip().lower())
        if rk in out:
            out[rk] = name.strip()
    return out


def load_records(tsv_text: str) -> List[Dict[str, str]]:
    """hymet2cami.py:104-112 (rows whose lineage names at least one CAMI rank)."""
    recs = []
    for row in csv.DictReader(io.StringIO(tsv_text), delimiter="\t"):
        p = parse_lineage(row.get("Lineage", ""))
        if any(p.values()):
            recs.append(p)
    return recs


def cami_profile(records: List[Dict[str, str]], name2tid: Dict[str, str],
                 taxid2path: Dict[str, Tuple[str, str]], sample_id: str = "sample_0") -> str:
    """hymet2cami.py:115-149: per rank, the share of records whose name at that rank maps
    to a taxid, by count descending (stable), '%.6f' percentages."""
    counts = {r: defaultdict(int) for r in CAMI_RANKS}
    totals = {r: 0 for r in CAMI_RANKS}
    for p in records:
        for r in CAMI_RANKS:
            name = p.get(r)
            if not name:
                continue
            tid = name2tid.get(name)
            if not tid:
                continue
            counts[r][tid] += 1
            totals[r] += 1
    out = io.StringIO()
    out.write("#CAMI Submission for Taxonomic Profiling\n")
    out.write(f"@Version:0.9.1 @Ranks:superkingdom|phylum|class|order|family|genus|species @SampleID:{sample_id}\n")
    out.write("@@TAXID RANK TAXPATH TAXPATHSN PERCENTAGE\n")
    for r in CAMI_RANKS:
        total = totals[r]
        if total <= 0:
            continue
        for tid, c in sorted(counts[r].items(), key=lambda kv: kv[1], reverse=True):
            path = taxid2path.get(tid)
            if not path:
                continue
            names, ids = path
            out.write(f"{tid}\t{r}\t{ids}\t{names}\t{100.0 * c / total:.6f}\n")
    return out.getvalue()


def hymet2cami(tsv_path: str, taxdb: str, log=sys.stderr) -> str:
    """tools/hymet2cami.py main: the CAMI profile text (stdout) of a classified TSV."""
    import os
    print(f"[hymet2cami] using taxonomy DB at {taxdb}", file=log)
    with open(tsv_path, encoding="utf-8", errors="ignore") as f:
        recs = load_records(f.read())
    print(f"[hymet2cami] parsed {len(recs)} lineages", file=log)
    names = {n for p in recs for n in p.values() if n}
    print(f"[hymet2cami] converting {len(names)} unique taxon names", file=log)
    d = TaxDump(os.path.join(taxdb, "names.dmp"), os.path.join(taxdb, "nodes.dmp"), all_names=True)
    n2t = name2taxid(d, names)
    print(f"[hymet2cami] mapped {len(n2t)} names to taxids", file=log)
    needed = {n2t[n] for p in recs for n in p.values() if n and n2t.get(n)}
    print(f"[hymet2cami] converting {len(needed)} taxids to paths", file=log)
    t2p = reformat(d, sorted(needed))
    text = cami_profile(recs, n2t, t2p)
    print("[hymet2cami] done", file=log)
    return text

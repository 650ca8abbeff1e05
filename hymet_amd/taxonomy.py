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
from collections import Counter
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
    want = [r.split("|") for r in fmt_ranks]   # alternatives in preference order
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
_SLOT = {r: i for i, r in enumerate(CAMI_RANKS)}


def rank_names(lineage: str) -> List[str]:
    """A Lineage cell -> the name at each CAMI rank ("" where absent): 'label:name' parts,
    labels folded through CAMI_ALIAS (hymet2cami.py:15-32,46-58), a later part overriding an
    earlier one at the same rank, other labels ignored."""
    slots = [""] * len(CAMI_RANKS)
    for part in (lineage or "").split(";"):
        label, sep, name = part.strip().partition(":")
        if not sep:
            continue
        key = label.strip().lower()
        i = _SLOT.get(CAMI_ALIAS.get(key, key))
        if i is not None:
            slots[i] = name.strip()
    return slots


def parse_lineage(lineage: str) -> Dict[str, str]:
    return dict(zip(CAMI_RANKS, rank_names(lineage)))


def load_records(tsv_text: str) -> List[Dict[str, str]]:
    """The rows (csv.DictReader over the TSV) whose Lineage names at least one CAMI rank,
    as rank -> name (hymet2cami.py:104-112)."""
    rows = (rank_names(r.get("Lineage", "")) for r in csv.DictReader(io.StringIO(tsv_text), delimiter="\t"))
    return [dict(zip(CAMI_RANKS, slots)) for slots in rows if any(slots)]


def cami_profile(records: List[Dict[str, str]], name2tid: Dict[str, str],
                 taxid2path: Dict[str, Tuple[str, str]], sample_id: str = "sample_0") -> str:
    """The CAMI profile text (hymet2cami.py:115-149): for each rank, the records whose name
    there maps to a taxid are tallied per taxid; each taxid with a reformat path is printed
    with its share of the rank's tally, largest tally first (ties in first-seen order),
    '%.6f'.  A rank without any mapped name prints nothing."""
    lines = ["#CAMI Submission for Taxonomic Profiling",
             f"@Version:0.9.1 @Ranks:{'|'.join(CAMI_RANKS)} @SampleID:{sample_id}",
             "@@TAXID RANK TAXPATH TAXPATHSN PERCENTAGE"]
    for rank in CAMI_RANKS:
        tally = Counter(t for t in (name2tid.get(r.get(rank) or "") for r in records) if t)
        total = sum(tally.values())
        for tid, n in sorted(tally.items(), key=lambda kv: -kv[1]):
            path = taxid2path.get(tid) if total > 0 else None
            if path:
                lines.append(f"{tid}\t{rank}\t{path[1]}\t{path[0]}\t{100.0 * n / total:.6f}")
    return "\n".join(lines) + "\n"


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

"""C9: the classification fallback of run_hymet_cami.sh:183-205.

When classification_cami.py leaves fewer than 2 lines in classified_sequences.tsv, the
reference builds an identifier -> TaxID map (tools/build_id_map.py:17-48) and assigns each
query the TaxID of its first mappable PAF target (tools/mini_classify.py:7-30), then writes
`Query\tunknown\tunknown\t1.0000` rows (the awk step, run_hymet_cami.sh:198-199).

This is host-side text work on a rare branch (no device code: it reads two text files once).
"""
from __future__ import annotations

import csv
import gzip
import io
import sys
from collections import OrderedDict
from typing import Dict, Iterable, List, Sequence, Tuple


_ID_ROLES = ("GCF", "TaxID", "Identifiers")


def _taxonomy_rows(taxonomy_path: str):
    """(TaxID, [identifier tokens]) per usable row of detailed_taxonomy.tsv, with columns
    found by header name, else by position (tools/build_id_map.py:26-30)."""
    with open(taxonomy_path, "r", encoding="utf-8", errors="ignore", newline="") as f:
        head = f.readline()
        if not head:
            raise SystemExit("empty taxonomy file")
        names = head.rstrip("\n").split("\t")
        col = ({r: names.index(r) for r in _ID_ROLES} if all(r in names for r in _ID_ROLES)
               else {r: k for k, r in enumerate(_ID_ROLES)})
        need = max(col["GCF"], col["TaxID"])
        for raw in f:
            if not raw.strip():
                continue
            cells = raw.rstrip("\n").split("\t")
            if len(cells) <= need:
                continue
            extra = cells[col["Identifiers"]] if len(cells) > col["Identifiers"] else ""
            yield cells[col["TaxID"]].strip(), [cells[col["GCF"]]] + extra.strip().split(";")


def build_id_map(taxonomy_path: str) -> "OrderedDict[str, str]":
    """tools/build_id_map.py:17-43 on the classifier's identifier rule (classify.add_alias):
    the GCF and every ';'-separated identifier of a row, and their versionless forms, map to
    the row's TaxID; the first row to name a key keeps it."""
    from .classify import add_alias
    id2tax: "OrderedDict[str, str]" = OrderedDict()
    for tax, tokens in _taxonomy_rows(taxonomy_path):
        for tok in tokens:
            add_alias(id2tax, tok, tax)
    return id2tax


def write_id_map(id2tax: Dict[str, str], path: str) -> str:
    """build_id_map.py:45-50 output (csv.writer, tab-delimited, CRLF rows)."""
    with open(path, "w", encoding="utf-8", newline="") as w:
        wr = csv.writer(w, delimiter="\t")
        for k, v in id2tax.items():
            wr.writerow([k, v])
    return f"wrote {len(id2tax):,} ids -> TaxID to {path}"


def read_id_map(path: str) -> Dict[str, str]:
    """mini_classify.py:7-11: first row per id wins."""
    idmap: Dict[str, str] = {}
    with open(path, encoding="utf-8", newline="") as f:
        for row in csv.reader(f, delimiter="\t"):
            if not row:
                continue
            idmap.setdefault(row[0], row[1])
    return idmap


def _open_paf(p: str):
    if p.endswith(".gz"):
        return gzip.open(p, "rt", encoding="utf-8", errors="ignore")
    return open(p, "r", encoding="utf-8", errors="ignore")


def first_hits(lines: Iterable[Tuple[str, str]], idmap: Dict[str, str]) -> Tuple[List[Tuple[str, str, str]], int]:
    """mini_classify.py:17-29 over (qname, tname) pairs in PAF order: the first line of a
    query whose target (or its part before the first '.') has a TaxID.  Returns the rows and
    the number of alignments seen."""
    seen, rows, tot = set(), [], 0
    for q, t in lines:
        tot += 1
        if q in seen:
            continue
        tax = idmap.get(t) or idmap.get(t.split(".", 1)[0])
        if tax:
            rows.append((q, t, tax))
            seen.add(q)
    return rows, tot


def paf_pairs(paf_path: str):
    with _open_paf(paf_path) as f:
        for ln in f:
            if not ln or ln[0] == "#":
                continue
            p = ln.rstrip("\n").split("\t")
            if len(p) < 6:
                continue
            yield p[0], p[5]


def mini_classify(paf_path: str, idmap: Dict[str, str], out_path: str) -> str:
    rows, tot = first_hits(paf_pairs(paf_path), idmap)
    with open(out_path, "w", encoding="utf-8", newline="") as w:
        wr = csv.writer(w, delimiter="\t")
        wr.writerow(["qname", "tname", "taxid"])
        wr.writerows(rows)
    return f"[mini] Classified {len(rows)}/{tot} alignments (first-hit per query) -> {out_path}"


def hymet_tsv(rows: Sequence[Tuple[str, str, str]]) -> bytes:
    """run_hymet_cami.sh:198-199 (awk, OFS tab, '\\n'): the fallback classified_sequences.tsv."""
    out = io.StringIO()
    out.write("Query\tLineage\tTaxonomic Level\tConfidence\n")
    for q, _, _ in rows:
        out.write(f"{q}\tunknown\tunknown\t1.0000\n")
    return out.getvalue().encode("utf-8")


def fallback_tsv(table_pairs: Iterable[Tuple[str, str]], taxonomy_path: str) -> bytes:
    """The whole fallback branch on an in-memory PAF (pairs in PAF line order)."""
    idmap = dict(build_id_map(taxonomy_path))
    rows, _ = first_hits(table_pairs, idmap)
    return hymet_tsv(rows) if rows else b""


def main_build_id_map(argv: Sequence[str]) -> int:
    if len(argv) != 2:
        sys.exit("usage: build_id_map.py detailed_taxonomy.tsv out_map.tsv")
    print(write_id_map(build_id_map(argv[0]), argv[1]))
    return 0


def main_mini_classify(argv: Sequence[str]) -> int:
    if len(argv) != 3:
        sys.exit("usage: mini_classify.py input.paf id_to_taxid.tsv out.tsv")
    print(mini_classify(argv[0], read_id_map(argv[1]), argv[2]))
    return 0

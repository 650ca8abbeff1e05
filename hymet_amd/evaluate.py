"""CAMI evaluation of HYMET output: the metrics of tools/eval_cami.py.

Two levels, as the reference reports them:

* profiles -- a predicted and a truth CAMI profile, per rank: L1 total variation, Bray-Curtis
  and presence precision / recall / F1 (eval_cami.py:369-385, 599-632);
* contigs -- each classified contig resolved to its most specific TaxID and paired with the
  truth mapping, exact-TaxID and per-rank accuracy (eval_cami.py:388-568).

Structure (not the reference's): a profile is a `Profile` of seven rank tables; profile
files go through a list of `_PROFILE_READERS`, each a (can-read, read) pair over a parsed
table whose columns are found by role through `_ROLES`; a contig's TaxID comes from the
first of four `_RESOLVERS` that yields one; pairs come from the first of three pairing
strategies that yields any.  The metrics are computed on aligned numpy vectors over the
union of taxa and summed with math.fsum (exactly rounded; the reference's float sums follow
set iteration order, so they agree to the last bit only up to that order).

taxonkit (`name2taxid --show-rank`, `reformat -I 1 -f "{k}|..|{s}" -t`) is restated from
names.dmp / nodes.dmp by hymet_amd.taxonomy; eval_cami's {k} is taken as its superkingdom
rank, i.e. domain-or-superkingdom like hymet2cami's {d} (taxonkit is absent: unpinned,
DESIGN.md §4).  The last-resort pairing by `minimap2 -x asm10` of predicted against truth
contigs (eval_cami.py:519-528) runs only when a minimap2 binary is on PATH, as there.
Host-side text work, no device code.
"""
from __future__ import annotations

import collections
import csv
import gzip
import hashlib
import math
import os
import pathlib
import re
import shutil
import subprocess
import sys
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from .taxonomy import TaxDump, name2taxid as _name2taxid, reformat as _reformat

csv.field_size_limit(1024 * 1024 * 1024)

RANKS = ("superkingdom", "phylum", "class", "order", "family", "genus", "species")
RANK_SLOT = {r: i for i, r in enumerate(RANKS)}
# lineage rank labels -> rank (eval_cami.py:19-40: wider than hymet2cami's, strains fold
# into species)
_LABEL_RANK = dict(
    [(a, "superkingdom") for a in ("domain", "kingdom", "sk", "k", "superkingdom")]
    + [(a, "phylum") for a in ("phylum", "p")] + [(a, "class") for a in ("class", "c")]
    + [(a, "order") for a in ("order", "o")] + [(a, "family") for a in ("family", "f")]
    + [(a, "genus") for a in ("genus", "g")] + [(a, "species") for a in ("species", "s", "subspecies", "ss", "strain")])
# eval_cami's `reformat -f "{k}|{p}|{c}|{o}|{f}|{g}|{s}"`, rank by rank.  {k} is read as
# superkingdom, or domain in NCBI's 2025 dumps (which renamed the rank); taxonkit 0.20's own
# reading of {k} on such a dump is unpinned.
EVAL_FORMAT_RANKS = ("superkingdom|domain", "phylum", "class", "order", "family", "genus", "species")
_GCFA = re.compile(r"GC[AF]_\d+(?:\.\d+)?(?:_PRJ[A-Z]+\d+)?")
_ACC = re.compile(r"(NC_\d+\.\d+|NZ_[A-Z]{2}\d+\.\d+|NZ_[A-Z]{5}\d+\.\d+|CP\d+\.\d+|CM\d+\.\d+|[A-Z]{2}_\d+\.\d+)")
_DIGITS = re.compile(r"[0-9]+")
_DECIMAL = re.compile(r"[0-9]+(?:\.[0-9]+)?")


# ----------------------------------------------------------------- small helpers
def is_num(s: Optional[str]) -> bool:
    """A plain decimal number ("12", "12.5"; no sign, no exponent)."""
    t = (s or "").strip()
    return bool(t) and _DECIMAL.fullmatch(t) is not None


def normalize_taxid(val: Optional[str]) -> str:
    """The first run of digits ("taxid:562.1" -> "562"), or ""."""
    m = _DIGITS.search(val or "")
    return m.group(0) if m else ""


def parse_lineage_string(lineage: str) -> Dict[str, str]:
    """'rank:name; ...' -> {rank: name} over RANKS (later parts win; unknown labels and empty
    names are skipped)."""
    got: Dict[str, str] = {}
    for part in (lineage or "").split(";"):
        label, sep, name = part.strip().partition(":")
        rank = _LABEL_RANK.get(label.strip().lower()) if sep else None
        if rank and name.strip():
            got[rank] = name.strip()
    return got


def _fasta_records(path: str):
    """(first header word, stripped sequence lines) per record."""
    name, lines = None, []
    with open(path) as fh:
        for ln in fh:
            if ln.startswith(">"):
                if name is not None:
                    yield name, lines
                name, lines = ln[1:].strip().split()[0], []
            else:
                lines.append(ln.strip())
    if name is not None:
        yield name, lines


def fasta_lengths(paths: Iterable[Optional[str]]) -> Dict[str, int]:
    """Sequence length per record name over several files (the first file naming it wins)."""
    out: Dict[str, int] = {}
    for p in paths:
        if p and os.path.isfile(p):
            for name, lines in _fasta_records(p):
                if name not in out:
                    out[name] = sum(map(len, lines))
    return out


def fasta_md5(path: Optional[str]) -> Dict[str, str]:
    """MD5 of each record's concatenated sequence lines (eval_cami.py's contig pairing key)."""
    out: Dict[str, str] = {}
    if path and os.path.isfile(path):
        for name, lines in _fasta_records(path):
            out[name] = hashlib.md5("".join(lines).encode()).hexdigest()
    return out


fasta_hashes = fasta_md5


# ------------------------------------------------------------- taxonkit, restated
class Taxonomy:
    """The taxdump eval_cami's taxonkit calls read (--taxdb), parsed on first use."""

    def __init__(self, taxdb: str):
        self.taxdb = taxdb
        self._dump: Optional[TaxDump] = None
        self._tried = False

    def _load(self) -> Optional[TaxDump]:
        if not self._tried:
            self._tried = True
            names, nodes = (os.path.join(self.taxdb, f) for f in ("names.dmp", "nodes.dmp"))
            if os.path.isfile(names) and os.path.isfile(nodes):
                self._dump = TaxDump(names, nodes, all_names=True)
        return self._dump

    def name2taxid(self, names: Iterable[str]) -> Dict[str, str]:
        want = [n for n in names if n]
        d = self._load() if want else None
        return {} if d is None else {n: t for n, t in _name2taxid(d, want).items() if is_num(t)}

    def taxpath(self, taxids: Iterable[str]) -> Dict[str, Tuple[str, str]]:
        want = [t for t in taxids if t]
        d = self._load() if want else None
        return {} if d is None else _reformat(d, want, fmt_ranks=EVAL_FORMAT_RANKS)

    def rank_ids(self, taxids: Iterable[str]) -> Dict[str, List[str]]:
        """taxid -> the 7 rank taxids of its reformat path."""
        return {t: ids.split("|") for t, (_, ids) in self.taxpath(taxids).items()}


# --------------------------------------------------------------------- id map
class IdMap(dict):
    """Identifier -> TaxID over detailed_taxonomy.tsv (eval_cami.py:145-165): every token is
    entered with and without its version suffix, the first row naming a token wins; tokens
    come from the GCF / GCA columns, the Identifiers column split on [;|, whitespace], and
    GCF/GCA or accession patterns anywhere in the row."""

    _SPLIT = re.compile(r"[;|,\s]+")

    def add(self, tok: str, taxid: str):
        tok = (tok or "").strip()
        if tok:
            self.setdefault(tok, taxid)
            head, dot, _ = tok.partition(".")
            if dot:
                self.setdefault(head, taxid)

    @classmethod
    def from_file(cls, path: str) -> "IdMap":
        m = cls()
        if not os.path.isfile(path):
            return m
        with open(path, newline="") as fh:
            for row in csv.DictReader(fh, delimiter="\t"):
                taxid = normalize_taxid(row.get("TaxID") or "")
                if not taxid:
                    continue
                toks = [(row.get(k) or "").strip() for k in ("GCF", "GCA")]
                toks += cls._SPLIT.split(row.get("Identifiers") or "")
                for v in filter(None, row.values()):
                    toks += _GCFA.findall(v) + _ACC.findall(v)
                for t in toks:
                    m.add(t, taxid)
        return m

    def taxid_of_target(self, target: str) -> str:
        """A PAF target through the map: the whole name, the part before '|', that without
        its version."""
        head = target.split("|", 1)[0]
        for key in (target, head) + ((head.split(".", 1)[0],) if "." in head else ()):
            t = normalize_taxid(self.get(key, "")) if key in self else ""
            if t:
                return t
        return ""


def load_id_map(path: str) -> IdMap:
    return IdMap.from_file(path)


# ------------------------------------------------------------------- profiles
class Profile:
    """Abundance per taxid for each of the seven ranks (percent)."""

    def __init__(self):
        self.tables: List[collections.Counter] = [collections.Counter() for _ in RANKS]

    def __getitem__(self, rank: str) -> collections.Counter:
        return self.tables[RANK_SLOT[rank]]

    def add(self, rank: str, taxid: str, value: float):
        self.tables[RANK_SLOT[rank]][taxid] += value

    @property
    def empty(self) -> bool:
        return not any(self.tables)

    def normalise(self):
        """Each rank's values as percentages of the rank total."""
        for tab in self.tables:
            tot = sum(tab.values())
            if tot > 0:
                for k in list(tab):
                    tab[k] = 100.0 * tab[k] / tot


# column roles of headed profile / mapping tables and the header names that fill them
_ROLES = {
    "taxid": ("taxid", "taxon_id", "ncbi_taxid", "ncbi_tax_id"),
    "rank": ("rank",),
    "perc": ("percentage", "abundance", "rel_abundance", "fraction_total_reads"),
    "taxpath": ("taxpath",),
    "taxpathsn": ("taxpathsn", "taxpath_sn", "taxpath_names", "lineage"),
}


class _Table:
    """A headed tab-separated table with its columns located by role."""

    def __init__(self, header: List[str], rows: List[List[str]]):
        self.h = [c.strip().lower() for c in header]
        self.rows = rows
        self.col = {role: next((self.h.index(n) for n in names if n in self.h), -1) for role, names in _ROLES.items()}

    def scale(self) -> float:
        """Fractions / abundances are scaled to percent."""
        name = self.h[self.col["perc"]]
        return 100.0 if ("abundance" in name or "fraction" in name) else 1.0


def _cami_rows(lines: Sequence[str], prof: Profile, tax: Taxonomy) -> bool:
    """Leading CAMI rows (TAXID, RANK, TAXPATH, TAXPATHSN, PERCENTAGE; comment and '@' lines
    skipped) until the first other row; True when any row counted."""
    counted = False
    for ln in lines:
        if not ln.strip() or ln[0] in "#@":
            continue
        f = ln.rstrip("\n").split("\t")
        if len(f) < 5 or not is_num(f[0]):
            break
        rank = f[1].strip().lower()
        if rank in RANK_SLOT:
            try:
                prof.add(rank, f[0], float(f[4]))
                counted = True
            except ValueError:
                pass
    return counted


def _by_taxid(t: _Table, prof: Profile, tax: Taxonomy):
    c, mul = t.col, t.scale()
    for f in t.rows:
        try:
            taxid, rank, val = normalize_taxid(f[c["taxid"]]), f[c["rank"]].strip().lower(), float(f[c["perc"]]) * mul
        except (ValueError, IndexError):
            continue
        if rank in RANK_SLOT and taxid:
            prof.add(rank, taxid, val)


def _by_taxpath(t: _Table, prof: Profile, tax: Taxonomy):
    """The rank's taxid is the rank-th element of TAXPATH once empty and NA parts are
    dropped (the reference's indexing, kept)."""
    c, mul = t.col, t.scale()
    for f in t.rows:
        try:
            rank = f[c["rank"]].strip().lower()
            ids = [x for x in f[c["taxpath"]].strip().split("|") if x and x != "NA"]
            slot = RANK_SLOT.get(rank, -1)
            if 0 <= slot < len(ids):
                prof.add(rank, ids[slot], float(f[c["perc"]]) * mul)
        except (ValueError, IndexError):
            continue


def _by_names(t: _Table, prof: Profile, tax: Taxonomy):
    """TAXPATHSN names mapped through name2taxid, the rank-th name per row."""
    c, mul = t.col, t.scale()
    picked = []   # (rank, name at the rank slot or None, row)
    for f in t.rows:
        try:
            rank = f[c["rank"]].strip().lower()
            names = [p.strip() for p in f[c["taxpathsn"]].split("|")]
        except IndexError:
            continue
        slot = RANK_SLOT.get(rank, -1)
        picked.append((rank, names[slot] if 0 <= slot < len(names) else None, f))
    tids = tax.name2taxid({n for _, n, _ in picked if n})
    for rank, name, f in picked:
        tid = tids.get(name) if name is not None else None
        if tid:
            try:
                prof.add(rank, tid, float(f[c["perc"]]) * mul)
            except (ValueError, IndexError):
                pass


# (applies-to-table, reader) in the reference's order of preference (eval_cami.py:193-233)
_PROFILE_READERS: List[Tuple[Callable[[_Table], bool], Callable]] = [
    (lambda t: min(t.col["taxid"], t.col["rank"], t.col["perc"]) >= 0, _by_taxid),
    (lambda t: t.col["rank"] >= 0 and t.col["perc"] >= 0 and t.col["taxpath"] >= 0, _by_taxpath),
    (lambda t: t.col["rank"] >= 0 and t.col["perc"] >= 0 and t.col["taxpathsn"] >= 0, _by_names),
]


def parse_cami_like(lines: Sequence[str], tax: Taxonomy) -> Profile:
    """A profile file's lines: CAMI rows, else a headed table read by the first reader whose
    columns it has."""
    prof = Profile()
    if _cami_rows(lines, prof, tax):
        return prof
    body = list(csv.reader([ln for ln in lines if ln.strip() and ln[0] not in "#@"], delimiter="\t"))
    if not body:
        return prof
    t = _Table(body[0], body[1:])
    for applies, read in _PROFILE_READERS:
        if applies(t):
            read(t, prof, tax)
            break
    return prof


def load_profile_any(path: str, tax: Taxonomy) -> Profile:
    if not os.path.isfile(path):
        return Profile()
    with open(path) as fh:
        return parse_cami_like(fh.readlines(), tax)


def profile_from_contigs(contig_tid: Dict[str, str], lengths: Dict[str, int], tax: Taxonomy) -> Profile:
    """Length-weighted (1 bp when the FASTA lacks the contig) rank composition of contig
    TaxIDs through their reformat paths; an empty rank id is a taxon of its own, NA is
    skipped (eval_cami.py:306-329)."""
    prof = Profile()
    tids = {c: normalize_taxid(t) for c, t in contig_tid.items()}
    tids = {c: t for c, t in tids.items() if t}
    if not tids:
        return prof
    paths = tax.rank_ids(set(tids.values()))
    for contig, tid in tids.items():
        ids = paths.get(tid)
        if ids is None:
            continue
        w = lengths.get(contig, 1)
        for slot, rank_id in enumerate(ids[:len(RANKS)]):
            if rank_id != "NA":
                prof.tables[slot][rank_id] += w
    prof.normalise()
    return prof


profiles_from_contig_maps = profile_from_contigs


# --------------------------------------------------------------------- metrics
def _aligned(a: Dict[str, float], b: Dict[str, float]) -> Tuple[np.ndarray, np.ndarray]:
    keys = list(set(a) | set(b))
    return (np.fromiter((a.get(k, 0.0) for k in keys), np.float64, len(keys)),
            np.fromiter((b.get(k, 0.0) for k in keys), np.float64, len(keys)))


def l1_and_braycurtis(a: Dict[str, float], b: Dict[str, float]) -> Tuple[float, float]:
    """Half the L1 distance (percentage points) and the Bray-Curtis dissimilarity (%)."""
    va, vb = _aligned(a, b)
    if len(va) == 0:
        return 0.0, 0.0
    l1 = 0.5 * math.fsum(np.abs(va - vb))
    tot = math.fsum(va) + math.fsum(vb)
    bc = 1.0 - 2.0 * math.fsum(np.minimum(va, vb)) / (tot if tot > 0 else 1.0)
    return l1, 100.0 * bc


def prf_presence(a: Dict[str, float], b: Dict[str, float], thr: float = 0.1):
    """Presence at >= thr: precision, recall, F1 (%), TP, FP, FN."""
    pa = {k for k, v in a.items() if v >= thr}
    pb = {k for k, v in b.items() if v >= thr}
    tp, fp, fn = len(pa & pb), len(pa - pb), len(pb - pa)
    p = tp / (tp + fp) if tp + fp else 0.0
    r = tp / (tp + fn) if tp + fn else 0.0
    f = 2 * p * r / (p + r) if p + r else 0.0
    return 100.0 * p, 100.0 * r, 100.0 * f, tp, fp, fn


# ------------------------------------------------------------ truth mapping
def load_gt_contigs(gt_file: str) -> Dict[str, str]:
    """Contig -> TaxID of a CAMI gsa_mapping (tab / comma / whitespace separated): the
    TaxID-like column, else the last TAXPATH id, else the first numeric field
    (eval_cami.py:243-303).  The first line is sniffed as plain text, as there."""
    if not gt_file or not os.path.isfile(gt_file):
        return {}
    with open(gt_file) as fh:
        first = fh.readline()
    opener = (lambda: gzip.open(gt_file, "rt")) if gt_file.endswith(".gz") else (lambda: open(gt_file))
    with opener() as fh:
        if "\t" in first or "," in first:
            rows = list(csv.reader(fh, delimiter="\t" if "\t" in first else ","))
            header, rows = rows[0], rows[1:]
        else:
            next(fh)
            header = first.strip().split()
            rows = [ln.split() for ln in (x.strip() for x in fh) if ln]
    h = [c.strip().lstrip("#").lower() for c in header]
    contig_cols = [i for i, k in enumerate(h) if any(x in k for x in ("contig", "sequence", "scaffold"))]
    tax_cols = [i for i, k in enumerate(h) if "tax" in k and "path" not in k]
    tax_cols += [i for i, k in enumerate(h) if k in ("ncbi_taxid", "ncbi_tax_id", "taxid", "tax_id", "species_taxid",
                                                      "genome_taxid")]
    ci = contig_cols[0] if contig_cols else 0
    out: Dict[str, str] = {}
    if tax_cols:
        ti = tax_cols[0]
        for f in rows:
            if len(f) > max(ci, ti):
                tid = normalize_taxid((f[ti] or "").strip())
                if tid:
                    out[f[ci]] = tid
    elif "taxpath" in h:
        pi = h.index("taxpath")
        for f in rows:
            ids = [x for x in f[pi].split("|") if x and x != "NA"]
            tid = normalize_taxid(ids[-1]) if ids else ""
            if tid:
                out[f[ci]] = tid
    else:
        for f in rows:
            num = next((x for x in f[1:] if is_num(x)), None)
            if num is not None:
                out[f[0]] = normalize_taxid(num)
    return out


# ----------------------------------------------------------- PAF helpers
def _paf_rows(path: str):
    with open(path) as fh:
        for ln in fh:
            if ln.strip() and ln[0] != "#":
                yield ln.rstrip("\n").split("\t")


def paf_firsthit_q2t(paf_path: Optional[str]) -> Dict[str, str]:
    """Each query's first PAF target."""
    out: Dict[str, str] = {}
    if paf_path and os.path.isfile(paf_path):
        for f in _paf_rows(paf_path):
            if len(f) >= 6:
                out.setdefault(f[0], f[5])
    return out


def besthit_map_from_paf(paf_path: str, min_cov: float = 0.95, min_id: float = 0.95) -> Dict[str, str]:
    """Per query the target of its line with the most matches among lines covering >= min_cov
    of the query at >= min_id identity (the first such line on ties)."""
    best: Dict[str, Tuple[int, str]] = {}
    for f in _paf_rows(paf_path):
        if len(f) < 12:
            continue
        qlen, qs, qe, nm, al = int(f[1]), int(f[2]), int(f[3]), int(f[9]), int(f[10])
        if (qe - qs) / qlen < min_cov if qlen > 0 else True:
            continue
        if (nm / al if al > 0 else 0.0) < min_id:
            continue
        if f[0] not in best or nm > best[f[0]][0]:
            best[f[0]] = (nm, f[5])
    return {q: t for q, (_, t) in best.items()}


# --------------------------------------------------------- contig resolution
class _Classified:
    """classified_sequences.tsv rows: per query its lineage names (if any), TaxID column and
    target column (header names matched case-insensitively)."""

    def __init__(self, path: str):
        self.lineage: Dict[str, Dict[str, str]] = {}
        self.extra: Dict[str, Tuple[Optional[str], Optional[str]]] = {}   # query -> (taxid, target)
        if not os.path.isfile(path):
            return
        with open(path, encoding="utf-8", errors="ignore") as fh:
            rd = csv.DictReader(fh, delimiter="\t")
            raw = rd.fieldnames or []
            low = {(x or "").strip().lower(): x for x in reversed(raw)}   # first header of a name wins
            k_q, k_tax, k_lin = low.get("query"), low.get("taxid"), low.get("lineage")
            k_tgt = low.get("target", low.get("tname"))
            for row in rd:
                q = row.get(k_q) if k_q else (row.get("Query") or row.get("qname") or row.get("q"))
                if not q:
                    continue
                lin = parse_lineage_string(row.get(k_lin, "") if k_lin else row.get("Lineage", ""))
                if lin:
                    self.lineage[q] = lin
                self.extra[q] = (row.get(k_tax) if k_tax else row.get("TaxID"),
                                 row.get(k_tgt) if k_tgt else (row.get("Target") or row.get("tname")))


def _from_lineage(c: _Classified, tax: Taxonomy, idmap: IdMap, paf: Optional[str]) -> Dict[str, str]:
    names = {n for lin in c.lineage.values() for n in lin.values() if n}
    n2t = tax.name2taxid(names) if names else {}
    out = {}
    for q, lin in c.lineage.items():
        for rank in reversed(RANKS):   # most specific rank whose name resolves
            tid = normalize_taxid(n2t.get(lin.get(rank) or "", ""))
            if tid:
                out[q] = tid
                break
    return out


def _from_taxid_column(c, tax, idmap, paf):
    return {q: t for q, (raw, _) in c.extra.items() if (t := normalize_taxid(raw or ""))}


def _from_target_column(c, tax, idmap, paf):
    return {q: t for q, (_, tg) in c.extra.items() if (tg or "").strip() and (t := idmap.taxid_of_target(tg.strip()))}


def _from_first_paf_hit(c, tax, idmap, paf):
    return {q: t for q, tg in paf_firsthit_q2t(paf).items() if (t := idmap.taxid_of_target(tg))}


_RESOLVERS = (_from_lineage, _from_taxid_column, _from_target_column, _from_first_paf_hit)


def preds_taxid_from_classified(classified_tsv: str, tax: Taxonomy, idmap: IdMap, paf_path: Optional[str]) -> Dict[str, str]:
    """Most specific resolvable TaxID per classified contig: its lineage names, else a TaxID
    column, else its target through the id map, else its first PAF hit through the id map
    (eval_cami.py:388-483)."""
    c = _Classified(classified_tsv)
    out: Dict[str, str] = {}
    for resolve in _RESOLVERS:
        for q, t in resolve(c, tax, idmap, paf_path).items():
            out.setdefault(q, t)
    return out


# ------------------------------------------------------------- contig pairing
def _pair_by_name(pred, gt, ctx, log):
    return [(q, t, gt[q]) for q, t in pred.items() if q in gt]


def _pair_by_md5(pred, gt, ctx, log):
    if not ctx["have_fasta"]:
        return []
    ph, by_hash = fasta_md5(ctx["pred_fasta"]), collections.defaultdict(list)
    for name, h in fasta_md5(ctx["gt_fasta"]).items():
        by_hash[h].append(name)
    pairs = [(q, pred[q], gt[t]) for q in pred if ph.get(q) for t in by_hash.get(ph[q], ()) if gt.get(t)]
    print(f"[DEBUG] MD5‑paired contigs: {len(pairs)}", file=log)
    return pairs


def _pair_by_minimap2(pred, gt, ctx, log):
    if not ctx["have_fasta"] or shutil.which("minimap2") is None:
        return []
    paf = os.path.join(ctx["outdir"], "pred_vs_truth.paf")
    with open(paf, "w") as w:
        subprocess.run(["minimap2", "-x", "asm10", "--secondary=no", "-t", str(ctx["threads"]), ctx["gt_fasta"],
                        ctx["pred_fasta"]], check=True, stdout=w)
    pairs = [(q, pred[q], gt[t]) for q, t in besthit_map_from_paf(paf).items() if pred.get(q) and gt.get(t)]
    print(f"[DEBUG] minimap‑paired contigs: {len(pairs)}", file=log)
    return pairs


def rank_accuracy(pairs, tax: Taxonomy) -> Dict[str, dict]:
    """Per rank: pairs whose predicted and truth paths both have a (non-NA) id there, and how
    many of those agree."""
    paths = tax.rank_ids({p for _, p, _ in pairs} | {g for _, _, g in pairs})
    out = {}
    for slot, rank in enumerate(RANKS):
        n = ok = 0
        for _, p, g in pairs:
            pv, gv = paths.get(p), paths.get(g)
            if not pv or not gv or slot >= len(pv) or slot >= len(gv) or "NA" in (pv[slot], gv[slot]):
                continue
            n += 1
            ok += pv[slot] == gv[slot]
        out[rank] = {"n": n, "acc": 100.0 * ok / n if n else 0.0, "correct": ok}
    return out


def _write_tsv(path: str, header, rows):
    with open(path, "w", newline="") as w:
        wr = csv.writer(w, delimiter="\t")
        wr.writerow(header)
        wr.writerows(rows)


def eval_contigs(pred_file: str, gt_files: Sequence[str], tax: Taxonomy, outdir: str, pred_fasta=None, gt_fasta=None,
                 threads: int = 8, taxmap_path: str = "", paf_path: Optional[str] = None, log=sys.stderr) -> dict:
    """Contig-level accuracy; writes contigs_exact.tsv / contigs_per_rank.tsv when any pair
    exists, else removes stale ones (eval_cami.py:486-568)."""
    pred = preds_taxid_from_classified(pred_file, tax, load_id_map(taxmap_path), paf_path)
    gt: Dict[str, str] = {}
    for g in gt_files:
        if g:
            gt.update(load_gt_contigs(g))
    print(f"[DEBUG] loaded pred contigs with TaxID: {len(pred)}", file=log)
    print(f"[DEBUG] loaded truth contigs with TaxID: {len(gt)}", file=log)
    ctx = {"pred_fasta": pred_fasta, "gt_fasta": gt_fasta, "outdir": outdir, "threads": threads,
           "have_fasta": bool(pred_fasta and gt_fasta and os.path.isfile(pred_fasta) and os.path.isfile(gt_fasta))}
    pairs: list = []
    for strategy in (_pair_by_name, _pair_by_md5, _pair_by_minimap2):
        pairs = strategy(pred, gt, ctx, log)
        if pairs:
            break
    usable, exact = len(pairs), sum(p == g for _, p, g in pairs)
    per_rank = rank_accuracy(pairs, tax)
    files = (os.path.join(outdir, "contigs_exact.tsv"), os.path.join(outdir, "contigs_per_rank.tsv"))
    if usable:
        _write_tsv(files[0], ["metric", "value"], [["usable_pairs", usable], ["exact_taxid_matches", exact],
                                                   ["exact_taxid_accuracy_percent", 100.0 * exact / usable]])
        _write_tsv(files[1], ["rank", "n", "correct", "accuracy_percent"],
                   [[r, m["n"], m["correct"], f"{m['acc']:.4f}"] for r, m in per_rank.items()])
    else:
        for f in files:
            if os.path.exists(f):
                os.remove(f)
    return {"usable_pairs": usable, "exact": exact, "per_rank": per_rank, "pred_n": len(pred), "gt_n": len(gt)}


# ----------------------------------------------------------------------- CLI
_DEFAULTS = {  # eval_cami.py's layout
    "pred_profile": "/data/hymet_out/sample_0/hymet.sample_0.cami.tsv",
    "truth_profile": "/data/cami/sample_0/taxonomic_profile_0.txt",
    "pred_contigs": "/data/hymet_out/sample_0/work/classified_sequences.tsv",
    "pred_fasta": "/data/cami/sample_0.fna",
    "truth_fasta": "/data/cami/sample_0/2017.12.29_11.37.26_sample_0/contigs/anonymous_gsa.fasta",
    "taxdb": "/data/HYMET/taxonomy_files",
    "taxmap": "/data/HYMET/data/detailed_taxonomy.tsv",
    "paf": "/data/hymet_out/sample_0/work/resultados.paf",
    "outdir": "/data/hymet_out/sample_0/eval",
}
_GT_DIR = "/data/cami/sample_0/2017.12.29_11.37.26_sample_0/contigs/"


def main(argv: Optional[Sequence[str]] = None) -> int:
    """tools/eval_cami.py's command line: same flags, output files and stdout lines."""
    import argparse
    ap = argparse.ArgumentParser(description="Evaluate HYMET vs CAMI ground truth (post-processing only; classifier unchanged).")
    for flag in ("pred-profile", "truth-profile", "pred-contigs"):
        ap.add_argument("--" + flag, default=_DEFAULTS[flag.replace("-", "_")])
    ap.add_argument("--truth-contigs", default="")
    for flag in ("pred-fasta", "truth-fasta", "taxdb", "taxmap", "paf", "outdir"):
        ap.add_argument("--" + flag, default=_DEFAULTS[flag.replace("-", "_")])
    ap.add_argument("--presence-thresh", type=float, default=0.1)
    ap.add_argument("--threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "8")))
    a = ap.parse_args(argv)
    pathlib.Path(a.outdir).mkdir(parents=True, exist_ok=True)
    gt_files = [a.truth_contigs] if a.truth_contigs else [_GT_DIR + "gsa_mapping_new.tsv", _GT_DIR + "gsa_mapping.tsv"]
    tax = Taxonomy(a.taxdb)
    pred, truth = load_profile_any(a.pred_profile, tax), load_profile_any(a.truth_profile, tax)
    lens = fasta_lengths([a.pred_fasta, a.truth_fasta]) if (pred.empty or truth.empty) else {}
    if pred.empty:
        print("[INFO] Rebuilding predicted profile from per‑contig classifications.", file=sys.stderr)
        pred = profile_from_contigs(preds_taxid_from_classified(a.pred_contigs, tax, load_id_map(a.taxmap), a.paf),
                                    lens, tax)
    if truth.empty:
        print("[INFO] Rebuilding truth profile from contig mapping.", file=sys.stderr)
        gt: Dict[str, str] = {}
        for g in gt_files:
            gt.update(load_gt_contigs(g))
        truth = profile_from_contigs(gt, lens, tax)
    table = {r: l1_and_braycurtis(pred[r], truth[r]) + prf_presence(pred[r], truth[r], a.presence_thresh) for r in RANKS}
    _write_tsv(os.path.join(a.outdir, "profile_summary.tsv"),
               ["rank", "L1_total_variation_pctpts", "BrayCurtis_pct", "Precision_%", "Recall_%", "F1_%", "TP", "FP", "FN"],
               [[r, f"{v[0]:.4f}", f"{v[1]:.4f}", f"{v[2]:.2f}", f"{v[3]:.2f}", f"{v[4]:.2f}", *v[5:]] for r, v in table.items()])
    print("# Profile-level metrics (per rank)")
    for r, (l1, bc, pr, rc, f1, tp, fp, fn) in table.items():
        print(f"{r:14s}  L1={l1:.3f}  BC={bc:.3f}%  P/R/F1={pr:.1f}/{rc:.1f}/{f1:.1f}% (TP={tp}, FP={fp}, FN={fn})")
    print("\n# Contig-level accuracy")
    c = eval_contigs(a.pred_contigs, gt_files, tax, a.outdir, pred_fasta=a.pred_fasta, gt_fasta=a.truth_fasta,
                     threads=a.threads, taxmap_path=a.taxmap, paf_path=a.paf)
    usable, exact = c["usable_pairs"], c["exact"]
    print(f"Exact TaxID: {exact}/{usable} ({(100.0 * exact / usable if usable else 0.0):.2f}%)")
    for r in RANKS:
        m = c["per_rank"][r]
        print(f"{r:14s}  n={m['n']:<8d}  acc={m['acc']:.2f}%")
    info = [("pred_profile_path", a.pred_profile), ("truth_profile_path", a.truth_profile),
            ("pred_contigs_path", a.pred_contigs)]
    with open(os.path.join(a.outdir, "_debug_info.txt"), "w") as w:
        w.writelines(f"{k}: {v}\n" for k, v in info)
        w.write("truth_contigs_paths:\n  " + "\n  ".join(g for g in gt_files if g) + "\n")
        w.writelines(f"{k}: {v}\n" for k, v in (("pred_fasta", a.pred_fasta), ("truth_fasta", a.truth_fasta),
                                               ("taxdb", a.taxdb), ("taxmap", a.taxmap), ("paf", a.paf)))
    for name in ("profile_summary.tsv", "contigs_exact.tsv", "contigs_per_rank.tsv"):
        print(("\n" if name == "profile_summary.tsv" else "") + f"[WROTE] {os.path.join(a.outdir, name)}")
    print(f"[WROTE] debug: {os.path.join(a.outdir, '_debug_info.txt')}")
    return 0

"""Classify stage: drop-in for scripts/classification_cami.py and scripts/classification.py
(SURVEY.md §3.5, §8a rows C1-C9).

Host (this module): the string work the reference does per distinct identifier --
identifier -> TaxID maps (regex / versionless keys for the CAMI variant, exact ';'-split
keys for the legacy one), lineage parsing, target -> taxid resolution (cached per target),
PAF parsing -- turned into integer arrays once.  Device (libhymet_gpu.so, lca.hip): the
global per-target line counts and the per-query weighted LCA in double precision.
Output bytes equal the reference's csv.writer output (CRLF, minimal quoting, "%.4f").
"""
from __future__ import annotations

import csv
import gzip
import io
import re
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np

from ._lib import ptr

csv.field_size_limit(1 << 30)

RANKS = ["superkingdom", "phylum", "class", "order", "family", "genus", "species", "strain"]
_ALIAS = {
    "domain": "superkingdom", "kingdom": "superkingdom", "sk": "superkingdom", "k": "superkingdom",
    "phylum": "phylum", "p": "phylum", "class": "class", "c": "class", "order": "order", "o": "order",
    "family": "family", "f": "family", "genus": "genus", "g": "genus", "species": "species", "s": "species",
    "subspecies": "strain", "ss": "strain", "strain": "strain",
}
_GCFA = re.compile(r"GC[AF]_\d+(?:\.\d+)?(?:_PRJ[A-Z]+\d+)?")                                 # classification_cami.py:27
_ACC = re.compile(r"(NC_\d+\.\d+|NZ_[A-Z]{2}\d+\.\d+|NZ_[A-Z]{5}\d+\.\d+|CP\d+\.\d+|CM\d+\.\d+|[A-Z]{2}_\d+\.\d+)")  # :28
_SPLIT_IDS = re.compile(r"[;|,\s]+")
_SPLIT_LIN = re.compile(r"[;|]+")
_HEAD = re.compile(r"[|\s]+")

CAMI, LEGACY = 0, 1


# ------------------------------------------------------------------ taxonomy maps
def add_alias(m: Dict[str, str], tok, tax) -> None:
    """The identifier rule shared by classification_cami.py:84-93 and build_id_map.py:20-24:
    a stripped, non-empty token maps to its TaxID unless an earlier row claimed it, and so
    does its versionless form (the part before the first '.')."""
    tok = (tok or "").strip()
    if not tok:
        return
    m.setdefault(tok, tax)
    if "." in tok:
        m.setdefault(tok.split(".", 1)[0], tax)


class TaxonomyMap:
    """identifier -> TaxID string.  CAMI variant: classification_cami.py:63-102 (first row
    wins, versionless aliases, GCF/GCA and accession regex hits from every column); legacy:
    classification.py:14-25 (exact ';'-split identifiers, last row wins)."""

    def __init__(self, path, variant: int):
        self.variant = variant
        self.m: Dict[str, str] = {}
        if variant == CAMI:
            self._load_cami(path)
        else:
            with open(path, "r") as f:
                for row in csv.DictReader(f, delimiter="\t"):
                    tax = row["TaxID"]
                    for ident in row["Identifiers"].split(";"):
                        c = ident.strip()
                        if c:
                            self.m[c] = tax

    def _add(self, tok, tax):
        add_alias(self.m, tok, tax)

    def _load_cami(self, path):
        with open(path, "r", newline="") as f:
            rd = csv.DictReader(f, delimiter="\t")
            if "TaxID" not in rd.fieldnames:
                raise RuntimeError("TaxID column not found in taxonomy file")
            for row in rd:
                tax = (row.get("TaxID") or "").strip()
                if not tax:
                    continue
                vals = list(row.values())
                for v in vals:
                    if v:
                        for acc in _GCFA.findall(v):
                            self._add(acc, tax)
                ids = row.get("Identifiers") or ""
                if ids:
                    for tok in _SPLIT_IDS.split(ids):
                        if tok.strip():
                            self._add(tok, tax)
                for v in [ids] + [row.get(k) or "" for k in row.keys()]:
                    if v:
                        for acc in _ACC.findall(v):
                            self._add(acc, tax)

    def lookup(self, tname: str) -> Optional[str]:
        if self.variant == LEGACY:
            return self.m.get(tname)
        cands: List[str] = []

        def add(x):
            if x and x not in cands:
                cands.append(x)
            if x and "." in x:
                xv = x.split(".", 1)[0]
                if xv not in cands:
                    cands.append(xv)

        add(tname)
        add(_HEAD.split(tname)[0])
        for g in _GCFA.findall(tname):
            add(g)
        for a in _ACC.findall(tname):
            add(a)
        for c in cands:
            t = self.m.get(c)
            if t:
                return t
        return None


def _names_cami(raw: str) -> List[str]:
    """classification_cami.py:104-156 -- names per RANKS ('' = absent)."""
    out = [""] * 8
    if not raw:
        return out
    s = raw.strip()
    sep = ":" if ":" in s else ("__" if "__" in s else None)
    if sep:
        for part in _SPLIT_LIN.split(s):
            part = part.strip()
            if not part or sep not in part:
                continue
            rk, nm = part.split(sep, 1)
            rk = _ALIAS.get(rk.strip().lower())
            nm = nm.strip()
            if rk and nm:
                out[RANKS.index(rk)] = nm
        return out
    seq = [p.strip() for p in _SPLIT_LIN.split(s) if p.strip() and p.strip().upper() != "NA"]
    for i, nm in enumerate(seq[:8]):
        out[i] = nm
    return out


class Hierarchy:
    """TaxID -> per-rank labels, interned to integer ids for the device.
    CAMI: names (classification_cami.py:158-174).  Legacy: raw lineage string and, per rank,
    the first ';'-part starting with 'rank:' (classification.py:118-124)."""

    def __init__(self, path, variant: int):
        self.variant = variant
        self.rows: Dict[str, object] = {}
        if variant == CAMI:
            with open(path, "r", newline="") as f:
                rd = csv.DictReader(f, delimiter="\t")
                if "TaxID" not in rd.fieldnames or "Lineage" not in rd.fieldnames:
                    raise RuntimeError("Hierarchy file must have TaxID and Lineage columns")
                for row in rd:
                    tid = (row.get("TaxID") or "").strip()
                    lin = (row.get("Lineage") or "").strip()
                    if tid:
                        self.rows[tid] = _names_cami(lin)
        else:
            with open(path, "r") as f:
                for row in csv.DictReader(f, delimiter="\t"):
                    self.rows[row["TaxID"]] = row["Lineage"].strip()

    def labels(self, tid: str) -> Optional[List[str]]:
        v = self.rows.get(tid)
        if v is None:
            return None
        if self.variant == CAMI:
            return v
        parts = v.split(";")
        out = [""] * 8
        for r, rank in enumerate(RANKS):
            for p in parts:
                if p.startswith(f"{rank}:"):
                    out[r] = p
                    break
        return out


def legacy_level(lineage: str) -> str:
    """classification.py:61-81 determine_taxonomic_level."""
    cur = None
    for part in lineage.split(";"):
        part = part.strip()
        if ":" in part:
            rank = part.split(":", 1)[0].strip().lower()
            if rank in RANKS and (cur is None or RANKS.index(rank) > RANKS.index(cur)):
                cur = rank
    return cur if cur is not None else "root"


# ------------------------------------------------------------------------- PAF input
@dataclass
class PafTable:
    """PAF lines as arrays in file order (only what the classifiers read)."""
    queries: List[str]            # first-appearance order
    line_q: np.ndarray            # int32 query index per line
    targets: List[str]
    line_t: np.ndarray            # int32 target index
    line_blen: np.ndarray         # int64 (col 11, 0 on parse failure)
    line_qlen: np.ndarray         # int64 (col 2)
    line_exact: np.ndarray        # uint8 (legacy: query == target and cov >= 0.99)

    @property
    def n_lines(self):
        return len(self.line_q)


def read_paf(path, variant: int) -> PafTable:
    """classification_cami.py:181-208 / classification.py:37-59 line filters."""
    op = gzip.open(path, "rt") if str(path).endswith(".gz") and variant == CAMI else open(path, "r")
    qidx: Dict[str, int] = {}
    tidx: Dict[str, int] = {}
    lq, lt, lb, ll, le = [], [], [], [], []
    with op as f:
        for line in f:
            if variant == CAMI:
                if not line or line.startswith("#"):
                    continue
                parts = line.rstrip("\n").split("\t")
                if len(parts) < 11:
                    continue
                try:
                    qlen = int(parts[1])
                    blen = int(parts[10])
                except Exception:
                    qlen = blen = 0
                exact = 0
            else:
                parts = line.strip().split("\t")
                if len(parts) < 11:
                    continue
                qlen = int(parts[1])   # raises like the reference on a non-integer
                blen = int(parts[10])
                cov = blen / qlen if qlen > 0 else 0
                exact = int(parts[0] == parts[5] and cov >= 0.99)
            q, t = parts[0], parts[5]
            lq.append(qidx.setdefault(q, len(qidx)))
            lt.append(tidx.setdefault(t, len(tidx)))
            lb.append(blen)
            ll.append(qlen)
            le.append(exact)
    return PafTable(list(qidx), np.array(lq, np.int32), list(tidx), np.array(lt, np.int32), np.array(lb, np.int64),
                    np.array(ll, np.int64), np.array(le, np.uint8))


# ---------------------------------------------------------------------- classifier
@dataclass
class LcaResult:
    queries: List[str]
    depth: np.ndarray       # -1: legacy exact shortcut, 0: Unknown/root
    names: np.ndarray       # (n_q, 8) label ids
    conf: np.ndarray
    tax: np.ndarray         # legacy exact shortcut taxid index


class Classifier:
    """Integer-encodes a taxonomy + hierarchy once; classifies PAF tables on the GPU."""

    def __init__(self, gpu, taxonomy, hierarchy, variant: int = CAMI):
        self.gpu, self.variant = gpu, variant
        self.tax = TaxonomyMap(taxonomy, variant)
        self.hier = Hierarchy(hierarchy, variant)
        self.label_id: Dict[str, int] = {}
        self.labels: List[str] = []
        self.taxids: List[str] = []
        self.tax_index: Dict[str, int] = {}
        self._tax_names: List[List[int]] = []
        self._in_hier: List[int] = []
        self._tcache: Dict[str, int] = {}
        self._dev: Dict[str, object] = {}

    def _taxid_index(self, tid: str) -> int:
        i = self.tax_index.get(tid)
        if i is not None:
            return i
        i = len(self.taxids)
        self.tax_index[tid] = i
        self.taxids.append(tid)
        labs = self.hier.labels(tid)
        self._in_hier.append(0 if labs is None else 1)
        ids = []
        for r in range(8):
            lab = labs[r] if labs else ""
            if lab:
                j = self.label_id.setdefault(lab, len(self.labels))
                if j == len(self.labels):
                    self.labels.append(lab)
                ids.append(j)
            else:
                ids.append(-1)
        self._tax_names.append(ids)
        return i

    def target_tax(self, targets: Sequence[str]) -> np.ndarray:
        out = np.full(len(targets), -1, np.int32)
        for k, t in enumerate(targets):
            v = self._tcache.get(t)
            if v is None:
                tid = self.tax.lookup(t)
                # CAMI: only truthy taxids count (_lookup_taxid :243-249); legacy: any key
                # present in the map counts, even an empty TaxID (classification.py:88-93)
                ok = (tid is not None) if self.variant == LEGACY else bool(tid)
                v = self._taxid_index(tid) if ok else -1
                self._tcache[t] = v
            out[k] = v
        return out

    def device_tables(self, target_names: Optional[Sequence[str]]):
        """The integer tables in HBM for the fused path: target -> taxid index for
        `target_names` (the index set's targets, cached per list), taxid -> 8 label ids,
        in-hierarchy flags, the label byte pool, and for the legacy variant each taxid's raw
        lineage and determine_taxonomic_level string (the exact-match shortcut's output).
        Rebuilt only when a new target list or new taxids / labels appear."""
        torch = self.gpu.torch

        def dev(a):
            return torch.from_numpy(np.ascontiguousarray(a)).to(self.gpu.dev)

        def pool(strs):
            bs = [x.encode() for x in strs]
            off = np.zeros(len(bs) + 1, np.int64)
            np.cumsum([len(b) for b in bs], out=off[1:])
            return dev(np.frombuffer(b"".join(bs) or b"\0", np.uint8).copy()), dev(off)

        d = self._dev
        if target_names is not None and d.get("targets_of") is not target_names:
            t_tax = self.target_tax(list(target_names))
            d["t_tax"] = dev(t_tax if len(t_tax) else np.full(1, -1, np.int32))
            d["targets_of"] = target_names
        sizes = (len(self.taxids), len(self.labels))
        if d.get("sizes") != sizes:
            d["tax_names"] = dev(np.array(self._tax_names if self._tax_names else [[-1] * 8], np.int32).reshape(-1))
            d["in_hier"] = dev(np.array(self._in_hier if self._in_hier else [0], np.uint8))
            d["label"], d["label_off"] = pool(self.labels)
            if self.variant == LEGACY:
                lins = [self.hier.rows.get(t, "") if h else "" for t, h in zip(self.taxids, self._in_hier)]
                d["taxlin"], d["taxlin_off"] = pool(lins)
                d["taxlvl"], d["taxlvl_off"] = pool([legacy_level(x) for x in lins])
            d["sizes"] = sizes
        return d

    def run(self, paf: PafTable, ref_counts: Optional[np.ndarray] = None, comm=None) -> LcaResult:
        gpu, torch = self.gpu, self.gpu.torch
        nq, nl = len(paf.queries), paf.n_lines
        t_tax = self.target_tax(paf.targets)
        tax_names = np.array(self._tax_names if self._tax_names else [[-1] * 8], np.int32).reshape(-1)
        in_hier = np.array(self._in_hier if self._in_hier else [0], np.uint8)
        order = np.argsort(paf.line_q, kind="stable")
        q_off = np.zeros(nq + 1, np.int64)
        np.add.at(q_off, paf.line_q.astype(np.int64) + 1, 1)
        q_off = np.cumsum(q_off)

        def dev(a):
            return torch.from_numpy(np.ascontiguousarray(a)).to(gpu.dev)

        d_t = dev(paf.line_t[order] if nl else np.zeros(1, np.int32))
        d_all_t = dev(paf.line_t if nl else np.zeros(1, np.int32))
        counts = gpu.zeros(max(len(paf.targets), 1), torch.int32)
        if ref_counts is None:
            gpu.call("hymet_lca_ref_counts", ptr(d_all_t), nl, ptr(counts))
            if comm is not None and comm.world > 1:
                comm.allreduce_sum_(counts)
        else:
            counts = dev(ref_counts.astype(np.int32))
        d_b = dev(paf.line_blen[order] if nl else np.zeros(1, np.int64))
        d_l = dev(paf.line_qlen[order] if nl else np.zeros(1, np.int64))
        d_e = dev(paf.line_exact[order] if nl else np.zeros(1, np.uint8))
        d_qoff = dev(q_off)
        d_ttax = dev(t_tax if len(t_tax) else np.full(1, -1, np.int32))
        d_names = dev(tax_names)
        d_hier = dev(in_hier)
        n_scr = max(nl, 1)
        s_tid = gpu.empty(n_scr, torch.int32)
        s_w = gpu.empty(n_scr, torch.float64)
        s_nm = gpu.empty(n_scr, torch.int32)
        s_nw = gpu.empty(n_scr, torch.float64)
        o_depth = gpu.zeros(max(nq, 1), torch.int32)
        o_names = gpu.zeros(max(nq, 1) * 8, torch.int32)
        o_conf = gpu.zeros(max(nq, 1), torch.float64)
        o_tax = gpu.zeros(max(nq, 1), torch.int32)
        gpu.call("hymet_lca", self.variant, nq, ptr(d_qoff), ptr(d_t), ptr(d_b), ptr(d_l), ptr(d_e), ptr(counts),
                 ptr(d_ttax), ptr(d_names), ptr(d_hier), ptr(s_tid), ptr(s_w), ptr(s_nm), ptr(s_nw), ptr(o_depth),
                 ptr(o_names), ptr(o_conf), ptr(o_tax))
        return LcaResult(paf.queries, o_depth[:nq].cpu().numpy(), o_names[:nq * 8].cpu().numpy().reshape(nq, 8),
                         o_conf[:nq].cpu().numpy(), o_tax[:nq].cpu().numpy())

    # ----------------------------------------------------------------- output
    def rows(self, res: LcaResult):
        out = []
        lin_cache = {}  # (depth, name ids) -> lineage string: few distinct lineages, many queries
        depth, names, conf = res.depth, res.names, res.conf
        for q, name in enumerate(res.queries):
            d = int(depth[q])
            if self.variant == CAMI:
                if d <= 0:
                    out.append((name, "Unknown", "root", 0.0))
                else:
                    key = (d,) + tuple(names[q, :d].tolist())
                    lin = lin_cache.get(key)
                    if lin is None:
                        lin = "; ".join(f"{RANKS[i]}:{self.labels[names[q, i]]}" for i in range(d))
                        lin_cache[key] = lin
                    out.append((name, lin, RANKS[d - 1], float(conf[q])))
            else:
                if d == -1:
                    lin = self.hier.rows[self.taxids[int(res.tax[q])]]
                    out.append((name, lin, legacy_level(lin), 1.0))
                elif d == 0:
                    out.append((name, "Unknown", "root", 0.0))
                else:
                    key = (d,) + tuple(names[q, :d].tolist())
                    hit = lin_cache.get(key)
                    if hit is None:
                        full = ";".join(self.labels[names[q, i]] for i in range(d))
                        hit = (full, legacy_level(full))
                        lin_cache[key] = hit
                    out.append((name, hit[0], hit[1], float(conf[q])))
        return out

    def tsv_bytes(self, res: LcaResult, rows=None) -> bytes:
        buf = io.StringIO(newline="")
        w = csv.writer(buf, delimiter="\t")
        w.writerow(["Query", "Lineage", "Taxonomic Level", "Confidence"])
        w.writerows([q, lin, lvl, f"{conf:.4f}"] for q, lin, lvl, conf in (rows if rows is not None else self.rows(res)))
        return buf.getvalue().encode()


def classify_file(gpu, paf_path, taxonomy, hierarchy, output, variant: int = CAMI) -> int:
    """The whole drop-in: returns the number of classified queries (lineage != Unknown)."""
    c = Classifier(gpu, taxonomy, hierarchy, variant)
    paf = read_paf(paf_path, variant)
    if variant == LEGACY and len(paf.queries) == 0:
        raise ZeroDivisionError("division by zero")  # classification.py:182 on an empty PAF
    res = c.run(paf)
    data = c.tsv_bytes(res)
    with open(output, "wb") as f:
        f.write(data)
    return int(sum(1 for r in c.rows(res) if r[1] != "Unknown"))

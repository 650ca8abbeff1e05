"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the classify stage.

This module is a plain-Python restatement of the reference classifiers, used by
``tests/`` (as the checker), ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg.  The product path (``hymet_amd``) never imports it.

Parity is pinned: ``tests/test_classify_oracle.py`` checks this restatement
byte-for-byte against ``tests/golden/classify/*`` which were produced by running
the reference scripts themselves in the build container
(``tests/golden/make_goldens.py``).

Reference (read-only, /root/reference):
  * scripts/classification_cami.py  -- CLI-path classifier (``run_hymet_cami.sh:175``)
  * scripts/classification.py       -- legacy classifier (``main.pl:113``)
  * tools/build_id_map.py, tools/mini_classify.py -- fallback (``run_hymet_cami.sh:182-206``)
"""
from __future__ import annotations

import csv
import gzip
import io
import re
from collections import defaultdict

csv.field_size_limit(1 << 30)

# scripts/classification_cami.py:16-28
RANKS = ["superkingdom", "phylum", "class", "order", "family", "genus", "species", "strain"]
RANK_ALIAS = {
    "domain": "superkingdom", "kingdom": "superkingdom", "sk": "superkingdom", "k": "superkingdom",
    "phylum": "phylum", "p": "phylum", "class": "class", "c": "class", "order": "order", "o": "order",
    "family": "family", "f": "family", "genus": "genus", "g": "genus", "species": "species", "s": "species",
    "subspecies": "strain", "ss": "strain", "strain": "strain",
}
GCFA_RE = re.compile(r"GC[AF]_\d+(?:\.\d+)?(?:_PRJ[A-Z]+\d+)?")
ACC_RE = re.compile(r"(NC_\d+\.\d+|NZ_[A-Z]{2}\d+\.\d+|NZ_[A-Z]{5}\d+\.\d+|CP\d+\.\d+|CM\d+\.\d+|[A-Z]{2}_\d+\.\d+)")


# ---------------------------------------------------------------- cami variant
def _add_token(m, tok, taxid):  # classification_cami.py:43-53
    if not tok:
        return
    tok = tok.strip()
    if not tok:
        return
    m.setdefault(tok, taxid)
    if "." in tok:
        m.setdefault(tok.split(".", 1)[0], taxid)


def load_taxonomy_cami(path):  # classification_cami.py:63-102
    m = {}
    with open(path, "r", newline="") as f:
        rd = csv.DictReader(f, delimiter="\t")
        if "TaxID" not in rd.fieldnames:
            raise RuntimeError("TaxID column not found in taxonomy file")
        for row in rd:
            taxid = (row.get("TaxID") or "").strip()
            if not taxid:
                continue
            for v in row.values():
                if not v:
                    continue
                for acc in GCFA_RE.findall(v):
                    _add_token(m, acc, taxid)
            ids = row.get("Identifiers") or ""
            for tok in [p for p in (x.strip() for x in re.split(r"[;|,\s]+", ids)) if p] if ids else []:
                _add_token(m, tok, taxid)
            for v in (ids,) + tuple(row.get(k) or "" for k in row.keys()):
                if not v:
                    continue
                for mm in ACC_RE.findall(v):
                    _add_token(m, mm, taxid)
    return m


def parse_lineage_to_names(raw):  # classification_cami.py:104-156
    out = [""] * len(RANKS)
    if not raw:
        return out
    s = raw.strip()
    for sep in (":", "__"):
        if sep in s:
            for part in re.split(r"[;|]+", s):
                part = part.strip()
                if not part or sep not in part:
                    continue
                rk, nm = part.split(sep, 1)
                rk = RANK_ALIAS.get(rk.strip().lower())
                nm = nm.strip()
                if not rk or not nm:
                    continue
                out[RANKS.index(rk)] = nm
            return out
    seq = [p.strip() for p in re.split(r"[;|]+", s) if p.strip() and p.strip().upper() != "NA"]
    for i, nm in enumerate(seq[: len(RANKS)]):
        out[i] = nm
    return out


def load_hierarchy_cami(path):  # classification_cami.py:158-174
    h = {}
    with open(path, "r", newline="") as f:
        rd = csv.DictReader(f, delimiter="\t")
        if "TaxID" not in rd.fieldnames or "Lineage" not in rd.fieldnames:
            raise RuntimeError("Hierarchy file must have TaxID and Lineage columns")
        for row in rd:
            tid = (row.get("TaxID") or "").strip()
            lin = (row.get("Lineage") or "").strip()
            if tid:
                h[tid] = parse_lineage_to_names(lin)
    return h


def _open_text(path):
    return gzip.open(path, "rt") if str(path).endswith(".gz") else open(path, "r")


def parse_paf_cami(path):  # classification_cami.py:181-208
    qmap = defaultdict(list)
    counts = defaultdict(int)
    with _open_text(path) as f:
        for line in f:
            if not line or line.startswith("#"):
                continue
            parts = line.rstrip("\n").split("\t")
            if len(parts) < 11:
                continue
            try:
                qlen = int(parts[1])
                blk = int(parts[10])
            except Exception:
                qlen = blk = 0
            cov = (blk / qlen) if qlen > 0 else 0.0
            qmap[parts[0]].append((parts[5], cov))
            counts[parts[5]] += 1
    return qmap, counts


def lookup_candidates(tname):  # classification_cami.py:212-241
    c = []

    def add(x):
        if x and x not in c:
            c.append(x)
        if x and "." in x:
            xv = x.split(".", 1)[0]
            if xv not in c:
                c.append(xv)

    add(tname)
    add(re.split(r"[|\s]+", tname)[0])
    for g in GCFA_RE.findall(tname):
        add(g)
    for a in ACC_RE.findall(tname):
        add(a)
    return c


def lookup_taxid(tax, tname):  # classification_cami.py:243-249
    for cand in lookup_candidates(tname):
        tid = tax.get(cand)
        if tid:
            return tid
    return None


def weighted_lca_cami(tw, hier):  # classification_cami.py:251-288
    if sum(tw.values()) <= 0:
        return "Unknown", "root", 0.0
    chosen, conf = [], 1.0
    for r in range(len(RANKS)):
        name_w = defaultdict(float)
        denom = 0.0
        for tid, w in tw.items():
            names = hier.get(tid)
            if not names:
                continue
            nm = names[r] if r < len(names) else ""
            if nm:
                name_w[nm] += w
                denom += w
        if denom <= 0 or not name_w:
            break
        best, bw = max(name_w.items(), key=lambda kv: kv[1])
        chosen.append(best)
        conf *= bw / denom
    if not chosen:
        return "Unknown", "root", 0.0
    lin = "; ".join(f"{RANKS[i]}:{n}" for i, n in enumerate(chosen))
    return lin, RANKS[len(chosen) - 1], min(conf, 1.0)


def classify_cami(paf, taxonomy, hierarchy, ref_counts=None):
    """Return the exact TSV bytes classification_cami.py writes (:333-339).  ref_counts
    (target -> PAF line count) replaces the file's own counts when the PAF is a sample of a
    larger run (bench.py's CPU leg: ref_abundance is global over the whole PAF)."""
    tax = load_taxonomy_cami(taxonomy)
    hier = load_hierarchy_cami(hierarchy)
    qmap, counts = parse_paf_cami(paf)
    if ref_counts is not None:
        counts = ref_counts
    tcache = {}
    buf = io.StringIO(newline="")
    w = csv.writer(buf, delimiter="\t")
    w.writerow(["Query", "Lineage", "Taxonomic Level", "Confidence"])
    for q, refs in qmap.items():  # _process_one :290-308
        tw = defaultdict(float)
        hit = False
        for t, cov in refs:
            if t not in tcache:
                tcache[t] = lookup_taxid(tax, t)
            tid = tcache[t]
            if not tid:
                continue
            hit = True
            tw[tid] += cov * counts.get(t, 1)
        lin, lvl, conf = weighted_lca_cami(tw, hier) if hit else ("Unknown", "root", 0.0)
        w.writerow([q, lin, lvl, f"{conf:.4f}"])
    return buf.getvalue().encode()


# -------------------------------------------------------------- legacy variant
LEGACY_RANKS = RANKS


def load_taxonomy_legacy(path):  # classification.py:14-25
    t = {}
    with open(path, "r") as f:
        for row in csv.DictReader(f, delimiter="\t"):
            for ident in row["Identifiers"].split(";"):
                c = ident.strip()
                if c:
                    t[c] = row["TaxID"]
    return t


def load_hierarchy_legacy(path):  # classification.py:27-35
    h = {}
    with open(path, "r") as f:
        for row in csv.DictReader(f, delimiter="\t"):
            h[row["TaxID"]] = row["Lineage"].strip()
    return h


def parse_paf_legacy(path):  # classification.py:37-59
    qmap = defaultdict(list)
    counts = defaultdict(int)
    with open(path, "r") as f:
        for line in f:
            parts = line.strip().split("\t")
            if len(parts) < 11:
                continue
            qid, qlen, rid, alen = parts[0], int(parts[1]), parts[5], int(parts[10])
            cov = alen / qlen if qlen > 0 else 0
            qmap[qid].append((rid, cov, (qid == rid) and (cov >= 0.99)))
            counts[rid] += 1
    return qmap, counts


def taxonomic_level_legacy(lineage):  # classification.py:61-81
    cur = None
    for part in lineage.split(";"):
        part = part.strip()
        if ":" in part:
            rank = part.split(":", 1)[0].strip().lower()
            if rank in LEGACY_RANKS:
                if cur is None or LEGACY_RANKS.index(rank) > LEGACY_RANKS.index(cur):
                    cur = rank
    return cur if cur is not None else "root"


def lca_legacy(refs, counts, tax, hier):  # classification.py:83-157
    ex = [r for r, _, e in refs if e and r in tax]
    if ex:
        tid = tax[ex[0]]
        if tid in hier:
            return hier[tid], taxonomic_level_legacy(hier[tid]), 1.0
    tw = defaultdict(float)
    total = 0.0
    for rid, cov, _ in refs:
        if rid not in tax:
            continue
        w = cov * counts.get(rid, 1)
        tw[tax[rid]] += w
        total += w
    if total == 0:
        return "Unknown", "root", 0.0
    lins = [(hier[t].split(";"), w / total) for t, w in tw.items() if t in hier]
    if not lins:
        return "Unknown", "root", 0.0
    cons, conf = {}, 1.0
    for rank in LEGACY_RANKS:
        lc = defaultdict(float)
        for lin, w in lins:
            for part in lin:
                if part.startswith(f"{rank}:"):
                    lc[part] += w
                    break
        if not lc:
            break
        best, c = max(lc.items(), key=lambda x: x[1])
        cons[rank] = best
        conf *= c
    parts = [cons.get(r) for r in LEGACY_RANKS if cons.get(r)]
    if not parts:
        return "Unknown", "root", 0.0
    full = ";".join(parts)
    return full, taxonomic_level_legacy(full), min(conf, 1.0)


def classify_legacy(paf, taxonomy, hierarchy):
    """Exact TSV bytes of classification.py (:171-179); raises ZeroDivisionError
    on an empty PAF exactly like the reference does at :182."""
    tax = load_taxonomy_legacy(taxonomy)
    hier = load_hierarchy_legacy(hierarchy)
    qmap, counts = parse_paf_legacy(paf)
    buf = io.StringIO(newline="")
    w = csv.writer(buf, delimiter="\t")
    w.writerow(["Query", "Lineage", "Taxonomic Level", "Confidence"])
    n = 0
    for q, refs in qmap.items():
        lin, lvl, conf = lca_legacy(refs, counts, tax, hier)
        w.writerow([q, lin, lvl, f"{conf:.4f}"])
        n += 1
    if n == 0:
        raise ZeroDivisionError("division by zero")
    return buf.getvalue().encode()


# ------------------------------------------------------------------- fallback
def fallback_classify(paf, taxonomy):
    """tools/build_id_map.py:17-48 + tools/mini_classify.py:16-30 + the awk rewrite at
    run_hymet_cami.sh:197-202.  Returns the final classified_sequences.tsv bytes."""
    id2tax = {}

    def emit(k, tax):
        if not k:
            return
        id2tax.setdefault(k, tax)
        if "." in k:
            id2tax.setdefault(k.split(".", 1)[0], tax)

    with open(taxonomy, "r", encoding="utf-8", errors="ignore", newline="") as f:
        hdr = f.readline().rstrip("\n").split("\t")
        try:
            ig, it, ii = hdr.index("GCF"), hdr.index("TaxID"), hdr.index("Identifiers")
        except ValueError:
            ig, it, ii = 0, 1, 2
        for line in f:
            if not line.strip():
                continue
            row = line.rstrip("\n").split("\t")
            if len(row) <= max(ig, it):
                continue
            tax = row[it].strip()
            emit(row[ig].strip(), tax)
            ids = row[ii].strip() if len(row) > ii else ""
            if ids:
                for tok in ids.split(";"):
                    emit(tok.strip(), tax)
    # build_id_map writes the map through csv then mini_classify re-reads it with
    # setdefault; keys are unique so the round trip is the identity.
    seen = set()
    rows = []
    with _open_text(paf) as f:
        for ln in f:
            if not ln or ln[0] == "#":
                continue
            p = ln.rstrip("\n").split("\t")
            if len(p) < 6:
                continue
            q, t = p[0], p[5]
            if q in seen:
                continue
            tax = id2tax.get(t) or id2tax.get(t.split(".", 1)[0])
            if tax:
                rows.append(q)
                seen.add(q)
    out = "Query\tLineage\tTaxonomic Level\tConfidence\n"
    for q in rows:
        out += f"{q}\tunknown\tunknown\t1.0000\n"
    return out.encode()

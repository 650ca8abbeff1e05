"""CAMI evaluation of HYMET output: tools/eval_cami.py restated.

Profile level (eval_cami.py:168-240, 369-385, 611-632): the predicted and truth CAMI profiles
per rank -> L1 total variation, Bray-Curtis, presence precision / recall / F1.  Contig level
(:388-568): every classified contig resolved to its most specific TaxID (lineage names via
name2taxid, else a TaxID column, else its target through the detailed_taxonomy id map, else
its first PAF hit), paired with the truth mapping (by name, else by sequence MD5), compared
per rank on taxonomy paths.

The reference shells out to taxonkit (`name2taxid --show-rank`, `reformat -I 1 -f
"{k}|{p}|{c}|{o}|{f}|{g}|{s}" -t`); both are restated from names.dmp / nodes.dmp by
hymet_amd.taxonomy (taxonkit is absent: unpinned).  {k} is read as domain-or-superkingdom,
as hymet2cami's {d} is, so NCBI's 2025 "domain" dumps keep their top rank.  The last-resort
pairing by `minimap2 -x asm10` of predicted against truth contigs (:519-528) runs only when a
`minimap2` binary is on PATH, as in the reference.  Host-side text work: no device code.
"""
from __future__ import annotations

import collections
import csv
import gzip
import hashlib
import os
import pathlib
import re
import shutil
import subprocess
import sys
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

from .taxonomy import TaxDump, name2taxid as _name2taxid, reformat as _reformat

csv.field_size_limit(1024 * 1024 * 1024)

RANKS = ["superkingdom", "phylum", "class", "order", "family", "genus", "species"]
RANKC = ["k", "p", "c", "o", "f", "g", "s"]
LINEAGE_ALIAS = {  # eval_cami.py:19-40 (wider than hymet2cami's: strains fold into species)
    "domain": "superkingdom", "kingdom": "superkingdom", "sk": "superkingdom", "k": "superkingdom",
    "superkingdom": "superkingdom", "phylum": "phylum", "p": "phylum", "class": "class", "c": "class",
    "order": "order", "o": "order", "family": "family", "f": "family", "genus": "genus", "g": "genus",
    "species": "species", "s": "species", "subspecies": "species", "ss": "species", "strain": "species",
}
GCFA_RE = re.compile(r"GC[AF]_\d+(?:\.\d+)?(?:_PRJ[A-Z]+\d+)?")
ACC_RE = re.compile(r"(NC_\d+\.\d+|NZ_[A-Z]{2}\d+\.\d+|NZ_[A-Z]{5}\d+\.\d+|CP\d+\.\d+|CM\d+\.\d+|[A-Z]{2}_\d+\.\d+)")


# ------------------------------------------------------------------ utilities
def is_num(s: Optional[str]) -> bool:
    s = (s or "").strip()
    return bool(s) and (s.isdigit() or re.fullmatch(r"[0-9]+(?:\.[0-9]+)?", s) is not None)


def normalize_taxid(val: Optional[str]) -> str:
    if not val:
        return ""
    m = re.search(r"[0-9]+", val)
    return m.group(0) if m else ""


def _open_any(path: str):
    return gzip.open(path, "rt") if path.endswith(".gz") else open(path, "r")


def parse_lineage_string(lineage_raw: str) -> Dict[str, str]:
    out: Dict[str, str] = {}
    for part in (seg.strip() for seg in (lineage_raw or "").split(";")):
        if not part or ":" not in part:
            continue
        rk, nm = part.split(":", 1)
        rk = LINEAGE_ALIAS.get(rk.strip().lower())
        nm = nm.strip()
        if rk and nm:
            out[rk] = nm
    return out


def _fasta_records(path: str):
    """(name, stripped sequence lines) per record, the way eval_cami.py:81-108 reads."""
    name, lines = None, []
    with open(path) as f:
        for ln in f:
            if ln.startswith(">"):
                if name is not None:
                    yield name, lines
                name, lines = ln[1:].strip().split()[0], []
            else:
                lines.append(ln.strip())
    if name is not None:
        yield name, lines


def fasta_lengths(paths: Iterable[Optional[str]]) -> Dict[str, int]:
    lens: Dict[str, int] = {}
    for path in paths:
        if path and os.path.isfile(path):
            for name, lines in _fasta_records(path):
                lens.setdefault(name, sum(len(x) for x in lines))
    return lens


def fasta_hashes(path: Optional[str]) -> Dict[str, str]:
    out: Dict[str, str] = {}
    if path and os.path.isfile(path):
        for name, lines in _fasta_records(path):
            md = hashlib.md5()
            for s in lines:
                if s:
                    md.update(s.encode())
            out[name] = md.hexdigest()
    return out


# ------------------------------------------------------- taxonkit, restated
class Taxonomy:
    """The taxdump a run's taxonkit calls read (TAXONKIT_DB / --taxdb), loaded once."""

    def __init__(self, taxdb: str):
        self.taxdb = taxdb
        self._d: Optional[TaxDump] = None

    @property
    def dump(self) -> Optional[TaxDump]:
        if self._d is None:
            names, nodes = os.path.join(self.taxdb, "names.dmp"), os.path.join(self.taxdb, "nodes.dmp")
            if not (os.path.isfile(names) and os.path.isfile(nodes)):
                return None
            self._d = TaxDump(names, nodes, all_names=True)
        return self._d

    def name2taxid(self, names: Iterable[str]) -> Dict[str, str]:
        names = [n for n in names if n]
        if not names or self.dump is None:
            return {}
        return {k: v for k, v in _name2taxid(self.dump, names).items() if is_num(v)}

    def taxpath(self, taxids: Iterable[str]) -> Dict[str, Tuple[str, str]]:
        taxids = [t for t in taxids if t]
        if not taxids or self.dump is None:
            return {}
        return _reformat(self.dump, taxids)


# ----------------------------------------------------------------- id map
def _add_tok(m: Dict[str, str], tok: str, taxid: str) -> None:
    tok = (tok or "").strip()
    if not tok:
        return
    m.setdefault(tok, taxid)
    if "." in tok:
        m.setdefault(tok.split(".", 1)[0], taxid)


def load_id_map(taxmap_path: str) -> Dict[str, str]:
    """eval_cami.py:145-165 over detailed_taxonomy.tsv."""
    id2tax: Dict[str, str] = {}
    if not os.path.isfile(taxmap_path):
        return id2tax
    with open(taxmap_path, newline="") as f:
        for row in csv.DictReader(f, delimiter="\t"):
            tax = normalize_taxid(row.get("TaxID") or "")
            if not tax:
                continue
            for key in ("GCF", "GCA"):
                v = (row.get(key) or "").strip()
                if v:
                    _add_tok(id2tax, v, tax)
            for tok in re.split(r"[;|,\s]+", row.get("Identifiers") or ""):
                _add_tok(id2tax, tok, tax)
            for v in row.values():
                if not v:
                    continue
                for g in GCFA_RE.findall(v):
                    _add_tok(id2tax, g, tax)
                for a in ACC_RE.findall(v):
                    _add_tok(id2tax, a, tax)
    return id2tax


# ---------------------------------------------------------------- profiles
def _empty_profile():
    return {r: collections.Counter() for r in RANKS}


def parse_cami_like(lines: Sequence[str], tax: Taxonomy):
    """eval_cami.py:168-234: CAMI rows (TAXID RANK TAXPATH TAXPATHSN PERCENTAGE), else a
    headed table with taxid / taxpath / taxpathsn columns."""
    prof = _empty_profile()
    ok = False
    for ln in lines:
        if not ln.strip() or ln[0] in "#@":
            continue
        ps = ln.rstrip("\n").split("\t")
        if len(ps) >= 5 and is_num(ps[0]):
            rk = ps[1].strip().lower()
            if rk in prof:
                try:
                    prof[rk][ps[0]] += float(ps[4])
                    ok = True
                except ValueError:
                    pass
            continue
        break
    if ok:
        return prof
    rdr = csv.reader([ln for ln in lines if ln.strip() and ln[0] not in "#@"], delimiter="\t")
    try:
        hdr = next(rdr)
    except StopIteration:
        return prof
    h = [c.strip().lower() for c in hdr]

    def idx(*names):
        for n in names:
            if n in h:
                return h.index(n)
        return -1

    i_taxid = idx("taxid", "taxon_id", "ncbi_taxid", "ncbi_tax_id")
    i_rank = idx("rank")
    i_perc = idx("percentage", "abundance", "rel_abundance", "fraction_total_reads")
    i_taxpath = idx("taxpath")
    i_taxpathsn = idx("taxpathsn", "taxpath_sn", "taxpath_names", "lineage")
    rows = list(rdr)
    if i_taxid >= 0 and i_rank >= 0 and i_perc >= 0:
        mul = 100.0 if "abundance" in h[i_perc] or "fraction" in h[i_perc] else 1.0
        for ps in rows:
            try:
                tid = normalize_taxid(ps[i_taxid])
                rk = ps[i_rank].strip().lower()
                val = float(ps[i_perc]) * mul
                if rk in prof and tid:
                    prof[rk][tid] += val
            except (ValueError, IndexError):
                pass
        return prof
    if i_rank >= 0 and (i_taxpath >= 0 or i_taxpathsn >= 0) and i_perc >= 0:
        rk_to_idx = dict(zip(RANKS, range(len(RANKS))))
        mul = 100.0 if "abundance" in h[i_perc] or "fraction" in h[i_perc] else 1.0
        if i_taxpath >= 0:
            for ps in rows:
                try:
                    rk = ps[i_rank].strip().lower()
                    ids = [x for x in ps[i_taxpath].strip().split("|") if x and x != "NA"]
                    r = rk_to_idx.get(rk, -1)
                    if 0 <= r < len(ids):
                        prof[rk][ids[r]] += float(ps[i_perc]) * mul
                except (ValueError, IndexError):
                    pass
            return prof
        names, keep = set(), []
        for ps in rows:
            try:
                rk = ps[i_rank].strip().lower()
                pathn = [p.strip() for p in ps[i_taxpathsn].split("|")]
                r = rk_to_idx.get(rk, -1)
                if 0 <= r < len(pathn) and pathn[r]:
                    names.add(pathn[r])
                keep.append(ps)
            except IndexError:
                pass
        m = tax.name2taxid(names)
        for ps in keep:
            try:
                rk = ps[i_rank].strip().lower()
                pathn = [p.strip() for p in ps[i_taxpathsn].split("|")]
                r = rk_to_idx.get(rk, -1)
                if 0 <= r < len(pathn):
                    tid = m.get(pathn[r])
                    if tid:
                        prof[rk][tid] += float(ps[i_perc]) * mul
            except (ValueError, IndexError):
                pass
    return prof


def load_profile_any(path: str, tax: Taxonomy):
    if not os.path.isfile(path):
        return _empty_profile()
    with open(path) as f:
        return parse_cami_like(f.readlines(), tax)


def load_gt_contigs(gt_file: str) -> Dict[str, str]:
    """eval_cami.py:243-303: contig -> TaxID of a CAMI gsa_mapping (tab, comma or space
    separated; a TaxID-like column, else the last taxpath id, else the first numeric field)."""
    out: Dict[str, str] = {}
    if not gt_file or not os.path.isfile(gt_file):
        return out
    with _open_any(gt_file) as fh:
        first = fh.readline()
    if "\t" in first or "," in first:
        with _open_any(gt_file) as f:
            rdr = csv.reader(f, delimiter="\t" if "\t" in first else ",")
            hdr = next(rdr)
            rows = list(rdr)
    else:
        hdr = [c.strip() for c in first.strip().split()]
        rows = []
        with _open_any(gt_file) as f:
            next(f)
            for line in f:
                line = line.strip()
                if line:
                    rows.append(line.split())
    h = [c.strip().lstrip("#").lower() for c in hdr]
    contig_keys = [k for k in h if any(x in k for x in ("contig", "sequence", "scaffold"))]
    taxid_keys = [k for k in h if ("tax" in k and "path" not in k)] + \
                 [k for k in h if k in ("ncbi_taxid", "ncbi_tax_id", "taxid", "tax_id", "species_taxid", "genome_taxid")]
    ci = h.index(contig_keys[0]) if contig_keys else 0
    ti = h.index(taxid_keys[0]) if taxid_keys else -1
    if ti >= 0:
        for ps in rows:
            if len(ps) <= max(ci, ti):
                continue
            raw = (ps[ti] or "").strip()
            if raw and not is_num(raw):
                raw = normalize_taxid(raw)
            if raw:
                out[ps[ci]] = normalize_taxid(raw)
    elif "taxpath" in h:
        tpi = h.index("taxpath")
        for ps in rows:
            ids = [x for x in ps[tpi].split("|") if x and x != "NA"]
            if ids:
                tid = normalize_taxid(ids[-1])
                if tid:
                    out[ps[ci]] = tid
    else:
        for ps in rows:
            for x in ps[1:]:
                if is_num(x):
                    out[ps[0]] = normalize_taxid(x)
                    break
    return out


def profiles_from_contig_maps(contig2tid: Dict[str, str], lengths: Dict[str, int], tax: Taxonomy):
    """eval_cami.py:306-329: length-weighted per-rank percentages from contig TaxIDs."""
    prof = _empty_profile()
    norm = {c: normalize_taxid(t) for c, t in contig2tid.items() if normalize_taxid(t)}
    if not norm:
        return prof
    paths = tax.taxpath(set(norm.values()))
    acc = collections.Counter()
    for cont, tid in norm.items():
        w = lengths.get(cont, 1)
        ni = paths.get(tid)
        if not ni:
            continue
        ids = ni[1].split("|")
        for i in range(len(RANKC)):
            if i < len(ids) and ids[i] != "NA":
                prof[RANKS[i]][ids[i]] += w
                acc[RANKS[i]] += w
    for r in RANKS:
        s = acc[r]
        if s > 0:
            for k in list(prof[r].keys()):
                prof[r][k] = 100.0 * prof[r][k] / s
    return prof


# --------------------------------------------------------------------- PAF
def besthit_map_from_paf(paf_path: str, min_cov: float = 0.95, min_id: float = 0.95) -> Dict[str, str]:
    best: Dict[str, tuple] = {}
    with open(paf_path) as f:
        for ln in f:
            if not ln.strip() or ln[0] == "#":
                continue
            p = ln.rstrip("\n").split("\t")
            if len(p) < 12:
                continue
            q, qlen, qs, qe = p[0], int(p[1]), int(p[2]), int(p[3])
            nmatch, alen = int(p[9]), int(p[10])
            cov = (qe - qs) / qlen if qlen > 0 else 0.0
            iden = nmatch / alen if alen > 0 else 0.0
            if cov < min_cov or iden < min_id:
                continue
            cur = best.get(q)
            if cur is None or nmatch > cur[0]:
                best[q] = (nmatch, p[5])
    return {q: t for q, (_, t) in best.items()}


def paf_firsthit_q2t(paf_path: str) -> Dict[str, str]:
    q2t: Dict[str, str] = {}
    if not paf_path or not os.path.isfile(paf_path):
        return q2t
    with open(paf_path) as f:
        for ln in f:
            if not ln.strip() or ln[0] == "#":
                continue
            p = ln.rstrip("\n").split("\t")
            if len(p) >= 6 and p[0] not in q2t:
                q2t[p[0]] = p[5]
    return q2t


# ------------------------------------------------------------------ metrics
def l1_and_braycurtis(a: Dict[str, float], b: Dict[str, float]) -> Tuple[float, float]:
    keys = set(a) | set(b)
    if not keys:
        return 0.0, 0.0
    l1 = 0.5 * sum(abs(a.get(k, 0.0) - b.get(k, 0.0)) for k in keys)
    sump = sum(a.get(k, 0.0) for k in keys)
    sumt = sum(b.get(k, 0.0) for k in keys)
    shared = sum(min(a.get(k, 0.0), b.get(k, 0.0)) for k in keys)
    bc = 1.0 - (2.0 * shared / (sump + sumt if (sump + sumt) > 0 else 1.0))
    return l1, bc * 100.0


def prf_presence(a: Dict[str, float], b: Dict[str, float], thr: float = 0.1):
    A = {k for k, v in a.items() if v >= thr}
    B = {k for k, v in b.items() if v >= thr}
    tp, fp, fn = len(A & B), len(A - B), len(B - A)
    prec = tp / (tp + fp) if (tp + fp) > 0 else 0.0
    rec = tp / (tp + fn) if (tp + fn) > 0 else 0.0
    f1 = 2 * prec * rec / (prec + rec) if (prec + rec) > 0 else 0.0
    return prec * 100.0, rec * 100.0, f1 * 100.0, tp, fp, fn


# ------------------------------------------------------------- contig level
def _via_idmap(target: str, idmap: Dict[str, str]) -> str:
    base = target.split("|", 1)[0]
    cands = [target, base] + ([base.split(".", 1)[0]] if "." in base else [])
    for c in cands:
        if c in idmap:
            t = normalize_taxid(idmap[c])
            if t:
                return t
    return ""


def preds_taxid_from_classified(classified_tsv: str, tax: Taxonomy, idmap: Dict[str, str],
                                paf_path: Optional[str]) -> Dict[str, str]:
    """eval_cami.py:388-483: most specific resolvable TaxID per classified contig."""
    cont2tid: Dict[str, str] = {}
    lineage_records: Dict[str, Dict[str, str]] = {}
    fallback: Dict[str, dict] = {}
    all_names = set()
    if os.path.isfile(classified_tsv):
        with open(classified_tsv, encoding="utf-8", errors="ignore") as f:
            reader = csv.DictReader(f, delimiter="\t")
            raw = reader.fieldnames or []
            hs = [(h or "").strip().lower() for h in raw]
            k_query = raw[hs.index("query")] if "query" in hs else None
            k_taxid = raw[hs.index("taxid")] if "taxid" in hs else None
            i_target = next((hs.index(c) for c in ("target", "tname") if c in hs), None)
            k_target = raw[i_target] if i_target is not None else None
            k_lineage = raw[hs.index("lineage")] if "lineage" in hs else None
            for row in reader:
                q = row.get(k_query) if k_query else (row.get("Query") or row.get("qname") or row.get("q"))
                if not q:
                    continue
                lin = parse_lineage_string(row.get(k_lineage, "") if k_lineage else row.get("Lineage", ""))
                if lin:
                    lineage_records[q] = lin
                    all_names.update(nm for nm in lin.values() if nm)
                fallback[q] = {"taxid": row.get(k_taxid) if k_taxid else row.get("TaxID"),
                               "target": row.get(k_target) if k_target else (row.get("Target") or row.get("tname"))}
    name_map = tax.name2taxid(all_names) if all_names else {}
    for q, lin in lineage_records.items():
        for rank in reversed(RANKS):
            nm = lin.get(rank)
            t = normalize_taxid(name_map.get(nm, "")) if nm else ""
            if t:
                cont2tid[q] = t
                break
    for q, info in fallback.items():
        if q not in cont2tid:
            t = normalize_taxid(info.get("taxid") or "")
            if t:
                cont2tid[q] = t
    for q, info in fallback.items():
        if q not in cont2tid:
            target = (info.get("target") or "").strip()
            t = _via_idmap(target, idmap) if target else ""
            if t:
                cont2tid[q] = t
    if paf_path and os.path.isfile(paf_path):
        for q, target in paf_firsthit_q2t(paf_path).items():
            if q not in cont2tid:
                t = _via_idmap(target, idmap)
                if t:
                    cont2tid[q] = t
    return cont2tid


def eval_contigs(pred_file: str, gt_files: Sequence[str], tax: Taxonomy, outdir: str, pred_fasta=None, gt_fasta=None,
                 threads: int = 8, taxmap_path: str = "", paf_path: Optional[str] = None, log=sys.stderr) -> dict:
    """eval_cami.py:486-568; writes contigs_exact.tsv / contigs_per_rank.tsv (removed when
    no contig pairs)."""
    idmap = load_id_map(taxmap_path)
    pred_tid = preds_taxid_from_classified(pred_file, tax, idmap, paf_path)
    gt_map: Dict[str, str] = {}
    for g in gt_files:
        gt_map.update(load_gt_contigs(g) if g else {})
    print(f"[DEBUG] loaded pred contigs with TaxID: {len(pred_tid)}", file=log)
    print(f"[DEBUG] loaded truth contigs with TaxID: {len(gt_map)}", file=log)
    pairs = [(q, t, gt_map[q]) for q, t in pred_tid.items() if q in gt_map]
    have_fa = bool(pred_fasta and gt_fasta and os.path.isfile(pred_fasta) and os.path.isfile(gt_fasta))
    if not pairs and have_fa:
        ph, gh = fasta_hashes(pred_fasta), fasta_hashes(gt_fasta)
        inv = collections.defaultdict(list)
        for gname, h in gh.items():
            inv[h].append(gname)
        n_md5 = 0
        for q in list(pred_tid.keys()):
            h = ph.get(q)
            for t in inv.get(h, []) if h else []:
                g = gt_map.get(t)
                if g:
                    pairs.append((q, pred_tid[q], g))
                    n_md5 += 1
        print(f"[DEBUG] MD5‑paired contigs: {n_md5}", file=log)
    if not pairs and have_fa and shutil.which("minimap2"):
        paf_tmp = os.path.join(outdir, "pred_vs_truth.paf")
        with open(paf_tmp, "w") as w:
            subprocess.run(["minimap2", "-x", "asm10", "--secondary=no", "-t", str(threads), gt_fasta, pred_fasta],
                           check=True, stdout=w)
        n_map = 0
        for q, t in besthit_map_from_paf(paf_tmp).items():
            pt, g = pred_tid.get(q), gt_map.get(t)
            if pt and g:
                pairs.append((q, pt, g))
                n_map += 1
        print(f"[DEBUG] minimap‑paired contigs: {n_map}", file=log)
    usable = len(pairs)
    exact = sum(1 for _, pt, g in pairs if pt == g)
    tpaths = tax.taxpath({pt for _, pt, _ in pairs} | {g for _, _, g in pairs})
    per_rank = {}
    for i, r in enumerate(RANKS):
        tot = ok = 0
        for _, pt, g in pairs:
            pids, gids = tpaths.get(pt, ("", ""))[1], tpaths.get(g, ("", ""))[1]
            if not pids or not gids:
                continue
            pv, gv = pids.split("|"), gids.split("|")
            if i >= len(pv) or i >= len(gv) or pv[i] == "NA" or gv[i] == "NA":
                continue
            tot += 1
            ok += pv[i] == gv[i]
        per_rank[r] = {"n": tot, "acc": 100.0 * ok / tot if tot else 0.0, "correct": ok}
    exact_path = os.path.join(outdir, "contigs_exact.tsv")
    perrank_path = os.path.join(outdir, "contigs_per_rank.tsv")
    if usable > 0:
        with open(exact_path, "w", newline="") as w:
            wr = csv.writer(w, delimiter="\t")
            wr.writerow(["metric", "value"])
            wr.writerow(["usable_pairs", usable])
            wr.writerow(["exact_taxid_matches", exact])
            wr.writerow(["exact_taxid_accuracy_percent", 100.0 * exact / usable])
        with open(perrank_path, "w", newline="") as w:
            wr = csv.writer(w, delimiter="\t")
            wr.writerow(["rank", "n", "correct", "accuracy_percent"])
            for r in RANKS:
                m = per_rank[r]
                wr.writerow([r, m["n"], m["correct"], f"{m['acc']:.4f}"])
    else:
        for p in (exact_path, perrank_path):
            if os.path.exists(p):
                os.remove(p)
    return {"usable_pairs": usable, "exact": exact, "per_rank": per_rank, "pred_n": len(pred_tid), "gt_n": len(gt_map)}


# --------------------------------------------------------------------- main
def main(argv: Optional[Sequence[str]] = None) -> int:
    """tools/eval_cami.py main (:571-658): same flags, files and stdout."""
    import argparse
    ap = argparse.ArgumentParser(description="Evaluate HYMET vs CAMI ground truth (post-processing only; classifier unchanged).")
    ap.add_argument("--pred-profile", default="/data/hymet_out/sample_0/hymet.sample_0.cami.tsv")
    ap.add_argument("--truth-profile", default="/data/cami/sample_0/taxonomic_profile_0.txt")
    ap.add_argument("--pred-contigs", default="/data/hymet_out/sample_0/work/classified_sequences.tsv")
    ap.add_argument("--truth-contigs", default="")
    ap.add_argument("--pred-fasta", default="/data/cami/sample_0.fna")
    ap.add_argument("--truth-fasta", default="/data/cami/sample_0/2017.12.29_11.37.26_sample_0/contigs/anonymous_gsa.fasta")
    ap.add_argument("--taxdb", default="/data/HYMET/taxonomy_files")
    ap.add_argument("--taxmap", default="/data/HYMET/data/detailed_taxonomy.tsv")
    ap.add_argument("--paf", default="/data/hymet_out/sample_0/work/resultados.paf")
    ap.add_argument("--outdir", default="/data/hymet_out/sample_0/eval")
    ap.add_argument("--presence-thresh", type=float, default=0.1)
    ap.add_argument("--threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "8")))
    a = ap.parse_args(argv)
    pathlib.Path(a.outdir).mkdir(parents=True, exist_ok=True)
    base = "/data/cami/sample_0/2017.12.29_11.37.26_sample_0/contigs/"
    gt_files = [a.truth_contigs] if a.truth_contigs else [base + "gsa_mapping_new.tsv", base + "gsa_mapping.tsv"]
    tax = Taxonomy(a.taxdb)
    pred_prof = load_profile_any(a.pred_profile, tax)
    truth_prof = load_profile_any(a.truth_profile, tax)
    need_pred = all(not pred_prof[r] for r in RANKS)
    need_truth = all(not truth_prof[r] for r in RANKS)
    lens = fasta_lengths([a.pred_fasta, a.truth_fasta]) if (need_pred or need_truth) else {}
    if need_pred:
        print("[INFO] Rebuilding predicted profile from per‑contig classifications.", file=sys.stderr)
        pred_prof = profiles_from_contig_maps(
            preds_taxid_from_classified(a.pred_contigs, tax, load_id_map(a.taxmap), a.paf), lens, tax)
    if need_truth:
        print("[INFO] Rebuilding truth profile from contig mapping.", file=sys.stderr)
        gt_map: Dict[str, str] = {}
        for g in gt_files:
            gt_map.update(load_gt_contigs(g))
        truth_prof = profiles_from_contig_maps(gt_map, lens, tax)

    def row(rank):
        l1, bc = l1_and_braycurtis(pred_prof[rank], truth_prof[rank])
        return (l1, bc) + prf_presence(pred_prof[rank], truth_prof[rank], a.presence_thresh)

    rows = {r: row(r) for r in RANKS}
    with open(os.path.join(a.outdir, "profile_summary.tsv"), "w", newline="") as w:
        wr = csv.writer(w, delimiter="\t")
        wr.writerow(["rank", "L1_total_variation_pctpts", "BrayCurtis_pct", "Precision_%", "Recall_%", "F1_%", "TP", "FP", "FN"])
        for r in RANKS:
            l1, bc, pr, rc, f1, tp, fp, fn = rows[r]
            wr.writerow([r, f"{l1:.4f}", f"{bc:.4f}", f"{pr:.2f}", f"{rc:.2f}", f"{f1:.2f}", tp, fp, fn])
    print("# Profile-level metrics (per rank)")
    for r in RANKS:
        l1, bc, pr, rc, f1, tp, fp, fn = rows[r]
        print(f"{r:14s}  L1={l1:.3f}  BC={bc:.3f}%  P/R/F1={pr:.1f}/{rc:.1f}/{f1:.1f}% (TP={tp}, FP={fp}, FN={fn})")
    print("\n# Contig-level accuracy")
    c = eval_contigs(a.pred_contigs, gt_files, tax, a.outdir, pred_fasta=a.pred_fasta, gt_fasta=a.truth_fasta,
                     threads=a.threads, taxmap_path=a.taxmap, paf_path=a.paf)
    usable, exact = c["usable_pairs"], c["exact"]
    print(f"Exact TaxID: {exact}/{usable} ({(100.0 * exact / usable if usable else 0.0):.2f}%)")
    for r in RANKS:
        m = c["per_rank"][r]
        print(f"{r:14s}  n={m['n']:<8d}  acc={m['acc']:.2f}%")
    with open(os.path.join(a.outdir, "_debug_info.txt"), "w") as w:
        w.write(f"pred_profile_path: {a.pred_profile}\n")
        w.write(f"truth_profile_path: {a.truth_profile}\n")
        w.write(f"pred_contigs_path: {a.pred_contigs}\n")
        w.write("truth_contigs_paths:\n  " + "\n  ".join([g for g in gt_files if g]) + "\n")
        w.write(f"pred_fasta: {a.pred_fasta}\n")
        w.write(f"truth_fasta: {a.truth_fasta}\n")
        w.write(f"taxdb: {a.taxdb}\n")
        w.write(f"taxmap: {a.taxmap}\n")
        w.write(f"paf: {a.paf}\n")
    print(f"\n[WROTE] {os.path.join(a.outdir, 'profile_summary.tsv')}")
    print(f"[WROTE] {os.path.join(a.outdir, 'contigs_exact.tsv')}")
    print(f"[WROTE] {os.path.join(a.outdir, 'contigs_per_rank.tsv')}")
    print(f"[WROTE] debug: {os.path.join(a.outdir, '_debug_info.txt')}")
    return 0

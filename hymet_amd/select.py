"""Candidate selection between the screen and the mapper (host-side text logic).

  * scripts/mash.sh:15-16  `sort -u -k5,5` then `sort -gr` of the screen rows (LC_ALL=C)
  * scripts/mash.sh:19-55  adaptive identity threshold (0.90 down to 0.70 by 0.02 in bc
                           decimal arithmetic, strict '>', fallback 0.71)
  * run_hymet_cami.sh:92-98 union of the per-DB selections, `sort -u` (LC_ALL=C byte order)
  * scripts/limit_candidates.py -- best score per candidate over the sorted screen tables,
    stable sort by (-score, input order), optional per-species dedupe, cap at --max
These operate on at most a few thousand rows; they stay on the host.
"""
from __future__ import annotations

import csv
import os
import re
from decimal import Decimal
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

_FIELD = re.compile(r"[ \t]*[^ \t]*")
_NUM = re.compile(r"[+-]?(?:(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?|inf(?:inity)?|nan)", re.I)


def _key5(line: str) -> bytes:
    """GNU sort key -k5,5 with default blank separation (leading blanks included)."""
    pos = 0
    for _ in range(4):
        m = _FIELD.match(line, pos)
        pos = m.end()
    return _FIELD.match(line, pos).group(0).encode()


def sort_unique_k5(rows: Sequence[str]) -> List[str]:
    seen = set()
    out = []
    for r in sorted(rows, key=_key5):          # Python's sort is stable: first of a run wins
        k = _key5(r)
        if k not in seen:
            seen.add(k)
            out.append(r)
    return out


def _gnum(line: str) -> float:
    m = _NUM.match(line.lstrip(" \t"))
    return float(m.group(0)) if m else float("-inf")


def sort_gr(rows: Sequence[str]) -> List[str]:
    """sort -gr: numeric descending; equal numbers by the reversed byte comparison."""
    return sorted(rows, key=lambda r: (_gnum(r), r.encode()), reverse=True)


def min_candidates(n_files: int) -> int:
    return max(int(float(Decimal(n_files) * Decimal("3.25")) + 0.5), 5)


def _bc(d: Decimal) -> str:
    s = format(d, "f")
    return s[1:] if s.startswith("0.") else s


def threshold_walk(rows: Sequence[str], initial: str = "0.9", n_files: int = 1):
    """scripts/mash.sh:23-55.  Returns (threshold as printed, top-hit rows, selected names =
    cut -f5, the script's stdout lines from the walk on)."""
    vals = []
    for r in rows:
        f = r.split()
        try:
            vals.append(float(f[0]) if f else 0.0)
        except ValueError:
            vals.append(0.0)
    need = min_candidates(n_files)
    cur, cur_s = Decimal(initial), initial
    best, found, count, log = "0.71", False, 0, []
    while cur >= Decimal("0.70"):
        t = float(cur_s)
        count = sum(v > t for v in vals)
        log += [f"Testing threshold: {cur_s}", f"Candidates found: {count}"]      # mash.sh:35-36
        if count >= need:
            best, found = cur_s, True
            break
        cur -= Decimal("0.02")
        cur_s = _bc(cur)
    t = float(best)
    top = [r for r, v in zip(rows, vals) if v > t]
    if not found:
        count = len(top)
        log.append("No suitable threshold found. Using 0.70.")                     # mash.sh:47-51
    log += ["====================================", f"Final threshold used: {best}", f"Candidates found: {count}",
            "===================================="]
    names = [(r.split("\t") + [""] * 5)[4] for r in top]
    return best, top, names, log


def select_threshold(rows: Sequence[str], initial: str = "0.9", n_files: int = 1) -> Tuple[str, List[str], List[str]]:
    """Returns (threshold as printed, top-hit rows, selected names = cut -f5)."""
    best, top, names, _ = threshold_walk(rows, initial, n_files)
    return best, top, names


def union_sorted(*lists: Iterable[str]) -> List[str]:
    u = set()
    for l in lists:
        u.update(l)
    return sorted(u, key=lambda s: s.encode())


def best_scores(tables: Sequence[Sequence[str]]) -> Dict[str, float]:
    """limit_candidates.py:97-122 load_scores over in-memory screen tables."""
    scores: Dict[str, float] = {}
    for rows in tables:
        for line in rows:
            if not line.strip():
                continue
            p = line.rstrip("\n").split("\t")
            if len(p) < 5:
                continue
            c = p[4].strip()
            if not c:
                continue
            try:
                s = float(p[0])
            except ValueError:
                continue
            if c not in scores or s > scores[c]:
                scores[c] = s
    return scores


def read_scores(paths: Sequence[str]) -> Dict[str, float]:
    tables = []
    for p in paths:
        try:
            with open(p, "r", encoding="utf-8", errors="ignore") as f:
                tables.append(f.read().split("\n"))
        except OSError:
            continue
    return best_scores(tables)


def species_map(assembly_dir: Optional[str]) -> Dict[str, Tuple[str, str]]:
    """limit_candidates.py:139-160 from local assembly_summary_*.txt only (never downloads)."""
    m: Dict[str, Tuple[str, str]] = {}
    if not assembly_dir:
        return m
    for name in ("assembly_summary_refseq.txt", "assembly_summary_genbank.txt"):
        path = os.path.join(assembly_dir, name)
        if not os.path.exists(path):
            continue
        with open(path, "r", encoding="utf-8", errors="ignore") as f:
            for row in csv.reader(f, delimiter="\t"):
                if not row or row[0].startswith("#") or len(row) < 8:
                    continue
                acc = row[0].strip()
                sp = (row[6] or row[5]).strip() if len(row) > 6 else row[5].strip()
                org = row[7].strip() if len(row) > 7 else ""
                if acc:
                    m[acc] = (sp or acc, org or acc)
    return m


def limit(names: Sequence[str], scores: Dict[str, float], max_n: int, dedupe: bool = False,
          smap: Optional[Dict[str, Tuple[str, str]]] = None) -> List[str]:
    smap = smap or {}
    keyed = []
    for i, n in enumerate(names):
        pieces = n.split("_", 2)
        acc = f"{pieces[0]}_{pieces[1]}" if len(pieces) >= 2 else n
        key = smap.get(acc, (acc, acc))[0] if dedupe else n
        keyed.append((-scores.get(n, float("-inf")), i, n, key))
    keyed.sort(key=lambda t: (t[0], t[1]))
    out, seen = [], set()
    for _, _, n, key in keyed:
        if key in seen:
            continue
        seen.add(key)
        out.append(n)
        if max_n > 0 and len(out) >= max_n:
            break
    return out

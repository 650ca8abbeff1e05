"""The reference's real Zymo data as test inputs (SURVEY.md §4 fixtures; §8(d) C1/C2).

* tests/golden/zymo/genomes/<species>/*.fna.gz: the 25 real genomes the reference ships
  (case/truth/zymo_refs/genomes, 63 sequences, 107.5 Mbp; copied by make_zymo_fixture.py);
* tests/golden/classify/zymo.paf: the real minimap2 PAF of the Zymo mock-community
  contigs against those references (case/truth/zymo_mc/zymo_mc_vs_refs.paf, 2,500 lines,
  1,043 contigs, 60 targets, 45 of which ship).

The contig FASTA itself is absent, so queries are re-cut from the genomes at the fixture's
primary-hit intervals: 322 contigs have a primary line on a shipped target (889 of the
2,500 lines fall on shipped targets).  Never reads /root/reference.
"""
from __future__ import annotations

import gzip
import hashlib
import json
from functools import lru_cache
from pathlib import Path

import numpy as np

GOLD = Path(__file__).resolve().parent / "golden"
ZYMO = GOLD / "zymo"
COMP = bytes.maketrans(b"ACGTacgtNn", b"TGCAtgcaNn")


def revcomp(s: bytes) -> bytes:
    return s[::-1].translate(COMP)


@lru_cache(maxsize=1)
def manifest():
    return json.loads((ZYMO / "manifest.json").read_text())


def check_manifest():
    for m in manifest():
        data = (ZYMO / "genomes" / m["species"] / m["file"]).read_bytes()
        assert len(data) == m["bytes"] and hashlib.sha256(data).hexdigest() == m["sha256"], m["file"]


def _parse(data: bytes):
    out, name, chunks = [], None, []
    for line in data.split(b"\n"):
        if line.startswith(b">"):
            if name is not None:
                out.append((name, b"".join(chunks)))
            name, chunks = line[1:].split()[0].decode(), []
        elif name is not None:
            chunks.append(line.strip())
    if name is not None:
        out.append((name, b"".join(chunks)))
    return out


@lru_cache(maxsize=1)
def genome_files():
    """[(species, gcf file name, [(seq name, bytes), ...])] in manifest (sorted) order."""
    return [(m["species"], m["file"], _parse(gzip.decompress((ZYMO / "genomes" / m["species"] / m["file"]).read_bytes())))
            for m in manifest()]


def sequences(species=None):
    """Every genome sequence, file by file (combined_genomes.fasta order)."""
    return [(n, s) for sp, _, recs in genome_files() if species is None or sp in species for n, s in recs]


@lru_cache(maxsize=1)
def seq_map():
    return dict(sequences())


def fixture_paf():
    return [l.split("\t") for l in (GOLD / "classify" / "zymo.paf").read_text().splitlines() if l]


def recut_queries(species=None):
    """One query per fixture contig with a primary line on a shipped target, cut at the
    first such line (minimap2 prints a query's regions by score): the target interval
    ts..te, reverse-complemented for '-' (the contig itself is absent).  Returns
    [(qname, seq, fixture line fields)] in fixture order."""
    seqs = seq_map()
    allowed = None if species is None else {n for n, _ in sequences(species)}
    out, seen = [], set()
    for p in fixture_paf():
        if p[0] in seen or p[12] != "tp:A:P" or p[5] not in seqs:
            continue
        seen.add(p[0])
        if allowed is not None and p[5] not in allowed:
            continue
        ts, te = int(p[7]), int(p[8])
        s = seqs[p[5]][ts:te]
        out.append((p[0], revcomp(s) if p[4] == "-" else s, p))
    return out


def primary_agreement(queries, paf_lines):
    """Per re-cut query, compare our FIRST primary line with the fixture's: same target and
    strand, and our target interval covering >= 90 % of the fixture's.  Returns counts and
    the mapq agreement where the fixture's mapq is 60.  A different target is a `tie` when
    the fixture's own primary had s1 == s2 (mapq 0: another strain scores the same and
    minimap2's hash tie-break, seeded by the query, picked one) and ours is among the
    fixture's lines for that query."""
    fix_targets = {}
    for p in fixture_paf():
        fix_targets.setdefault(p[0], set()).add(p[5])
    ours = {}
    for l in paf_lines:
        p = l.split("\t")
        if p[12] == "tp:A:P" and p[0] not in ours:
            ours[p[0]] = p
    n = hit = strand = ov90 = mq60 = mq60_ok = ties = 0
    misses = []
    for qn, _, f in queries:
        n += 1
        g = ours.get(qn)
        if g is None:
            misses.append((qn, "unmapped"))
            continue
        same = g[5] == f[5]
        hit += same
        strand += same and g[4] == f[4]
        if same:
            a0, a1, b0, b1 = int(g[7]), int(g[8]), int(f[7]), int(f[8])
            ov = max(0, min(a1, b1) - max(a0, b0)) / max(1, b1 - b0)
            ov90 += ov >= 0.9
        else:
            tags = dict(t.split(":", 1) for t in f[12:] if t.count(":") >= 2)
            tie = tags.get("s1") == tags.get("s2") and g[5] in fix_targets.get(qn, ())
            ties += tie
            misses.append((qn, f"{g[5]} vs fixture {f[5]}" + (" (fixture tie s1 == s2)" if tie else "")))
        if f[11] == "60":
            mq60 += 1
            mq60_ok += g[11] == "60"
    return {"queries": n, "same_target": hit, "same_strand": strand, "overlap90": ov90, "fixture_mapq60": mq60,
            "mapq60_agree": mq60_ok, "ties": ties, "misses": misses}


def c2_contigs(seed=1):
    """the 1,043 fixture contigs with their exact lengths (col 2); each
    is re-cut from its first primary hit placed as the alignment places it (the contig's
    qs..qe over the target's ts..te, clipped to the target), the rest -- primary targets
    that do not ship (Cryptococcus, 726 contigs) -- from one seeded synthetic 20 Mbp genome."""
    seqs = seq_map()
    rng = np.random.default_rng(seed)
    synth = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, 20_000_000)].tobytes()
    out, seen = [], {}
    first_primary = {}
    for p in fixture_paf():
        seen.setdefault(p[0], int(p[1]))
        if p[12] == "tp:A:P":
            first_primary.setdefault(p[0], p)
    for qn, L in seen.items():
        p = first_primary.get(qn)
        if p is not None and p[5] in seqs and len(seqs[p[5]]) >= L:
            t = seqs[p[5]]
            qs, qe, ts = int(p[2]), int(p[3]), int(p[7])
            st = ts - qs if p[4] == "+" else ts - (L - qe)
            st = min(max(0, st), len(t) - L)
            s = t[st:st + L]
            out.append((qn, revcomp(s) if p[4] == "-" else s))
        else:
            st = int(rng.integers(0, len(synth) - L)) if L < len(synth) else 0
            out.append((qn, synth[st:st + L]))
    return out


def expected_secondaries(q_entry):
    """The fixture's secondary lines of one re-cut query that the re-cut can reproduce: on a
    shipped target and lying (>= 90 % of their query span) inside the query interval of the
    primary line the query was re-cut from.  Returns {(target, strand)}."""
    seqs = seq_map()
    qn, _, f = q_entry
    fqs, fqe = int(f[2]), int(f[3])
    out = set()
    for p in _fixture_by_query().get(qn, ()):
        if p[12] != "tp:A:S" or p[5] not in seqs:
            continue
        qs, qe = int(p[2]), int(p[3])
        if max(0, min(qe, fqe) - max(qs, fqs)) >= 0.9 * max(1, qe - qs):
            out.add((p[5], p[4]))
    return out


@lru_cache(maxsize=1)
def _fixture_by_query():
    by = {}
    for p in fixture_paf():
        by.setdefault(p[0], []).append(p)
    return by


def secondary_agreement(queries, paf_lines, relaxed_lines=None):
    """Secondary (tp:A:S) lines against the real minimap2 fixture, per re-cut query, as
    (target, strand) sets.  recall: the fixture's in-interval secondaries
    (expected_secondaries) that we also report; precision: our secondaries whose (target,
    strand) the fixture lists for that query (any line type).  relaxed_lines: the same
    queries mapped with pri_ratio = 0 and best_n = 1000; a miss that appears there was
    dropped by mm_select_sub's pri_ratio test (the re-cut query is the primary target's own
    sequence, so its primary scores higher than the real contig's did) -- `explained`."""
    by = _fixture_by_query()

    def sets(lines):
        d = {}
        for l in lines:
            p = l.split("\t")
            if p[12] == "tp:A:S":
                d.setdefault(p[0], set()).add((p[5], p[4]))
        return d

    ours = sets(paf_lines)
    relaxed = sets(relaxed_lines) if relaxed_lines is not None else {}
    relaxed_all = {}
    for l in relaxed_lines or ():
        p = l.split("\t")
        relaxed_all.setdefault(p[0], set()).add((p[5], p[4]))
    exp_n = rec = got_n = prec = explained = 0
    misses, extras = [], []
    for entry in queries:
        qn = entry[0]
        exp = expected_secondaries(entry)
        got = ours.get(qn, set())
        listed = {(p[5], p[4]) for p in by.get(qn, ())}
        exp_n += len(exp)
        rec += len(exp & got)
        got_n += len(got)
        prec += len(got & listed)
        for e in sorted(exp - got):
            ok = e in relaxed_all.get(qn, set())
            explained += ok
            misses.append((qn, e, "pri_ratio" if ok else "no chain"))
        extras.extend((qn, e) for e in sorted(got - listed))
    return {"expected": exp_n, "recalled": rec, "ours": got_n, "ours_listed": prec, "misses_explained": explained,
            "misses": misses, "extras": extras}

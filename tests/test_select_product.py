"""hymet_amd.select (product host code) vs the reference-pinned goldens and the oracle."""
import json
import random
from pathlib import Path

import pytest

from hymet_amd import select as sel
from oracle import select_oracle as so

LIM = Path(__file__).resolve().parent / "golden" / "limit"
LCASES = json.loads((LIM / "cases.json").read_text())


@pytest.mark.parametrize("case", LCASES, ids=[Path(c["expect"]).stem for c in LCASES])
def test_limit_matches_reference_goldens(case):
    names = [l.strip() for l in (LIM / "selected.txt").read_text().splitlines() if l.strip()]
    scores = sel.read_scores([str(LIM / t) for t in case["tabs"]])
    got = sel.limit(names, scores, case["max"], dedupe=case["dedupe"])
    assert ("".join(n + "\n" for n in got)).encode() == (LIM / case["expect"]).read_bytes()


def _rows(rng, n):
    rows = []
    for i in range(n):
        ident = rng.choice(["1", "0.95", "0.9", "0.899999", "%g" % rng.random(), "0.88", "0.7", "0.71", "0.69"])
        name = rng.choice([f"GCF_{rng.randrange(50):06d}.1_x", "plain", "zz", "A b"])
        rows.append(f"{ident}\t{rng.randrange(1000)}/1000\t{rng.randrange(9)}\t{rng.random():g}\t{name}\t[1 seqs] c {i}")
    return rows


def test_selection_text_stages_match_oracle():
    rng = random.Random(5)
    for trial in range(300):
        rows = _rows(rng, rng.randrange(0, 40))
        a = sel.sort_gr(sel.sort_unique_k5(rows))
        b = so.sort_gr(so.sort_unique_k5(rows))
        assert a == b
        init = rng.choice(["0.9", "0.90", "0.8", "0.95"])
        nf = rng.randrange(1, 4)
        t1, top1, n1 = sel.select_threshold(a, init, nf)
        t2, top2, n2, _ = so.select_threshold(b, init, nf)
        assert (t1, top1, n1) == (t2, top2, n2)
    assert sel.union_sorted(["b", "a"], ["B"]) == so.union_sorted(["b", "a"], ["B"])

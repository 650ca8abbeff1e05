"""limit_candidates oracle pinned against the reference script's own outputs
(tests/golden/limit), plus known-answer tests for the mash.sh text stages written
from the script text (scripts/mash.sh:15-55) -- mash/bc/awk are absent here."""
import json
from pathlib import Path

import pytest

from oracle import select_oracle as so

LIM = Path(__file__).resolve().parent / "golden" / "limit"
LCASES = json.loads((LIM / "cases.json").read_text())


@pytest.mark.parametrize("case", LCASES, ids=[Path(c["expect"]).stem for c in LCASES])
def test_limit_oracle(case):
    names = [l.strip() for l in (LIM / "selected.txt").read_text().splitlines() if l.strip()]
    scores = so.load_scores([LIM / t for t in case["tabs"]])
    chosen, _ = so.limit_candidates(names, scores, case["max"], dedupe=case["dedupe"])
    assert ("".join(c + "\n" for c in chosen)).encode() == (LIM / case["expect"]).read_bytes()


def test_threshold_walk_stops_at_first_sufficient():
    lines = [f"0.9{i}\t1/1000\t1\t0\tr{i}\tc" for i in range(3)] + [f"0.87\t1/1000\t1\t0\ts{i}\tc" for i in range(3)]
    t, top, sel, log = so.select_threshold(so.sort_gr(lines), "0.9")
    assert log == [("0.9", 2), (".88", 3), (".86", 6)]
    assert t == ".86" and len(top) == 6 and sel[:2] == ["r2", "r1"]


def test_threshold_strict_greater_and_fallback():
    # identity exactly == threshold is NOT selected (awk '$1 > t'); nothing reaches 5 -> 0.71
    lines = ["0.9\t1/1\t1\t0\ta\tc", "0.72\t1/1\t1\t0\tb\tc", "0.71\t1/1\t1\t0\tc\tc"]
    t, top, sel, log = so.select_threshold(so.sort_gr(lines), "0.9")
    assert t == "0.71" and sel == ["a", "b"]
    assert log[-1][0] == ".70" and len(log) == 11


def test_min_candidates():
    assert [so.min_candidates(n) for n in (1, 2, 3, 4, 10)] == [5, 7, 10, 13, 33]


def test_sort_u_k5_keeps_first_in_input_order_and_sort_gr_ties():
    lines = ["0.5\t1/1\t1\t0\tB\tfirst", "0.7\t1/1\t1\t0\tA\tx", "0.9\t1/1\t1\t0\tB\tsecond"]
    u = so.sort_unique_k5(lines)
    assert u == ["0.7\t1/1\t1\t0\tA\tx", "0.5\t1/1\t1\t0\tB\tfirst"]
    g = so.sort_gr(["0.5\ta", "0.5\tb", "1\tz", "0.75\tq"])
    assert g == ["1\tz", "0.75\tq", "0.5\tb", "0.5\ta"]


def test_union_sorted_bytewise():
    assert so.union_sorted(["b", "a"], ["B", "a"]) == ["B", "a", "b"]


def test_identity_and_pvalue_formulas():
    assert so.estimate_identity(1000, 1000, 21) == 1.0
    assert so.estimate_identity(0, 1000, 21) == 0.0
    assert abs(so.estimate_identity(500, 1000, 21) - 0.5 ** (1 / 21)) < 1e-15
    assert so.p_value_within(0, 10**6, 4.0 ** 21, 1000) == 1.0
    # binomial tail sanity vs exact summation
    import math
    n, p = 50, 0.03
    for k in range(0, 10):
        exact = sum(math.comb(n, j) * p ** j * (1 - p) ** (n - j) for j in range(k + 1, n + 1))
        assert abs(so.binomial_q(k, p, n) - exact) <= 1e-12 * max(1.0, exact)
    assert so.fmt_g(0.9876543) == "0.987654" and so.fmt_g(1.0) == "1" and so.fmt_g(1.5e-45) == "1.5e-45"

"""Checks of the minimap2 restatement (oracle/mm_oracle.c).

minimap2 itself is absent so the mapping path is parity-UNPINNED; what the
reference does pin is the PAF fixture case/truth/zymo_mc/zymo_mc_vs_refs.paf (copied to
tests/golden/classify/zymo.paf): its tag layout and, for every primary line, the mapq that
mm_set_mapq derives from (s1, s2, cm, rl).  Self-consistency properties cover the rest."""
import ctypes
from pathlib import Path

import numpy as np
import pytest

from oracle import oracle_lib as ol
from tests._data import mutate, rand_seq, revcomp

PAF = Path(__file__).resolve().parent / "golden" / "classify" / "zymo.paf"


def _tags(p):
    return {t.split(":")[0]: t.split(":", 2)[2] for t in p[12:]}


def test_fixture_tag_layout_matches_writer():
    for line in PAF.read_text().splitlines():
        p = line.split("\t")
        assert len(p) in (17, 18)
        keys = [t[:5] for t in p[12:]]
        prim = p[12] == "tp:A:P"
        assert keys == (["tp:A:", "cm:i:", "s1:i:", "s2:i:", "dv:f:", "rl:i:"] if prim else ["tp:A:", "cm:i:", "s1:i:", "dv:f:", "rl:i:"])
        assert int(_tags(p)["s1"]) >= 40  # min chain score
        if not prim:
            assert p[11] == "0"


def test_fixture_mapq_reproduced_by_set_mapq():
    L = ol._mm_lib()
    L.mmo_mapq_one.restype = ctypes.c_int
    L.mmo_mapq_one.argtypes = [ctypes.c_int] * 4 + [ctypes.c_int64, ctypes.c_int, ctypes.c_int]
    rows = [l.split("\t") for l in PAF.read_text().splitlines()]
    by_q = {}
    for p in rows:
        by_q.setdefault(p[0], []).append(p)
    n_prim = n_ok0 = 0
    for q, ps in by_q.items():
        prims = [p for p in ps if p[12] == "tp:A:P"]
        sum_sc = sum(int(_tags(p)["s1"]) for p in prims)
        for p in prims:
            t = _tags(p)
            n_prim += 1
            args = (int(t["s1"]), int(t["s2"]), int(t["cm"]))
            rl = int(t["rl"])
            got = [L.mmo_mapq_one(*args, n_sub, sum_sc, rl, 40) for n_sub in range(0, 64)]
            assert int(p[11]) in got, (q, p[11], got[:4])
            n_ok0 += got[0] == int(p[11])
    assert n_prim == 1432
    assert n_ok0 / n_prim > 0.85  # most primaries have no sub-optimal chain with more anchors


@pytest.fixture(scope="module")
def toy():
    rng = np.random.default_rng(3)
    g = [rand_seq(rng, 250_000) for _ in range(4)]
    g.append(mutate(rng, g[0], 0.02))           # a strain of target 0
    idx = ol.MmIndex(g, names=[f"t{i}" for i in range(len(g))])
    opt = ol.asm10_opt()
    ol._mm_lib().mmo_opt_update_mid_occ(ctypes.byref(opt), idx.h)
    return rng, g, idx, opt


def test_sketch_is_strand_symmetric(toy):
    rng, g, idx, opt = toy
    s = g[1][:5000]
    a = ol.mm_sketch(s)
    b = ol.mm_sketch(revcomp(s))
    # canonical minimizers: the same hash multiset on both strands
    assert sorted(a[:, 0] >> np.uint64(8)) == sorted(b[:, 0] >> np.uint64(8))
    pos = (a[:, 1] & np.uint64(0xFFFFFFFF)) >> np.uint64(1)
    assert (np.diff(pos.astype(np.int64)) >= 0).all()
    assert 0.15 < len(a) / len(s) < 0.22  # density ~ 2/(w+1)


def test_index_content(toy):
    rng, g, idx, opt = toy
    keys, koff, pos = idx.export()
    assert (np.diff(keys.astype(np.float64)) > 0).all()
    for j in rng.integers(0, len(keys), 50):
        seg = pos[koff[j]:koff[j + 1]]
        assert (np.diff(seg.astype(np.float64)) >= 0).all()
    assert koff[-1] == sum(len(ol.mm_sketch(s, rid=i)) for i, s in enumerate(g))


def test_contig_maps_back_to_source(toy):
    rng, g, idx, opt = toy
    for t in range(4):
        st = int(rng.integers(0, 200_000))
        q = mutate(rng, g[t][st:st + 20_000], 0.01)
        strand = rng.random() < 0.5
        if strand:
            q = revcomp(q)
        regs, rl = ol.mm_map(idx, opt, q, f"q{t}")
        prim = regs[regs["id"] == regs["parent"]]
        best = prim[0]
        assert best["rid"] == t or (t == 0 and best["rid"] == 4)
        assert best["rev"] == int(strand)
        assert abs(best["rs"] - st) < 100 and best["qe"] - best["qs"] > 19_000
        assert best["mapq"] > 0 or t == 0


def test_repeat_and_edge_queries(toy):
    rng, g, idx, opt = toy
    for q in [b"", b"ACGT", b"N" * 500, g[2][:14], (g[1][:300] * 40), g[3][1000:1300] + b"N" * 50 + g[3][5000:9000]]:
        regs, rl = ol.mm_map(idx, opt, q, "edge")
        assert (regs["qe"] <= len(q)).all()


def test_map_from_threads_matches_sequential(toy):
    """bench.py's CPU baseline maps from worker threads (the C mapper releases the GIL): the
    oracle keeps no shared mutable state, so threaded results equal sequential ones."""
    from concurrent.futures import ThreadPoolExecutor
    _, refs, idx, opt = toy
    rng = np.random.default_rng(5)
    qs = []
    for i in range(24):
        t = int(rng.integers(0, len(refs)))
        L = int(rng.integers(2000, 20000))
        st = int(rng.integers(0, len(refs[t]) - L))
        s = mutate(rng, refs[t][st:st + L], 0.02)
        qs.append((f"q{i}", revcomp(s) if i % 3 == 0 else s))
    seq = [ol.mm_map(idx, opt, s, n) for n, s in qs]
    with ThreadPoolExecutor(8) as ex:
        par = list(ex.map(lambda q: ol.mm_map(idx, opt, q[1], q[0]), qs * 3))
    for k, (regs, rl) in enumerate(par):
        sr, srl = seq[k % len(qs)]
        assert rl == srl
        np.testing.assert_array_equal(regs, sr)

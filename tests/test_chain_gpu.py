"""Chaining DP (lchain.c mg_lchain_rmq f[]/p[]) on the GPU vs the oracle restatement, on
crafted anchor sets: long colinear groups (windows far beyond the LDS ring), dense repeats
(window > 512 summary blocks and the rmq_size_cap), integer-grid ties (canonical T2), the
index-0 quirk, and both asm10 passes (bw 1k / long join bw_long 100k)."""
import ctypes

import numpy as np
import pytest

from tests._anchors import PEN_GAP, assemble, colinear, pack

pytestmark = pytest.mark.gpu

PASSES = {"first": (10000, 1000, 1000), "long": (10000, 1000, 100000)}


@pytest.fixture(scope="module")
def gpu():
    from hymet_amd._lib import Gpu
    return Gpu(0)


def gpu_chain(gpu, x, y, max_dist, inner, bw, skip=25, cap=100000):
    n = len(x)
    f = np.zeros(n, np.int32)
    p = np.zeros(n, np.int64)
    x = np.ascontiguousarray(x, np.uint64)
    y = np.ascontiguousarray(y, np.uint64)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    gpu.call("hymet_mm_chain_dp", vp(x), vp(y), n, max_dist, inner, bw, skip, cap, ctypes.c_float(PEN_GAP),
             ctypes.c_float(0.0), vp(f), vp(p))
    return f, p


def oracle_chain(x, y, max_dist, inner, bw, skip=25, cap=100000):
    from oracle import oracle_lib
    a = np.stack([x, y], axis=1)
    return oracle_lib.mm_debug_chain(a, max_dist, inner, bw, skip, cap, float(PEN_GAP), 0.0)


def check(gpu, x, y, **kw):
    for name, (md, inner, bw) in PASSES.items():
        fg, pg = gpu_chain(gpu, x, y, md, inner, bw, **kw)
        fo, po = oracle_chain(x, y, md, inner, bw, **kw)
        bad = np.flatnonzero((fg != fo) | (pg != po))
        assert len(bad) == 0, f"{name}: {len(bad)} mismatches, first at {bad[0]}: gpu ({fg[bad[0]]},{pg[bad[0]]}) " \
                              f"oracle ({fo[bad[0]]},{po[bad[0]]})"


def test_chain_many_groups(gpu):
    rng = np.random.default_rng(1)
    parts = [colinear(rng, int(rng.integers(3, 3000)), rid=r, rev=int(rng.integers(2)), t0=int(rng.integers(0, 10**6)))
             for r in range(60)]
    check(gpu, *assemble(parts))


def test_chain_long_group(gpu):
    rng = np.random.default_rng(2)
    check(gpu, *assemble([colinear(rng, 60000, div=0.03), colinear(rng, 20000, rid=1, div=0.005)]))


def test_chain_dense_repeats(gpu):
    # 40k anchors inside 60 kbp of target: windows of > 512 blocks, rmq_size_cap hit with cap=20000
    rng = np.random.default_rng(3)
    tp = np.sort(rng.integers(0, 60000, 40000))
    qp = rng.integers(0, 60000, 40000)
    x, y = assemble([pack(tp, qp)])
    check(gpu, x, y)
    check(gpu, x, y, cap=20000)


def test_chain_grid_ties(gpu):
    rng = np.random.default_rng(4)
    parts = []
    for r in range(8):
        tp = np.sort(rng.integers(0, 400, 3000))
        qp = rng.integers(0, 400, 3000)
        parts.append(pack(tp, qp, rid=r))
    check(gpu, *assemble(parts))


def test_chain_index0_quirk(gpu):
    # anchor 0 shares its query position with later anchors of the same group
    tp = np.array([100, 150, 180, 200, 260, 300], np.int64)
    qp = np.array([50, 80, 50, 120, 50, 160], np.int64)
    x, y = pack(tp, qp)
    check(gpu, x, y)
    rng = np.random.default_rng(5)
    x2, y2 = colinear(rng, 500, rid=1)
    check(gpu, np.r_[x, x2], np.r_[y, y2])

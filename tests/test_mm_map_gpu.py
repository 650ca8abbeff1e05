"""GPU mapping (sketch -> seeds -> anchors -> chaining -> regions) vs the minimap2
restatement in oracle/mm_oracle.c: identical region records and PAF lines."""
import ctypes

import numpy as np
import pytest

from tests._data import add_noise, mutate, rand_seq, revcomp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    from hymet_amd._lib import Gpu
    return Gpu(0)


def _refs(rng):
    base = [rand_seq(rng, 400_000) for _ in range(3)]
    refs = list(base)
    refs.append(mutate(rng, base[0], 0.01))             # strain of target 0
    refs.append(mutate(rng, base[0], 0.05))             # a close relative
    rep = rand_seq(rng, 2_000)
    refs.append(rand_seq(rng, 50_000) + rep * 30 + rand_seq(rng, 50_000))  # repeat-rich target
    refs.append(revcomp(base[1][100_000:200_000]))      # reverse-complemented piece
    return refs


def _queries(rng, refs):
    qs = []
    for i in range(60):
        t = int(rng.integers(0, len(refs)))
        L = int(min(len(refs[t]) - 1, rng.lognormal(np.log(4000), 1.0) + 300))
        st = int(rng.integers(0, len(refs[t]) - L))
        s = mutate(rng, refs[t][st:st + L], float(rng.choice([0.0, 0.005, 0.02, 0.06])))
        if rng.random() < 0.4:
            s = revcomp(s)
        if rng.random() < 0.2:
            s = add_noise(rng, s)
        qs.append((f"ctg{i}", s))
    # chimera (two loci), edge cases
    qs.append(("chimera", refs[0][10_000:15_000] + refs[2][200_000:206_000]))
    qs.append(("tandem", rand_seq(rng, 40) * 400))
    qs.append(("tiny", refs[1][5:30]))
    qs.append(("empty", b""))
    qs.append(("allN", b"N" * 3000))
    qs.append(("long", mutate(rng, refs[1][0:300_000], 0.01)))
    # several copies of the 2 kb repeat: query minimizers of every copy hit the same target
    # positions, so anchors tie on (query, x) and are ordered by y (both strands)
    qs.append(("repeat_fwd", refs[5][49_000:62_500]))
    qs.append(("repeat_rev", revcomp(refs[5][49_500:63_000])))
    return qs


@pytest.mark.parametrize("bt_long,legacy,z_runs,resort,zm", [(None, None, None, None, None), ("4", None, None, None, None),
                                                            (None, "1", "1", None, None), (None, None, "2", None, None),
                                                            (None, None, None, "1", None), (None, None, None, None, "0,7"),
                                                            (None, None, None, None, "regions"),
                                                            (None, None, None, None, "regions_prim1")])
def test_map_matches_oracle(gpu, monkeypatch, bt_long, legacy, z_runs, resort, zm):
    """bt_long = "4": nearly every chain group takes the wave-per-group backtrack path.
    legacy = "1": anchors take the two-key sort path (used when the one-key anchor sort key
    would exceed 64 bits).  z_runs: backtrack-order groups of more ascending runs than this
    take the sort fallbacks (block bitonic / global radix) instead of the run merge.
    resort = "1": the long join re-sorts its anchors instead of compacting the first pass's.
    zm = "0,7": no merge group is staged in LDS; each is split into units of 7 entries, one
    block per unit (the path of merge groups above 6,144 entries).
    zm = "regions": every query of more than one chain takes the regions wave kernel, and from
    33 chains its global-scratch path (the path of queries above 256 chains).
    zm = "regions_prim1": the same, with one set_parent primary in registers and the rest in the
    LDS lists (the path of queries of more than 64 primaries)."""
    if zm in ("regions", "regions_prim1"):
        monkeypatch.setenv("HYMET_REG_WAVE", "1")
        monkeypatch.setenv("HYMET_REG_LDS", "32")
        if zm == "regions_prim1":
            monkeypatch.setenv("HYMET_REG_PRIM", "1")
    elif zm is not None:
        lds, unit = zm.split(",")
        monkeypatch.setenv("HYMET_ZM_LDS", lds)
        monkeypatch.setenv("HYMET_ZM_UNIT", unit)
    if resort is not None:
        monkeypatch.setenv("HYMET_RECHAIN_SORT", resort)
    if bt_long is not None:
        monkeypatch.setenv("HYMET_BT_LONG", bt_long)
    if legacy is not None:
        monkeypatch.setenv("HYMET_ANCHOR_LEGACY", legacy)
    if z_runs is not None:
        monkeypatch.setenv("HYMET_Z_RUNS", z_runs)
    from hymet_amd import mapper
    from hymet_amd.seqio import DevicePool, from_records
    from oracle import oracle_lib as ol
    rng = np.random.default_rng(21)
    refs = _refs(rng)
    names = [f"NC_{i:06d}.1" for i in range(len(refs))]
    ss = from_records([(n, "", s) for n, s in zip(names, refs)])
    part = mapper.IndexPart(gpu, ss)
    opt = mapper.MapOpt.asm10()
    opt.resolve_mid_occ(part)
    oi = ol.MmIndex(refs, names=names)
    oopt = ol.asm10_opt()
    ol._mm_lib().mmo_opt_update_mid_occ(ctypes.byref(oopt), oi.h)
    assert oopt.mid_occ == opt.mid_occ
    qs = _queries(rng, refs)
    qss = from_records([(n, "", s) for n, s in qs])
    qpool = DevicePool(gpu, qss, DevicePool.ALPHA_MINIMAP2)
    res = mapper.map_part(gpu, part, qpool, opt)
    n_mapped = 0
    for qi, (name, s) in enumerate(qs):
        oregs, orl = ol.mm_map(oi, oopt, s, name)
        gregs = res.query(qi)
        assert res.rep_len[qi] == orl or len(s) == 0, name
        assert len(gregs) == len(oregs), (name, len(gregs), len(oregs))
        for f in ("qs", "qe", "rs", "re", "rid", "rev", "mlen", "blen", "mapq", "cnt", "score", "subsc", "parent", "id", "n_sub"):
            np.testing.assert_array_equal(gregs[f], oregs[f], err_msg=f"{name}:{f}")
        np.testing.assert_array_equal(gregs["div"], oregs["div"], err_msg=name)
        g_lines = mapper.paf_lines(name, len(s), gregs, int(res.rep_len[qi]), names, ss.lengths)
        o_lines = ol.format_paf(name, len(s), oregs, orl, names, ss.lengths)
        assert g_lines == o_lines
        n_mapped += len(gregs) > 0
    assert n_mapped >= 55


def test_map_many_targets_matches_oracle(gpu):
    """An index part of 2,300 short targets: more (strand, target) bins (2^(1+12)) than the
    grouped anchor sort's LDS histogram holds, so large queries sort by coarse bins of two
    consecutive targets and then by (low target bit, rpos, y) inside them."""
    from hymet_amd import mapper
    from hymet_amd.seqio import DevicePool, from_records
    from oracle import oracle_lib as ol
    rng = np.random.default_rng(33)
    refs = [rand_seq(rng, int(rng.integers(1_500, 3_000))) for _ in range(2_300)]
    names = [f"NZ_T{i:05d}.1" for i in range(len(refs))]
    ss = from_records([(n, "", s) for n, s in zip(names, refs)])
    part = mapper.IndexPart(gpu, ss)
    opt = mapper.MapOpt.asm10()
    opt.resolve_mid_occ(part)
    oi = ol.MmIndex(refs, names=names)
    oopt = ol.asm10_opt()
    ol._mm_lib().mmo_opt_update_mid_occ(ctypes.byref(oopt), oi.h)
    qs = []
    for i in range(24):  # queries spanning 20-40 consecutive targets: > 4096 anchors each
        t = int(rng.integers(0, len(refs) - 40))
        s = b"".join(refs[t:t + int(rng.integers(20, 40))])
        qs.append((f"span{i}", mutate(rng, s, 0.01) if i % 2 else revcomp(s)))
    for i in range(24):
        t = int(rng.integers(0, len(refs)))
        qs.append((f"one{i}", mutate(rng, refs[t], 0.02)))
    qss = from_records([(n, "", s) for n, s in qs])
    qpool = DevicePool(gpu, qss, DevicePool.ALPHA_MINIMAP2)
    res = mapper.map_part(gpu, part, qpool, opt)
    for qi, (name, s) in enumerate(qs):
        oregs, orl = ol.mm_map(oi, oopt, s, name)
        gregs = res.query(qi)
        assert res.rep_len[qi] == orl, name
        g_lines = mapper.paf_lines(name, len(s), gregs, int(res.rep_len[qi]), names, ss.lengths)
        o_lines = ol.format_paf(name, len(s), oregs, orl, names, ss.lengths)
        assert g_lines == o_lines, name

"""GPU minimizer sketch + index build vs the minimap2 restatement (bit-exact)."""
import numpy as np
import pytest

from tests._data import add_noise, mutate, rand_seq, revcomp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    from hymet_amd._lib import Gpu
    return Gpu(0)


def _seqs(rng):
    g = [rand_seq(rng, int(rng.integers(1, 40_000))) for _ in range(30)]
    g += [add_noise(rng, rand_seq(rng, 20_000)) for _ in range(5)]
    g += [b"", b"A", b"ACGTACGTACGTACGT", b"N" * 100, (b"AC" * 3000), rand_seq(rng, 600) * 20, b"acgtNNacgtUUuuGGCC" * 50]
    g.append(rand_seq(rng, 2_100_000))  # long sequence: thousands of chunks
    return g


@pytest.mark.parametrize("w,k", [(10, 15), (5, 11), (19, 19), (15, 25)])
def test_sketch_matches_oracle(gpu, w, k):
    from hymet_amd import mapper
    from hymet_amd.seqio import DevicePool, from_records
    from oracle import oracle_lib as ol
    rng = np.random.default_rng(w * 100 + k)
    seqs = _seqs(rng)
    pool = DevicePool(gpu, from_records([(f"s{i}", "", s) for i, s in enumerate(seqs)]), DevicePool.ALPHA_MINIMAP2)
    x, y = mapper.sketch(gpu, pool, w, k, rid_mode=1)
    ref = [ol.mm_sketch(s, w, k, rid=i) for i, s in enumerate(seqs)]
    ref = np.concatenate([r for r in ref if len(r)])
    assert len(x) == len(ref)
    np.testing.assert_array_equal(x, ref[:, 0])
    np.testing.assert_array_equal(y, ref[:, 1])


def test_index_matches_oracle(gpu):
    from hymet_amd import mapper
    from hymet_amd.seqio import from_records
    from oracle import oracle_lib as ol
    rng = np.random.default_rng(4)
    seqs = [rand_seq(rng, 300_000) for _ in range(4)] + [b"ACGT" * 2000, b""]
    seqs.append(mutate(rng, seqs[0], 0.02))
    ss = from_records([(f"t{i}", "", s) for i, s in enumerate(seqs)])
    part = mapper.IndexPart(gpu, ss)
    hs, pos = part.export()
    oi = ol.MmIndex(seqs)
    keys, koff, opos = oi.export()
    np.testing.assert_array_equal(pos, opos)
    np.testing.assert_array_equal(hs.astype(np.uint64), np.repeat(keys, np.diff(koff)))
    assert part.max_occ(2e-4) == oi.max_occ(2e-4)
    assert part.max_occ(0.05) == oi.max_occ(0.05)



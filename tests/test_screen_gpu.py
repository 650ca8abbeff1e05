"""GPU screen vs the CPU oracle (bit-exact counts, shared, median, set size, output rows)."""
import json
from pathlib import Path

import numpy as np
import pytest

from tests._data import add_noise, mutate, rand_seq, revcomp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    from hymet_amd._lib import Gpu
    return Gpu(0)


def _make_db(rng, genomes, k, seed, s, n_decoys=50):
    from hymet_amd.msh import SketchDB
    from oracle import oracle_lib
    hl, names = [], []
    for i, g in enumerate(genomes):
        hl.append(np.sort(oracle_lib.sketch([g], k, seed, s)))
        names.append(f"GCF_{i:09d}.1_genome{i}.fna.gz")
    top = 2**63 if k > 16 else 2**31     # 32-bit sketches (k <= 16) hold x86_32 hashes
    for j in range(n_decoys):
        hl.append(np.sort(rng.integers(0, top, size=s, dtype=np.int64).astype(np.uint64) * 2 + 1))
        names.append(f"decoy_{j}")
    off = np.zeros(len(hl) + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(h) for h in hl])
    return SketchDB(k=k, seed=seed, sketch_size=s, names=names, comments=[f"[1 seqs] {n} comment" for n in names],
                    lengths=np.array([len(g) for g in genomes] + [10**6] * n_decoys), offsets=off,
                    hashes=np.concatenate(hl))


def _pool(rng, genomes, n_contigs, lo, hi, rate=0.01):
    recs = []
    for c in range(n_contigs):
        g = genomes[int(rng.integers(len(genomes)))]
        L = int(rng.integers(lo, hi))
        st = int(rng.integers(0, len(g) - L))
        s = mutate(rng, g[st:st + L], rate)
        if rng.random() < 0.5:
            s = revcomp(s)
        if rng.random() < 0.3:
            s = add_noise(rng, s)
        recs.append((f"ctg{c}", "", s))
    recs.append(("short", "", b"ACGTACGT"))   # shorter than k: skipped
    recs.append(("empty", "", b""))
    return recs


@pytest.mark.parametrize("k,seed,s", [(21, 42, 1000), (17, 7, 500), (32, 42, 200), (25, 0, 300),
                                      (16, 42, 1000), (13, 7, 400), (9, 42, 200)])
def test_screen_matches_oracle(gpu, k, seed, s):
    from hymet_amd import screen as scr
    from hymet_amd.seqio import DevicePool, from_records
    from oracle import oracle_lib, select_oracle
    rng = np.random.default_rng(k * 1000 + seed)
    genomes = [rand_seq(rng, int(rng.integers(200_000, 400_000)), gc=0.4 + 0.05 * i) for i in range(6)]
    db = _make_db(rng, genomes[:4], k, seed, s)
    recs = _pool(rng, genomes, 120, 2_000, 30_000)
    ss = from_records(recs)
    pool = DevicePool(gpu, ss, DevicePool.ALPHA_MASH)
    res = scr.screen(gpu, pool, [db])[0]
    sh, md, set_size, nk = oracle_lib.screen([r[2] for r in recs], k, seed, s, [db.ref_hashes(i) for i in range(db.n_refs)])
    assert res.n_kmers == nk
    np.testing.assert_array_equal(res.shared, sh)
    np.testing.assert_array_equal(res.median, md)
    assert res.set_size == set_size
    refs = [(db.names[i], db.comments[i], int(db.offsets[i + 1] - db.offsets[i])) for i in range(db.n_refs)]
    assert res.lines() == select_oracle.screen_lines(refs, sh, md, set_size, k)
    assert sum(1 for x in res.shared[:4] if x > 0) == 4


def test_screen_three_dbs_one_pass(gpu):
    from hymet_amd import screen as scr
    from hymet_amd.seqio import DevicePool, from_records
    from oracle import oracle_lib
    rng = np.random.default_rng(5)
    genomes = [rand_seq(rng, 150_000) for _ in range(5)]
    dbs = [_make_db(rng, genomes[i:i + 2], 21, 42, 1000, n_decoys=10) for i in range(3)]
    recs = _pool(rng, genomes, 40, 1_000, 20_000)
    pool = DevicePool(gpu, from_records(recs), DevicePool.ALPHA_MASH)
    out = scr.screen(gpu, pool, dbs)
    for db, r in zip(dbs, out):
        sh, md, set_size, nk = oracle_lib.screen([x[2] for x in recs], 21, 42, 1000, [db.ref_hashes(i) for i in range(db.n_refs)])
        np.testing.assert_array_equal(r.shared, sh)
        np.testing.assert_array_equal(r.median, md)
        assert r.set_size == set_size and r.n_kmers == nk


def test_screen_repetitive_pool_set_size(gpu):
    """A pool with fewer distinct k-mers than s exercises the candidate re-run path."""
    from hymet_amd import screen as scr
    from hymet_amd.seqio import DevicePool, from_records
    from oracle import oracle_lib
    rng = np.random.default_rng(9)
    unit = rand_seq(rng, 300)
    recs = [(f"r{i}", "", unit * 200) for i in range(20)]
    g = [rand_seq(rng, 50_000)]
    db = _make_db(rng, g, 21, 42, 1000, n_decoys=3)
    pool = DevicePool(gpu, from_records(recs), DevicePool.ALPHA_MASH)
    r = scr.screen(gpu, pool, [db])[0]
    sh, md, set_size, nk = oracle_lib.screen([x[2] for x in recs], 21, 42, 1000, [db.ref_hashes(i) for i in range(db.n_refs)])
    assert r.set_size == set_size and r.n_kmers == nk


def test_gpu_hash_kat(gpu):
    """Each KAT string is a one-k-mer record: its canonical hash must hit the table."""
    from hymet_amd import screen as scr
    from hymet_amd.msh import SketchDB
    from hymet_amd.seqio import DevicePool, from_records
    kat = json.loads((Path(__file__).resolve().parent / "golden" / "murmur3_kat.json").read_text())
    vecs = kat["zymo_canonical_k21_seed42"]
    hs = np.array([int(v["h0"], 16) for v in vecs], dtype=np.uint64)
    db = SketchDB(k=21, seed=42, sketch_size=len(vecs), names=[f"v{i}" for i in range(len(vecs))], comments=[""] * len(vecs),
                  lengths=np.ones(len(vecs), np.int64), offsets=np.arange(len(vecs) + 1, dtype=np.int64), hashes=hs)
    pool = DevicePool(gpu, from_records([(f"q{i}", "", v["s"].encode()) for i, v in enumerate(vecs)]), DevicePool.ALPHA_MASH)
    r = scr.screen(gpu, pool, [db])[0]
    # duplicates among the vectors make some counts > 1; every vector must be found
    assert (r.shared == 1).all()


def test_gpu_hash_kat_x86_32(gpu):
    """k <= 16: Mash's 32-bit sketches hash with MurmurHash3_x86_32 (KATs from an independent
    implementation); every canonical 16-mer's hash must hit the table."""
    from hymet_amd import screen as scr
    from hymet_amd.msh import SketchDB
    from hymet_amd.seqio import DevicePool, from_records
    kat = json.loads((Path(__file__).resolve().parent / "golden" / "murmur3_kat.json").read_text())
    vecs = kat["x86_32_zymo_canonical_k16_seed42"]
    hs = np.array([int(v["h32"], 16) for v in vecs], dtype=np.uint64)
    db = SketchDB(k=16, seed=42, sketch_size=len(vecs), names=[f"v{i}" for i in range(len(vecs))], comments=[""] * len(vecs),
                  lengths=np.ones(len(vecs), np.int64), offsets=np.arange(len(vecs) + 1, dtype=np.int64), hashes=hs)
    pool = DevicePool(gpu, from_records([(f"q{i}", "", v["s"].encode()) for i, v in enumerate(vecs)]), DevicePool.ALPHA_MASH)
    r = scr.screen(gpu, pool, [db])[0]
    assert (r.shared == 1).all()


@pytest.mark.parametrize("dup_frac", [0.0, 0.3, 0.9])
def test_table_canonical_index_is_the_first_holder(gpu, dup_frac):
    """hymet_screen_table_build: every DB hash's canonical index is the smallest index holding
    its key (hashes shared by references, the insert's duplicate fix-up), the all-ones key maps
    to the extra counter n, and each slot holds its key's high word and canonical index."""
    from hymet_amd import screen as scr
    from hymet_amd.msh import SketchDB
    rng = np.random.default_rng(int(dup_frac * 10) + 3)
    n = 400_000
    pool = rng.integers(0, 2**63, size=max(1, int(n * (1 - dup_frac))), dtype=np.int64).astype(np.uint64)
    h = np.concatenate([pool, rng.choice(pool, n - len(pool))]) if dup_frac else pool[:n]
    h = h[rng.permutation(len(h))]
    h[rng.choice(len(h), 3, replace=False)] = np.uint64(2**64 - 1)     # the reserved all-ones key
    per = 100
    db = SketchDB(names=[""] * (len(h) // per), comments=[""] * (len(h) // per), lengths=np.ones(len(h) // per, np.int64),
                  offsets=np.arange(len(h) // per + 1, dtype=np.int64) * per, hashes=h)
    t = scr.ScreenTable(gpu, db)
    gpu.sync()
    got = t.canon_of[:len(h)].cpu().numpy()
    _, first = np.unique(h, return_index=True)
    inv = np.unique(h, return_inverse=True)[1]
    want = first[inv].astype(np.int64)
    want[h == np.uint64(2**64 - 1)] = len(h)
    np.testing.assert_array_equal(got, want)
    tab = t.table.cpu().numpy().view(np.uint64)
    used = tab != np.uint64(2**64 - 1)
    canon = (tab[used] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    assert len(canon) == len(np.unique(h[h != np.uint64(2**64 - 1)]))     # one slot per distinct key
    np.testing.assert_array_equal(tab[used] >> np.uint64(32), h[canon] >> np.uint64(32))   # high word = key's
    keys = h[canon]
    np.testing.assert_array_equal(canon, first[np.searchsorted(np.unique(h), keys)])


def test_table_32bit_keys_hold_the_whole_key(gpu):
    """k <= 16 (Mash's 32-bit sketches): each slot holds the whole key and its canonical index,
    duplicates resolved to the first holder, and the screen's counts match a direct count."""
    from hymet_amd import screen as scr
    from hymet_amd.msh import SketchDB
    rng = np.random.default_rng(17)
    n = 200_000
    base = rng.integers(0, 2**32, size=n // 2, dtype=np.int64).astype(np.uint64)
    h = np.concatenate([base, rng.choice(base, n - len(base))])
    h = h[rng.permutation(n)]
    per = 100
    db = SketchDB(k=16, names=[""] * (n // per), comments=[""] * (n // per), lengths=np.ones(n // per, np.int64),
                  offsets=np.arange(n // per + 1, dtype=np.int64) * per, hashes=h)
    t = scr.ScreenTable(gpu, db)
    gpu.sync()
    assert t.key_bits == 32
    got = t.canon_of[:n].cpu().numpy()
    u, first, inv = np.unique(h, return_index=True, return_inverse=True)
    np.testing.assert_array_equal(got, first[inv])
    tab = t.table.cpu().numpy().view(np.uint64)
    used = tab != np.uint64(2**64 - 1)
    canon = (tab[used] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    assert len(canon) == len(u)
    np.testing.assert_array_equal(tab[used] >> np.uint64(32), h[canon])     # the whole key

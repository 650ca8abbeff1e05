"""The .msh reader pinned by hand-assembled bytes it did not write
(tests/golden/make_msh_fixtures.py): one and three segments, single- and double-far
pointers, the current reference list in either pointer slot, the old list, 32-bit (k <= 16)
and 64-bit hashes, unsorted hash lists, and older struct sizes.  The native reader
(csrc/msh.cpp, the product path) and the pure-Python one must both return expect.json; a
truncated file must fail loudly.  Host-only: no GPU call."""
import json
from pathlib import Path

import numpy as np
import pytest

from hymet_amd import msh

MSH = Path(__file__).resolve().parent / "golden" / "msh"
EXPECT = json.loads((MSH / "expect.json").read_text())


def _view(db):
    return {"k": db.k, "seed": db.seed, "sketch_size": db.sketch_size, "preserve_case": db.preserve_case,
            "noncanonical": db.noncanonical, "alphabet": db.alphabet, "names": list(db.names),
            "comments": list(db.comments), "lengths": [int(x) for x in db.lengths],
            "hashes": [[int(v) for v in db.ref_hashes(i)] for i in range(db.n_refs)]}


@pytest.mark.parametrize("name", sorted(EXPECT))
@pytest.mark.parametrize("reader", [msh.read_msh, msh.read_msh_py])
def test_hand_assembled_fixture(name, reader):
    assert _view(reader(MSH / name)) == EXPECT[name]


def test_truncated_file_fails_loudly(tmp_path):
    from hymet_amd._lib import HymetError
    data = (MSH / "v2_far32.msh").read_bytes()
    for cut in (4, 40, len(data) - 8):
        p = tmp_path / f"cut{cut}.msh"
        p.write_bytes(data[:cut])
        with pytest.raises(HymetError):
            msh.read_msh(p)
    with pytest.raises(HymetError):
        msh.read_msh(tmp_path / "missing.msh")


@pytest.mark.parametrize("name", ["bad_far_loop.msh", "bad_far_to_far.msh"])
def test_far_pointer_landing_pad_must_be_struct_or_list(name):
    """A single-far pointer's landing pad must be a struct or list pointer: one that is itself
    far (here: to itself) is rejected with HYMET_E_ARG instead of being followed."""
    from hymet_amd._lib import HymetError
    with pytest.raises(HymetError):
        msh.read_msh(MSH / name)


def test_writer_round_trip_native(tmp_path):
    rng = np.random.default_rng(3)
    hl = [np.sort(rng.integers(0, 2 ** 63, int(rng.integers(0, 50))).astype(np.uint64)) for _ in range(300)]
    off = np.zeros(len(hl) + 1, np.int64)
    off[1:] = np.cumsum([len(h) for h in hl])
    db = msh.SketchDB(names=[f"r{i}.fna" for i in range(300)], comments=[f"c{i}" * (i % 3) for i in range(300)],
                      lengths=np.arange(300, dtype=np.int64) * 7, offsets=off, hashes=np.concatenate(hl))
    msh.write_msh(db, tmp_path / "w.msh")
    got = msh.read_msh(tmp_path / "w.msh")
    assert got.names == db.names and got.comments == db.comments
    assert (got.offsets == db.offsets).all() and (got.hashes == db.hashes).all() and (got.lengths == db.lengths).all()


def test_sliced_host_hashes_fail_loudly():
    """read_msh(shard=...) leaves only this rank's slice valid in the host array; reading a
    reference outside it raises instead of returning stale pinned memory."""
    import numpy as np
    import pytest
    from hymet_amd.msh import SketchDB
    db = SketchDB(names=["a", "b", "c"], comments=["", "", ""], lengths=np.ones(3, np.int64),
                  offsets=np.array([0, 4, 8, 12], np.int64), hashes=np.arange(12, dtype=np.uint64))
    db.dev_slice = (4, 8, 4)                    # rank 1 of 3: hashes [4, 8)
    assert db.ref_hashes(1).tolist() == [4, 5, 6, 7]
    for i in (0, 2):
        with pytest.raises(RuntimeError, match="outside this rank's host slice"):
            db.ref_hashes(i)
    db.dev_slice = None
    assert db.ref_hashes(2).tolist() == [8, 9, 10, 11]

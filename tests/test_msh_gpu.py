"""The .msh hashes landed in HBM by the product loader (hymet_msh_upload / _range, csrc/msh.cpp):
whole, and as the per-rank slices a multi-GPU job loads and all-gathers (Pipeline._join_slices,
DESIGN.md §6), against the host reader on the hand-assembled fixtures (32- and 64-bit hashes,
unsorted lists) and on a DB large enough for the threaded gather (references cut by chunk,
thread and slice bounds)."""
from pathlib import Path

import numpy as np
import pytest

from hymet_amd import msh

pytestmark = pytest.mark.gpu

MSH = Path(__file__).resolve().parent / "golden" / "msh"


@pytest.fixture(scope="module")
def gpu():
    from hymet_amd._lib import Gpu
    return Gpu(0)


def _slices(gpu, path, world):
    """Every rank's slice of the DB's hashes, assembled as the all-gather would."""
    import torch
    n, parts = None, []
    for r in range(world):
        pin = torch.empty(0)

        def alloc(k):
            nonlocal pin
            pin = torch.zeros(k, dtype=torch.int64, pin_memory=True)
            return pin.numpy().view(np.uint64)

        db = msh.read_msh(path, alloc=alloc, upload=(gpu, lambda k: gpu.zeros(k, torch.int64)), shard=(r, world))
        lo, hi, c = db.dev_slice
        n = len(db.hashes)
        assert db.dev_hashes.numel() == max(world * c, 1) and lo == min(n, r * c) and hi == min(n, lo + c)
        gpu.sync()
        parts.append(db.dev_hashes[lo:hi].cpu().numpy().view(np.uint64).copy())
        np.testing.assert_array_equal(db.hashes[lo:hi], parts[-1])   # the pinned slice the DMAs read
    return np.concatenate(parts) if parts else np.zeros(0, np.uint64), n


def _fixtures(tmp_path):
    names = [p.name for p in sorted(MSH.glob("*.msh")) if not p.name.startswith("bad_")]
    out = [MSH / n for n in names]
    rng = np.random.default_rng(11)
    # 3,000 references of 0..1,500 hashes (some empty, some unsorted): ~2.2 M hashes, so the
    # gather runs threaded and its chunks, threads and slices cut references
    hl = []
    for i in range(3000):
        h = rng.integers(0, 2 ** 63, int(rng.integers(0, 1500)), dtype=np.int64).astype(np.uint64)
        hl.append(h if i % 7 == 0 else np.sort(h))
    off = np.zeros(len(hl) + 1, np.int64)
    off[1:] = np.cumsum([len(h) for h in hl])
    db = msh.SketchDB(names=[f"r{i}" for i in range(len(hl))], comments=[""] * len(hl),
                      lengths=np.ones(len(hl), np.int64), offsets=off, hashes=np.concatenate(hl))
    big = tmp_path / "big.msh"
    msh.write_msh(db, str(big))
    return out + [big]


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_upload_slices_equal_host_reader(gpu, tmp_path, world):
    for path in _fixtures(tmp_path):
        want = msh.read_msh(path).hashes
        got, n = _slices(gpu, path, world)
        assert n == len(want)
        np.testing.assert_array_equal(got, want, err_msg=f"{path.name} world {world}")


def test_whole_upload_equals_host_reader(gpu, tmp_path):
    import torch
    for path in _fixtures(tmp_path):
        want = msh.read_msh(path).hashes
        pin = []

        def alloc(k):
            pin.append(torch.zeros(k, dtype=torch.int64, pin_memory=True))
            return pin[-1].numpy().view(np.uint64)

        db = msh.read_msh(path, alloc=alloc, upload=(gpu, lambda k: gpu.zeros(k, torch.int64)))
        gpu.sync()
        assert db.dev_slice is None
        np.testing.assert_array_equal(db.dev_hashes[:len(want)].cpu().numpy().view(np.uint64), want)

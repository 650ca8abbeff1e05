"""The library's stable LSD radix sort (csrc/sort.hpp, hymet_sort_pairs_u64) vs numpy's
stable argsort on the key bits [begin, end): every tile-boundary size, partial bit ranges
(bits outside the range are ignored, as the callers rely on), heavy ties (stability)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    from hymet_amd._lib import Gpu
    return Gpu(0)


@pytest.mark.parametrize("n,begin,end,distinct", [(2, 0, 64, 0), (2047, 0, 64, 0), (2048, 0, 40, 0), (2049, 0, 16, 50),
                                                   (100_000, 8, 40, 0), (1_000_003, 0, 64, 1000), (300_000, 0, 3, 0),
                                                   (5_000_000, 0, 38, 0)])
def test_radix_sort_matches_stable_argsort(gpu, n, begin, end, distinct):
    torch = gpu.torch
    rng = np.random.default_rng(n + end)
    keys = rng.integers(0, 2 ** 63, n, dtype=np.int64).astype(np.uint64) * np.uint64(2) + np.uint64(rng.integers(0, 2))
    if distinct:
        keys = rng.choice(keys[:distinct], n)
    vals = np.arange(n, dtype=np.uint32)
    dk = torch.from_numpy(keys.view(np.int64)).to(gpu.dev)
    dv = torch.from_numpy(vals.view(np.int32)).to(gpu.dev)
    gpu.call("hymet_sort_pairs_u64", ctypes.c_void_p(dk.data_ptr()), ctypes.c_void_p(dv.data_ptr()), n, begin, end)
    mask = np.uint64(((1 << (end - begin)) - 1) if end - begin < 64 else (1 << 64) - 1)
    sub = (keys >> np.uint64(begin)) & mask
    order = np.argsort(sub, kind="stable")
    np.testing.assert_array_equal(dv.cpu().numpy().view(np.uint32), order.astype(np.uint32))
    np.testing.assert_array_equal(dk.cpu().numpy().view(np.uint64), keys[order])


@pytest.mark.parametrize("n", [1, 4095, 4096, 4097, 1_000_000, 4096 * 1024 + 7, 12_000_000])
def test_scan_exclusive_sum_and_running_max(gpu, n):
    """The library's two-launch scan (tile sums whose last block scans them, then the tile
    pass): every tile-count boundary, including more than 1024 tiles (several rounds in the
    last block), against numpy; then the running-maximum variant."""
    torch = gpu.torch
    rng = np.random.default_rng(n)
    cnt = rng.integers(0, 3000, n, dtype=np.uint32)
    d_in = torch.from_numpy(cnt.view(np.int32)).to(gpu.dev)
    d_out = torch.empty(n, dtype=torch.int64, device=gpu.dev)
    tot = ctypes.c_int64()
    for _ in range(2):   # twice: the ticket must be clear again after a call
        gpu.call("hymet_scan_u32", ctypes.c_void_p(d_in.data_ptr()), ctypes.c_void_p(d_out.data_ptr()), n, 0, ctypes.byref(tot))
        want = np.zeros(n, np.int64)
        np.cumsum(cnt[:-1], out=want[1:])
        np.testing.assert_array_equal(d_out.cpu().numpy(), want)
        assert tot.value == int(cnt.sum(dtype=np.int64))
    v = rng.integers(-2 ** 31, 2 ** 31 - 1, n, dtype=np.int64).astype(np.int32)
    d_v = torch.from_numpy(v).to(gpu.dev)
    d_m = torch.empty(n, dtype=torch.int32, device=gpu.dev)
    gpu.call("hymet_scan_u32", ctypes.c_void_p(d_v.data_ptr()), ctypes.c_void_p(d_m.data_ptr()), n, 1, None)
    np.testing.assert_array_equal(d_m.cpu().numpy(), np.maximum.accumulate(v))


def test_scan_many_tiles_while_another_stream_scans(gpu):
    """The tile-sum hand-off (sc1 stores, a vmcnt wait, then the ticket add; the last block's
    sc1 loads) at ~9,800 tiles per call, 12 calls in a row, while a second library context
    runs the same scans on its own stream from another thread: every offset and total exact
    (a stale tile sum read by the last block would shift every later offset)."""
    import threading
    torch = gpu.torch
    n = 40_000_000
    side = gpu.fork()
    rng = np.random.default_rng(5)
    cnt = [rng.integers(0, 3000, n, dtype=np.uint32) for _ in range(2)]
    want = []
    for c in cnt:
        w = np.zeros(n, np.int64)
        np.cumsum(c[:-1], out=w[1:])
        want.append((w, int(c.sum(dtype=np.int64))))
    errs = []

    def run(g, k):
        try:
            with torch.cuda.stream(g.stream):   # torch's copies on the context's own stream
                body(g, k)
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append(repr(e))

    def body(g, k):
        d_in = torch.from_numpy(cnt[k].view(np.int32)).to(g.dev)
        d_out = torch.empty(n, dtype=torch.int64, device=g.dev)
        tot = ctypes.c_int64()
        for _ in range(12):
            d_out.fill_(-1)
            g.call("hymet_scan_u32", ctypes.c_void_p(d_in.data_ptr()), ctypes.c_void_p(d_out.data_ptr()), n, 0,
                   ctypes.byref(tot))
            got = d_out.cpu().numpy()
            if tot.value != want[k][1] or not np.array_equal(got, want[k][0]):
                errs.append(f"context {k}: mismatch at {int(np.argmax(got != want[k][0]))}")
                return

    th = threading.Thread(target=run, args=(side, 1))
    th.start()
    run(gpu, 0)
    th.join()
    assert not errs, errs

"""The library's kernel-scratch cache (csrc/ctx.cpp scratch_alloc) and torch's caching
allocator share one device's HBM.  Each pool gives its unused blocks back when the other runs
out: torch's side retries after hymet_scratch_trim (hymet_amd._lib.Gpu.empty / zeros), the
library's side calls its out-of-memory hook, torch.cuda.empty_cache
(hymet_set_oom_hook, _lib._release_torch_cache)."""
import ctypes

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    from hymet_amd._lib import Gpu
    return Gpu(0)


def _cached(gpu):
    out = ctypes.c_int64()
    gpu.call("hymet_scratch_cached", ctypes.byref(out))
    return out.value


def _stats(gpu):
    out = (ctypes.c_int64 * 3)()
    gpu.call("hymet_scratch_stats", ctypes.cast(out, ctypes.c_void_p))
    return list(out)


def _big(gpu):
    """A live torch filler leaves 64 GiB free; the returned size is 60 % of what is then free:
    one such block per pool fits, two do not (a scratch size class rounds up by at most 25 %),
    and it stays under the scratch cache's cap (a block over the cap is freed, not cached)."""
    torch = gpu.torch
    gpu.trim()
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info(gpu.device)
    filler = torch.empty(max(free - (64 << 30), 1), dtype=torch.uint8, device=gpu.dev)
    free, _ = torch.cuda.mem_get_info(gpu.device)
    return int(free * 0.6) // 4096 * 4096, filler


def test_torch_allocation_takes_back_the_library_cache(gpu):
    torch = gpu.torch
    big, filler = _big(gpu)
    gpu.reserve(big)
    assert _cached(gpu) >= big
    t = gpu.empty(big, torch.uint8)       # does not fit beside the cached block
    assert t.numel() == big and _cached(gpu) == 0
    t[-1] = 7
    torch.cuda.synchronize()
    del t, filler
    torch.cuda.empty_cache()


def test_library_scratch_takes_back_the_torch_cache(gpu):
    torch = gpu.torch
    big, filler = _big(gpu)
    t = torch.empty(big, dtype=torch.uint8, device=gpu.dev)
    del t                                  # torch keeps the block reserved, unused
    assert torch.cuda.memory_reserved(gpu.device) >= big
    drops = _stats(gpu)[1]
    gpu.reserve(big)                       # hipMalloc fails, the hook empties torch's cache
    assert _stats(gpu)[1] == drops + 1
    assert _cached(gpu) >= big
    assert torch.cuda.memory_reserved(gpu.device) < big + filler.numel()
    del filler
    gpu.trim()


def test_too_large_still_fails_loudly(gpu):
    from hymet_amd._lib import HymetError
    torch = gpu.torch
    _, total = torch.cuda.mem_get_info(gpu.device)
    with pytest.raises(HymetError, match="hymet_scratch_reserve"):
        gpu.reserve(2 * total)
    with pytest.raises(torch.OutOfMemoryError):
        gpu.empty(2 * total, torch.uint8)

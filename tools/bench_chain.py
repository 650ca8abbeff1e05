"""Chaining-DP kernel timing on synthetic anchor sets (hymet_mm_chain_dp; kernel time from
the library's HIP-event profiler).  A: one long group (per-anchor latency: the tail of a
real batch), B: many typical groups (throughput)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tests._anchors import PEN_GAP, assemble, colinear  # noqa: E402


def run(gpu, x, y, bw):
    n = len(x)
    f = np.zeros(n, np.int32)
    p = np.zeros(n, np.int64)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    gpu.prof_reset()
    gpu.prof(True)
    gpu.call("hymet_mm_chain_dp", vp(x), vp(y), n, 10000, 1000, bw, 25, 100000, ctypes.c_float(PEN_GAP),
             ctypes.c_float(0.0), vp(f), vp(p))
    gpu.prof(False)
    t = gpu.prof_table()
    return sum(v[0] for k, v in t.items() if k.startswith("mm_chain"))


def main():
    rng = np.random.default_rng(0)
    A = assemble([colinear(rng, 60000, div=0.02)])
    if "--dump" in sys.argv:
        np.stack(A, axis=1).astype(np.uint64).tofile(sys.argv[sys.argv.index("--dump") + 1])
        return
    if "--dump-b" in sys.argv:  # many groups, smaller: 4000 groups
        sizes = np.clip(rng.lognormal(np.log(700), 1.0, 4000).astype(int), 3, 200000)
        B = assemble([colinear(rng, int(s), rid=i, t0=int(rng.integers(0, 10**6))) for i, s in enumerate(sizes)])
        np.stack(B, axis=1).astype(np.uint64).tofile(sys.argv[sys.argv.index("--dump-b") + 1])
        return
    from hymet_amd._lib import Gpu
    gpu = Gpu(0)
    sizes = np.clip(rng.lognormal(np.log(700), 1.0, 20000).astype(int), 3, 200000)
    B = assemble([colinear(rng, int(s), rid=i % 4000, rev=i // 4000 % 2, t0=int(rng.integers(0, 10**6)))
                  for i, s in enumerate(sizes)])
    for name, (x, y) in (("A one group", A), ("B many groups", B)):
        for bw in (1000, 100000):
            run(gpu, x, y, bw)
            ms = run(gpu, x, y, bw)
            print(f"{name:14s} n={len(x):9d} bw={bw:6d}: {ms:8.2f} ms  {ms * 1e6 / len(x):8.1f} ns/anchor", flush=True)


if __name__ == "__main__":
    main()

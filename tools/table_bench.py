"""Screen-table build in isolation (run under rocprofv3 --kernel-trace --stats): 1e8 random
hashes in 1e5 sorted lists, built 5 times; prints the host-timed build."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from hymet_amd._lib import Gpu  # noqa: E402
from hymet_amd import screen as scr  # noqa: E402
from hymet_amd.msh import SketchDB  # noqa: E402

gpu = Gpu(0)
n_ref, per = 100_000, 1000
rng = np.random.default_rng(5)
h = np.sort(rng.integers(0, 2 ** 63, (n_ref, per), dtype=np.int64).astype(np.uint64), axis=1).ravel()
db = SketchDB(names=[""] * n_ref, comments=[""] * n_ref, lengths=np.ones(n_ref, np.int64),
              offsets=np.arange(n_ref + 1, dtype=np.int64) * per, hashes=h)
d_h = torch.from_numpy(h.view(np.int64)).to(gpu.dev)
for rep in range(5):
    db.dev_hashes = d_h
    gpu.sync()
    t = time.perf_counter()
    tab = scr.ScreenTable(gpu, db)
    gpu.sync()
    print(f"build {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
    del tab

#!/usr/bin/env python3
"""GPU-box diagnostic: the chaining DP (hymet_mm_chain_dp) vs the oracle (mm_debug_chain)
on the ORACLE's anchors of every re-cut Zymo contig (tests/_zymo.py) against the 63 real
genome sequences, both asm10 passes, each run twice (a difference between the two GPU
runs is a race).  Prints one line per query with a mismatch.

    python tools/zymo_chain_debug.py [QNAME ...]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests._anchors import PEN_GAP  # noqa: E402

PASSES = {"first": (10000, 1000, 1000), "long": (10000, 1000, 100000)}


def main():
    from hymet_amd._lib import Gpu
    from oracle import oracle_lib
    from tests import _zymo as z
    seqs = z.sequences()
    q = z.recut_queries()
    if len(sys.argv) > 1:
        q = [x for x in q if x[0] in set(sys.argv[1:])]
    idx = oracle_lib.MmIndex([s for _, s in seqs], names=[n for n, _ in seqs])
    opt = oracle_lib.asm10_opt()
    oracle_lib._mm_lib().mmo_opt_update_mid_occ(ctypes.byref(opt), idx.h)
    print("mid_occ", opt.mid_occ, flush=True)
    gpu = Gpu(0)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    bad_q = 0
    for qn, s, _ in q:
        a, _ = oracle_lib.mm_debug_anchors(idx, opt, s)
        n = len(a)
        if n == 0:
            continue
        x = np.ascontiguousarray(a[:, 0])
        y = np.ascontiguousarray(a[:, 1])
        msgs = []
        for name, (md, inner, bw) in PASSES.items():
            fo, po = oracle_lib.mm_debug_chain(a, md, inner, bw, 25, 100000, float(PEN_GAP), 0.0)
            runs = []
            for _ in range(2):
                f = np.zeros(n, np.int32)
                p = np.zeros(n, np.int64)
                gpu.call("hymet_mm_chain_dp", vp(x), vp(y), n, md, inner, bw, 25, 100000, ctypes.c_float(PEN_GAP),
                         ctypes.c_float(0.0), vp(f), vp(p))
                runs.append((f, p))
            (f1, p1), (f2, p2) = runs
            race = int(((f1 != f2) | (p1 != p2)).sum())
            bad = np.flatnonzero((f1 != fo) | (p1 != po))
            if len(bad) or race:
                i = int(bad[0]) if len(bad) else -1
                gs = x >> np.uint64(32)
                g = gs[i] if i >= 0 else 0
                gsz = int((gs == g).sum()) if i >= 0 else 0
                msgs.append(f"{name}: {len(bad)} f/p mismatches (race {race}), first {i} in a group of {gsz}: "
                            f"gpu ({f1[i]},{p1[i]}) oracle ({fo[i]},{po[i]})" if i >= 0 else f"{name}: race {race}")
        if msgs:
            bad_q += 1
            print(qn, n, "anchors;", "; ".join(msgs), flush=True)
    print(f"queries {len(q)} with mismatches {bad_q}", flush=True)


if __name__ == "__main__":
    main()

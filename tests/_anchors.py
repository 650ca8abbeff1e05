"""Synthetic minimap2 anchor arrays (x = rev<<63 | rid<<32 | tpos, y = span<<32 | qpos),
sorted by x, for chaining-DP parity tests and timing."""
import numpy as np

PEN_GAP = np.float32(0.8 * 0.01 * 15)   # asm10: chain_gap_scale * 0.01 * k


def colinear(rng, n, rid=0, rev=0, t0=1000, q0=0, span=15, div=0.02, indel=0.002, spurious=0.05):
    """One colinear run of ~n anchors with substitution gaps, small indels and noise."""
    tp, qp = [], []
    t, q = t0, q0
    for _ in range(n):
        step = int(rng.integers(1, 11))
        if rng.random() < div * 5:
            step += int(rng.integers(5, 40))          # a mismatch removes minimizers
        t += step
        q += step
        if rng.random() < indel:
            d = int(rng.integers(-30, 31))
            t += max(d, 0)
            q += max(-d, 0)
        tp.append(t)
        qp.append(q)
    tp, qp = np.array(tp, np.int64), np.array(qp, np.int64)
    k = int(spurious * n)
    if k:
        tp = np.r_[tp, rng.integers(t0, t + 1, k)]
        qp = np.r_[qp, rng.integers(q0, q + 1, k)]
    return pack(tp, qp, rid, rev, span)


def pack(tp, qp, rid=0, rev=0, span=15):
    x = (np.uint64(rev) << np.uint64(63)) | (np.uint64(rid) << np.uint64(32)) | tp.astype(np.uint64)
    y = (np.uint64(span) << np.uint64(32)) | qp.astype(np.uint64)
    return x, y


def assemble(parts):
    x = np.concatenate([p[0] for p in parts])
    y = np.concatenate([p[1] for p in parts])
    o = np.lexsort((y, x))
    return x[o], y[o]

"""Screen stage: the MI355X replacement for `mash screen -p 8 -v 0.9 DB input/*.fna`
(scripts/mash.sh:14).

Device work (libhymet_gpu.so): sketch-hash tables in HBM, one pass over the packed query
pool that hashes every canonical k-mer once and probes every DB sharing (k, seed), and the
per-reference shared / median statistics.  Host work here: the pool set-size estimate from
the bottom-s candidates, Mash's identity and p-value in double, and the output lines.

Multi-GPU: every rank hashes a slice of the pooled k-mer positions; the
uint32 hit counts are summed with one all-reduce per DB (RCCL over xGMI) and the bottom-s
candidate sets are all-gathered (s x 8 B per rank) before the statistics.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from ._lib import ptr
from .msh import SketchDB

U64_MAX = (1 << 64) - 1


class ScreenTable:
    """One sketch DB resident in HBM: open-addressing key table, the canonical index of each
    slot's key and of each DB hash (hit counts live in the DB's own hash order), CSR offsets."""

    def __init__(self, gpu, db: SketchDB, pinned=None):
        """pinned: a pinned host int64 tensor whose first len(db.hashes) entries ARE the
        hashes (read_msh gathered them there): uploaded by one asynchronous DMA.  A DB read
        with read_msh(upload=...) carries its hashes in HBM already (db.dev_hashes, the DMAs
        queued on this context's stream)."""
        torch = gpu.torch
        self.gpu, self.db = gpu, db
        n = int(len(db.hashes))
        self.n_hashes = n
        self.n_slots = int(gpu.lib.hymet_screen_table_slots(n))
        self.table = gpu.empty(self.n_slots, torch.int64)   # slots: key's high word, canonical index
        self.canon_of = gpu.empty(max(n, 1), torch.int32)
        scratch = gpu.empty(max(n, 1) + 1, torch.int64)     # build scratch: duplicate keys
        dev = getattr(db, "dev_hashes", None)
        if not n:
            d_h = gpu.empty(1, torch.int64)
        elif dev is not None:
            d_h = dev
            db.dev_hashes = None    # consumed: the table build is queued behind the DMAs
        elif pinned is not None:
            d_h = pinned[:n].to(gpu.dev, non_blocking=True)
        else:
            d_h = torch.from_numpy(np.ascontiguousarray(db.hashes).view(np.int64)).to(gpu.dev)
        # the offsets first: a pageable upload waits for the stream's earlier work, and queued
        # behind the insert it would hold the host for the whole build
        self.ref_off = torch.from_numpy(np.ascontiguousarray(db.offsets, dtype=np.int64)).to(gpu.dev)
        # 32-bit sketches (k <= 16) keep the whole key in the slot: no second, dependent load of
        # the DB's hash per probe
        key_bits = 32 if db.k <= 16 else 64
        gpu.call("hymet_screen_table_build", ptr(d_h), n, ptr(self.table), self.n_slots, ptr(scratch), ptr(self.canon_of),
                 key_bits)
        # 64-bit keys: probes check full keys here; 32-bit: read by the (asynchronous) build only.
        # Either way it lives as long as the table
        self.hashes = d_h
        self.key_bits = key_bits
        del scratch


@dataclass
class ScreenResult:
    db: SketchDB
    shared: np.ndarray
    median: np.ndarray
    set_size: int
    n_kmers: int

    def lines(self, v_max: float = 0.9, identity_min: float = 0.0) -> List[str]:
        return format_screen(self.db, self.shared, self.median, self.set_size, v_max, identity_min)


def _bottom_s(values: np.ndarray, s: int) -> np.ndarray:
    u = np.unique(values.astype(np.uint64))
    return u[:s]


def count_pool(gpu, pool, tables: Sequence[ScreenTable], k: int, seed: int, s: int,
               pos_begin: int = 0, pos_end: Optional[int] = None):
    """Run the hash/probe/count kernel over pool k-mer start positions [pos_begin, pos_end).
    Returns (counts tensors, local bottom-s candidate hashes (np.uint64, sorted), n_kmers)."""
    torch = gpu.torch
    n_bases = pool.n_bases
    if pos_end is None:
        pos_end = max(0, n_bases - k + 1)
    span = max(1, pos_end - pos_begin)
    counts = [gpu.zeros(t.n_hashes + 1, torch.int32) for t in tables]   # by canonical index
    cap = 64 * s + 65536
    cand = gpu.empty(cap, torch.int64)
    cand_n = gpu.zeros(1, torch.int64)
    nk = gpu.zeros(1, torch.int64)
    frac = 16.0 * s / span
    top = hash_top(k)              # hashes are 64-bit for k > 16, 32-bit (x86_32) for k <= 16
    thr = U64_MAX if frac >= 1.0 else int(frac * float(top))
    keys_arr = (ctypes.c_void_p * 4)(*[ptr(t.table).value for t in tables])
    slots_arr = (ctypes.c_int64 * 4)(*[t.n_slots for t in tables])
    hash_arr = (ctypes.c_void_p * 4)(*[ptr(t.hashes).value for t in tables])
    nh_arr = (ctypes.c_int64 * 4)(*[t.n_hashes for t in tables])
    cnt_arr = (ctypes.c_void_p * 4)(*[ptr(c).value for c in counts])
    gpu.call("hymet_screen_count", ptr(pool.w2b), ptr(pool.wmask), n_bases, pos_begin, pos_end, k, seed,
             len(tables), keys_arr, slots_arr, hash_arr, nh_arr, cnt_arr, thr, ptr(cand), cap, ptr(cand_n), ptr(nk))
    n_kmers = int(nk.item())
    dummy = gpu.zeros(1, torch.int64)

    def rerun(thr_, cap_):
        buf = gpu.empty(cap_, torch.int64)
        cand_n.zero_()
        gpu.call("hymet_screen_count", ptr(pool.w2b), ptr(pool.wmask), n_bases, pos_begin, pos_end, k, seed,
                 0, keys_arr, slots_arr, hash_arr, nh_arr, cnt_arr, thr_, ptr(buf), cap_, ptr(cand_n), ptr(dummy))
        return buf

    while True:
        n = int(cand_n.item())
        if n > cap:  # overflow: same threshold again with an exact-size buffer (candidates only)
            cap = n
            cand = rerun(thr, cap)
            n = int(cand_n.item())
        bottom = _bottom_s(cand[:n].cpu().numpy().view(np.uint64), s)
        if len(bottom) >= s or thr == U64_MAX:
            break
        # fewer than s distinct hashes under the threshold (repetitive pool): raise it
        # monotonically and re-run the hash pass in candidates-only mode (ndb = 0)
        thr = U64_MAX if thr > top // 16 else thr * 16
        cand = rerun(thr, cap)
    return counts, bottom, n_kmers


def reduce_partials(comm, counts, bottom: np.ndarray, nk: int, s: int, tables=None):
    """Combine the ranks' partial screens of one pool: hit counts are
    summed (all-reduce, RCCL on the device tensors), the pool bottom-s sketch is the bottom
    s of the union of the ranks' candidates, and the k-mer totals add up.

    Every rank builds its own open-addressing table and parallel insertion makes slot
    positions rank-specific, but the counts are kept per canonical index (the smallest DB
    hash index holding the key, csrc/screen.hip), i.e. in the DB's own order, the same on
    every rank: they are all-reduced as they are (round 4 gathered them out of slot order
    and scattered them back, ~7 ms of random accesses per step on a 1e8-hash DB)."""
    if comm is None or comm.world <= 1:
        return counts, bottom, nk
    for c in counts:
        comm.allreduce_sum_(c)
    bottom = _bottom_s(np.concatenate(comm.allgather_np(np.asarray(bottom, np.uint64), tag="bottom")), s)
    nk = int(sum(int(x[0]) for x in comm.allgather_np(np.array([nk], dtype=np.int64), tag="n_kmers")))
    return counts, bottom, nk


def hash_top(k: int) -> int:
    """2^bits of Mash's k-mer hash: 64-bit (MurmurHash3_x64_128 word 0) for k > 16, 32-bit
    (MurmurHash3_x86_32) for k <= 16."""
    return 1 << 64 if k > 16 else 1 << 32


def set_size_from_bottom(bottom: np.ndarray, k: int = 21) -> int:
    """MinHashHeap::estimateSetSize: 2^bits * |heap| / max(heap), truncated to uint64."""
    if len(bottom) == 0:
        return 0
    return int(float(hash_top(k)) * float(len(bottom)) / float(int(bottom[-1])))


def table_stats(gpu, t: ScreenTable, counts):
    torch = gpu.torch
    n = t.db.n_refs
    sh = gpu.zeros(max(n, 1), torch.int32)
    md = gpu.zeros(max(n, 1), torch.int32)
    if n:
        gpu.call("hymet_screen_stats", ptr(t.ref_off), n, ptr(t.canon_of), ptr(counts), ptr(sh), ptr(md))
    return sh[:n].cpu().numpy().view(np.uint32).copy(), md[:n].cpu().numpy().view(np.uint32).copy()


def screen(gpu, pool, dbs: Sequence[SketchDB], tables: Optional[Sequence[ScreenTable]] = None, comm=None) -> List[ScreenResult]:
    """Screen the pool against every DB.  DBs sharing (k, seed) are probed in one pass."""
    tables = list(tables) if tables is not None else [ScreenTable(gpu, db) for db in dbs]
    results: List[Optional[ScreenResult]] = [None] * len(dbs)
    groups = {}
    for i, db in enumerate(dbs):
        if db.k < 1 or db.k > 32:
            raise ValueError(f"k={db.k}: Mash k-mer sizes are 1..32")
        if db.noncanonical:
            raise ValueError("noncanonical sketches are not supported")
        groups.setdefault((db.k, db.seed, db.preserve_case), []).append(i)
    for (k, seed, _pc), idx in groups.items():
        for j in range(0, len(idx), 4):
            chunk = idx[j:j + 4]
            s = max(dbs[i].sketch_size for i in chunk)
            n_pos = max(0, pool.n_bases - k + 1)
            if comm is not None and comm.world > 1 and comm.replicated_pool:
                b, e = comm.shard_range(n_pos)   # every rank holds the whole pool: split positions
            else:
                b, e = 0, n_pos                  # the pool is this rank's contig shard
            counts, bottom, nk = count_pool(gpu, pool, [tables[i] for i in chunk], k, seed, s, b, e)
            counts, bottom, nk = reduce_partials(comm, counts, bottom, nk, s, [tables[i] for i in chunk])
            for ci, i in enumerate(chunk):
                sh, md = table_stats(gpu, tables[i], counts[ci])
                b_i = bottom[:dbs[i].sketch_size]
                results[i] = ScreenResult(dbs[i], sh, md, set_size_from_bottom(b_i, k), nk)
    return results


# ----------------------------------------------------------- Mash output formatting
def _incbeta_cf(a, b, x):
    tiny = 4.450147717014403e-308
    eps2 = 4.440892098500626e-16
    d = 1.0 - (a + b) * x / (a + 1.0)
    d = 1.0 / (tiny if abs(d) < tiny else d)
    c = 1.0
    f = d
    m = 1
    while m <= 512:
        for num in (m * (b - m) * x / ((a - 1.0 + 2 * m) * (a + 2 * m)),
                    -(a + m) * (a + b + m) * x / ((a + 2 * m) * (a + 2 * m + 1.0))):
            d = 1.0 + num * d
            c = 1.0 + num / c
            d = tiny if abs(d) < tiny else d
            c = tiny if abs(c) < tiny else c
            d = 1.0 / d
            delta = d * c
            f *= delta
        if abs(delta - 1.0) < eps2:
            break
        m += 1
    return f


def binomial_upper_tail(k: int, p: float, n: int) -> float:
    """P(X > k) for X ~ Binomial(n, p) = I_p(k+1, n-k)  (gsl_cdf_binomial_Q)."""
    if k >= n:
        return 0.0
    a, b, x = k + 1.0, float(n - k), p
    if x <= 0.0:
        return 0.0
    if x >= 1.0:
        return 1.0
    pre = math.exp(math.lgamma(a + b) - math.lgamma(a) - math.lgamma(b) + a * math.log(x) + b * math.log1p(-x))
    if x < (a + 1.0) / (a + b + 2.0):
        return pre * _incbeta_cf(a, b, x) / a
    return 1.0 - pre * _incbeta_cf(b, a, 1.0 - x) / b


def format_screen(db: SketchDB, shared, median, set_size, v_max=0.9, identity_min=0.0) -> List[str]:
    """Mash screen output rows in sketch order: identity, shared/s, median-multiplicity,
    p-value, name, comment (C++ ostream default = %g with 6 significant digits)."""
    k = db.k
    kmer_space = math.pow(len(db.alphabet) or 4, k)
    r = 1.0 - math.pow(1.0 - 1.0 / kmer_space, float(set_size))
    out = []
    off = db.offsets
    # rows with no shared hash are dropped unless identity_min < 0: visit only the others
    # (a Python pass over every reference of a 100k-reference DB cost ~5 ms per step)
    rows = np.flatnonzero(np.asarray(shared)[:db.n_refs]) if identity_min >= 0.0 else range(db.n_refs)
    for i in rows:
        x = int(shared[i])
        if x == 0 and identity_min >= 0.0:
            continue
        sl = int(off[i + 1] - off[i])
        ident = 1.0 if x == sl else (0.0 if x == 0 else math.pow(x / sl, 1.0 / k))
        if ident < identity_min:
            continue
        pv = 1.0 if x == 0 else binomial_upper_tail(x - 1, r, sl)
        if pv > v_max:
            continue
        out.append("%g\t%d/%d\t%d\t%g\t%s\t%s" % (ident, x, sl, int(median[i]) if x else 0, pv, db.names[i], db.comments[i]))
    return out


def sketch_sequences(gpu, pool, k: int = 21, seed: int = 42, s: int = 1000):
    """Mash `sketch` of every record of a packed pool (one reference per record): the
    bottom-s distinct canonical k-mer hashes, sorted.  Used to build sketch DBs (.msh) on
    the device; hashing is the screen kernel in candidates-only mode (ndb = 0)."""
    out = []
    ss = pool.ss
    for i in range(ss.n):
        b = int(ss.starts[i])
        L = int(ss.lengths[i])
        if L < k:
            out.append(np.zeros(0, np.uint64))
            continue
        _, bottom, _ = count_pool(gpu, pool, [], k, seed, s, b, b + L - k + 1)
        out.append(bottom)
    return out

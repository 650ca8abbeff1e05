"""Query ingest for the fused path: FASTA bytes in host memory -> a device-resident shard.

The reference passes the pooled contigs as a FASTA file (run_hymet_cami.sh:64-68 copies
INPUT_FASTA into input/; mash.sh:14 and minimap2.sh:23 read it).  Here:

  * FastaIndex: the record table of the FASTA bytes (hymet_fasta_index, native, threaded):
    name / sequence byte ranges and base counts.  No sequence byte is touched in Python.
  * QueryShard: records [r0, r1) made resident in HBM with ONE host->device copy of their
    contiguous byte range; the device strips line breaks into the 'N'-joined ASCII pool
    (hymet_fasta_compact), packs it for the Mash and minimap2 alphabets (hymet_pack), and
    hashes the names (hymet_name_hash).  The shard also carries the query name pool the
    PAF / TSV writers read, and the mapping batches (contiguous record ranges sized for the
    anchor working set).

Multi-GPU: every rank holds the same FASTA bytes and indexes, uploads and
maps only its own contiguous byte range (`shard_bytes`: the cuts k * len / world moved to the
next record start), so the ranks' query indices are consecutive slices of the input order.
`FastaIndex.shard` (record ranges balanced by bases) serves inputs given as a whole-file
record table.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from ._lib import check, load, ptr
from .seqio import SeqSet

_c = ctypes
_vp = _c.c_void_p


def _np_ptr(a: np.ndarray):
    return a.ctypes.data_as(_vp)


def shard_bytes(data: bytes, rank: int, world: int):
    """Byte range [b0, b1) of this rank's records: the cuts k * len / world moved forward to the
    next record start ('>' at the start of a line), so each rank scans, uploads and maps only
    its own part of the FASTA (no rank reads the whole file).  Records are cut whole; a range
    may be empty when there are fewer records than ranks."""
    n = len(data)

    def cut(k):
        if k <= 0:
            return 0
        if k >= world:
            return n
        c = n * k // world
        if c > 0 and data[c - 1:c] == b"\n" and data[c:c + 1] == b">":
            return c
        j = data.find(b"\n>", c)
        return n if j < 0 else j + 1
    return cut(rank), cut(rank + 1)


class FastaIndex:
    """Record table of FASTA text held in host memory (semantics of seqio.parse_fasta_bytes).
    byte_range: index only the records starting in [b0, b1) (shard_bytes); offsets stay
    absolute into `data`."""

    def __init__(self, data: bytes, threads: Optional[int] = None, byte_range=None):
        self.data = data
        lib = load()
        threads = int(threads or min(16, os.cpu_count() or 1))
        n = _c.c_int64()
        buf = _c.c_char_p(data)
        self._buf = buf
        b0, b1 = byte_range if byte_range is not None else (0, len(data))
        self.byte_range = (int(b0), int(b1))
        base = _c.cast(buf, _vp).value + b0 if len(data) else None
        cap = max(16, (b1 - b0) // 64)
        while True:
            self.name_off = np.zeros(cap, np.int64)
            self.name_len = np.zeros(cap, np.int32)
            self.seq_off = np.zeros(cap, np.int64)
            self.seq_end = np.zeros(cap, np.int64)
            self.nbases = np.zeros(cap, np.int64)
            rc = lib.hymet_fasta_index(_vp(base), b1 - b0, threads, cap, _c.byref(n), _np_ptr(self.name_off),
                                       _np_ptr(self.name_len), _np_ptr(self.seq_off), _np_ptr(self.seq_end),
                                       _np_ptr(self.nbases))
            if rc == -3:
                cap = n.value
                continue
            check(rc, "hymet_fasta_index")
            break
        k = n.value
        self.n = k
        for a in ("name_off", "name_len", "seq_off", "seq_end", "nbases"):
            setattr(self, a, getattr(self, a)[:k])
        if b0:
            for a in ("name_off", "seq_off", "seq_end"):
                getattr(self, a)[:] += b0
        self._names: Optional[List[str]] = None

    @property
    def total_bases(self) -> int:
        return int(self.nbases.sum())

    def names(self) -> List[str]:
        if self._names is None:
            d = self.data
            self._names = [d[o:o + l].decode() for o, l in zip(self.name_off.tolist(), self.name_len.tolist())]
        return self._names

    def name_pool(self, r0: int = 0, r1: Optional[int] = None):
        """(uint8 array, int64 offsets) of the names of records [r0, r1), concatenated
        (hymet_fasta_names, native)."""
        r1 = self.n if r1 is None else r1
        n = r1 - r0
        off = np.zeros(n + 1, np.int64)
        pool = np.zeros(max(int(self.name_len[r0:r1].sum()), 1), np.uint8)
        no = np.ascontiguousarray(self.name_off[r0:r1])
        nl = np.ascontiguousarray(self.name_len[r0:r1])
        check(load().hymet_fasta_names(self._buf, _np_ptr(no), _np_ptr(nl), n, _np_ptr(pool), _np_ptr(off)),
              "hymet_fasta_names")
        return pool[:off[-1]], off

    def byte_shards(self, world: int):
        """Record ranges of the `world` byte shards (shard_bytes) of a whole-file index:
        [(r0, r1)] per rank, from where each cut lands."""
        out, r = [], 0
        for k in range(world):
            _, b1 = shard_bytes(self.data, k, world)
            r1 = int(np.searchsorted(self.name_off, b1, side="right"))  # a record's name starts in (its '>', next '>']
            out.append((r, r1))
            r = r1
        return out

    def shard(self, rank: int, world: int):
        """Contiguous record range [r0, r1) of this rank, balanced by bases (every rank
        computes the same split from the same table)."""
        if world <= 1:
            return 0, self.n
        cum = np.cumsum(self.nbases)
        total = int(cum[-1]) if self.n else 0
        cuts = [0] + [int(np.searchsorted(cum, total * r / world, side="left")) for r in range(1, world)] + [self.n]
        return cuts[rank], cuts[rank + 1]


def to_fasta(names: Sequence[str], seqs: Sequence[bytes], width: int = 0) -> bytes:
    """FASTA text of records (width > 0 wraps sequence lines like most assemblers do)."""
    out = []
    for n, s in zip(names, seqs):
        out.append(b">" + n.encode() + b"\n")
        if width > 0 and len(s) > width:
            out.append(b"\n".join(s[i:i + width] for i in range(0, len(s), width)) + b"\n")
        else:
            out.append(s + b"\n")
    return b"".join(out)


class PackedPool:
    """An ASCII pool packed for one alphabet (the screen / mapper read w2b + wmask)."""

    def __init__(self, gpu, d_ascii, n_bases: int, alphabet: int):
        torch = gpu.torch
        self.n_bases = n_bases
        self.alphabet = alphabet
        self.w2b = gpu.zeros((n_bases + 15) // 16 + 4, torch.int32)
        self.wmask = gpu.zeros((n_bases + 31) // 32 + 4, torch.int32)
        if n_bases:
            gpu.call("hymet_pack", ptr(d_ascii), n_bases, alphabet, ptr(self.w2b), ptr(self.wmask))


def _batches(lengths: np.ndarray, max_bases: int):
    """Greedy batches of consecutive records, each of at most max_bases unless a record alone
    exceeds it: a batch closes before the record that would take it past the limit."""
    n = len(lengths)
    if n == 0:
        return [(0, 0)]
    cs = np.cumsum(np.asarray(lengths, np.int64))
    out, b0, base = [], 0, 0
    while b0 < n:
        i = int(np.searchsorted(cs, base + max_bases, side="right"))  # first record past the limit
        i = max(i, b0 + 1)
        out.append((b0, i))
        base, b0 = int(cs[i - 1]), i
    return out


@dataclass
class QueryShard:
    """Queries resident in HBM (both packed alphabets, names, lengths, mapping batches)."""
    n: int
    q_base: Optional[int]       # index of the first query in the whole input (None: pending, Pipeline.shard_base)
    lengths: np.ndarray         # int64 per query
    starts: np.ndarray          # int64 pool offset per query
    mash: PackedPool
    mm: PackedPool
    qlen: object                # device int64 [n]
    name_hash: object           # device uint32 [n]
    qname: object               # device uint8 name pool
    qname_off: object           # device int64 [n + 1]
    batches: list
    names_host: Optional[List[str]] = None   # SeqSet input: names on the host
    fasta: Optional[FastaIndex] = None       # FASTA input: the record table the shard was cut from
    fasta_r0: int = 0                        # index in `fasta` of the shard's first record
    byte_sharded: bool = False               # a rank's byte range of a multi-rank run (Pipeline.ingest)

    @property
    def total_bases(self) -> int:
        return int(self.lengths.sum())

    @classmethod
    def from_fasta(cls, gpu, fx: FastaIndex, r0: int = 0, r1: Optional[int] = None, batch_bases: int = 40_000_000,
                   d_all=None, q_base: Optional[int] = None, d_base: int = 0):
        """One H2D copy of the records' contiguous byte range, then device-side compaction.
        d_all: the input's bytes from file offset d_base on, already in HBM (uploaded while the
        records were scanned: the whole file, or a rank's byte range).
        q_base: index of record r0 in the whole input (default r0: fx indexes the whole file)."""
        torch = gpu.torch
        r1 = fx.n if r1 is None else r1
        q_base = r0 if q_base is None else q_base
        n = r1 - r0
        nb = fx.nbases[r0:r1]
        pool_len = int(nb.sum()) + max(n - 1, 0)
        if n == 0:
            return cls._empty(gpu, q_base, batch_bases)
        lo = int(min(fx.name_off[r0], fx.seq_off[r0]))
        hi = int(fx.seq_end[r1 - 1])
        if d_all is not None:
            if lo < d_base or hi - d_base > d_all.numel():
                raise ValueError("from_fasta: the records lie outside the uploaded bytes")
            d_raw, lo = d_all, d_base
        else:
            # one upload through the library's double-buffered pinned staging (a pageable copy
            # staged the gigabyte on one thread)
            d_raw = gpu.empty(max(hi - lo, 1), torch.uint8)
            addr = ctypes.cast(fx._buf, ctypes.c_void_p).value + lo  # the record scan's pointer to the bytes
            check(gpu.lib.hymet_copy_to_device(gpu.ctx, ptr(d_raw), ctypes.c_void_p(addr), hi - lo, 16),
                  "hymet_copy_to_device")
        d_pool = gpu.empty(max(pool_len, 1) + 16, torch.uint8)
        d_start = gpu.empty(n, torch.int64)
        so = np.ascontiguousarray(fx.seq_off[r0:r1])
        se = np.ascontiguousarray(fx.seq_end[r0:r1])
        nbc = np.ascontiguousarray(nb)
        gpu.call("hymet_fasta_compact", ptr(d_raw), hi - lo, lo, _np_ptr(so), _np_ptr(se), _np_ptr(nbc), n, ptr(d_pool),
                 pool_len, ptr(d_start))
        lengths = nb.astype(np.int64)
        starts = np.zeros(n, np.int64)
        if n > 1:
            np.cumsum(lengths[:-1] + 1, out=starts[1:])
        # names: offsets into the uploaded range, hashed there; then a compact name pool
        noff = torch.from_numpy(np.ascontiguousarray(fx.name_off[r0:r1] - lo)).to(gpu.dev)
        nlen = torch.from_numpy(np.ascontiguousarray(fx.name_len[r0:r1])).to(gpu.dev)
        d_hash = gpu.empty(n, torch.int32)
        gpu.call("hymet_name_hash", ptr(d_raw), ptr(noff), ptr(nlen), n, ptr(d_hash))
        pool_b, pool_off = fx.name_pool(r0, r1)
        return cls._finish(gpu, n, q_base, lengths, starts, d_pool, pool_len, d_hash, pool_b, pool_off, batch_bases)

    @classmethod
    def from_seqset(cls, gpu, ss: SeqSet, q_base: int = 0, batch_bases: int = 40_000_000):
        """A SeqSet already joined by 'N' (seqio layout): upload its buffer as the pool."""
        torch = gpu.torch
        n = ss.n
        if n == 0:
            return cls._empty(gpu, q_base, batch_bases)
        pool_len = len(ss.buf)
        d_pool = gpu.empty(max(pool_len, 1) + 16, torch.uint8)
        if pool_len:
            d_pool[:pool_len].copy_(torch.frombuffer(bytearray(ss.buf), dtype=torch.uint8))
        names_b = [x.encode() for x in ss.names]
        pool_b = b"".join(names_b)
        pool_off = np.zeros(n + 1, np.int64)
        np.cumsum([len(x) for x in names_b], out=pool_off[1:])
        d_names = torch.frombuffer(bytearray(pool_b or b"\0"), dtype=torch.uint8).to(gpu.dev)
        noff = torch.from_numpy(pool_off[:-1].copy()).to(gpu.dev)
        nlen = torch.from_numpy(np.diff(pool_off).astype(np.int32)).to(gpu.dev)
        d_hash = gpu.empty(n, torch.int32)
        gpu.call("hymet_name_hash", ptr(d_names), ptr(noff), ptr(nlen), n, ptr(d_hash))
        sh = cls._finish(gpu, n, q_base, np.asarray(ss.lengths, np.int64), np.asarray(ss.starts, np.int64), d_pool,
                         pool_len, d_hash, pool_b, pool_off, batch_bases)
        sh.names_host = list(ss.names)
        return sh

    @classmethod
    def _finish(cls, gpu, n, q_base, lengths, starts, d_pool, pool_len, d_hash, pool_b, pool_off, batch_bases):
        torch = gpu.torch
        from .seqio import DevicePool
        mash = PackedPool(gpu, d_pool, pool_len, DevicePool.ALPHA_MASH)
        mm = PackedPool(gpu, d_pool, pool_len, DevicePool.ALPHA_MINIMAP2)
        qlen = torch.from_numpy(lengths).to(gpu.dev)
        pool_np = np.frombuffer(pool_b, np.uint8) if isinstance(pool_b, (bytes, bytearray)) else pool_b
        # np.frombuffer over bytes is read-only: copy before torch.from_numpy (it warns on
        # non-writable arrays); the copy is the name pool only (~10 B per contig)
        qname = torch.from_numpy(np.array(pool_np, np.uint8, copy=True) if len(pool_np) else np.zeros(1, np.uint8)).to(gpu.dev)
        qname_off = torch.from_numpy(pool_off).to(gpu.dev)
        return cls(n, q_base, lengths, starts, mash, mm, qlen, d_hash, qname, qname_off, _batches(lengths, batch_bases))

    @classmethod
    def _empty(cls, gpu, q_base, batch_bases):
        torch = gpu.torch
        z = gpu.zeros(16, torch.uint8)
        from .seqio import DevicePool
        e64 = np.zeros(0, np.int64)
        return cls(0, q_base, e64, e64, PackedPool(gpu, z, 0, DevicePool.ALPHA_MASH),
                   PackedPool(gpu, z, 0, DevicePool.ALPHA_MINIMAP2), gpu.zeros(1, torch.int64), gpu.zeros(1, torch.int32),
                   gpu.zeros(1, torch.uint8), gpu.zeros(1, torch.int64), [])

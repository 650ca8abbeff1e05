"""Align stage: the MI355X replacement for scripts/minimap2.sh.

    minimap2 -I2g -d reference.mmi combined_genomes.fasta      (index, default k=15 w=10)
    minimap2 -x asm10 reference.mmi input/*.fna > resultados.paf

The index is built on the GPU per `-I` part (<= 2e9 bases, split at sequence boundaries
the way minimap2's reader does: mini-batches of >= 50 Mbp until the part passes the
limit) and mapped with asm10 options; the PAF writer here formats the region records the
device returns (format.c mm_write_paf3 / write_tags, no CIGAR).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from ._lib import check, ptr
from .seqio import DevicePool, SeqSet, from_records

_c = ctypes


def parse_num(s: str) -> int:
    """minimap2 mm_parse_num: k/m/g suffixes are powers of 1000."""
    s = str(s).strip()
    mult = {"k": 1e3, "K": 1e3, "m": 1e6, "M": 1e6, "g": 1e9, "G": 1e9}.get(s[-1:], None)
    return int(float(s[:-1]) * mult) if mult else int(float(s))


def split_parts(lengths: np.ndarray, batch_size: float = 2e9, mini_batch: float = 50e6) -> List[np.ndarray]:
    """index.c mm_idx_gen + bseq.c mm_bseq_read: a part keeps reading mini-batches (each
    ends once it has accumulated >= mini_batch bases) while the part's total is <= batch_size."""
    parts, cur, part_len = [], [], 0
    i, n = 0, len(lengths)
    while i < n:
        if part_len > batch_size:
            parts.append(np.array(cur, dtype=np.int64))
            cur, part_len = [], 0
        mb = 0
        while i < n:
            cur.append(i)
            mb += int(lengths[i])
            part_len += int(lengths[i])
            i += 1
            if mb >= mini_batch:
                break
    if cur:
        parts.append(np.array(cur, dtype=np.int64))
    return parts


class IndexPart:
    """One minimizer index part resident in HBM (hymet_mm_index)."""

    def __init__(self, gpu, ss: SeqSet, w: int = 10, k: int = 15, pool: Optional[DevicePool] = None):
        self.gpu, self.w, self.k = gpu, w, k
        self.names = list(ss.names)
        self.lens = np.ascontiguousarray(ss.lengths, dtype=np.int64)
        pool = pool or DevicePool(gpu, ss, DevicePool.ALPHA_MINIMAP2)
        starts = np.ascontiguousarray(ss.starts, dtype=np.int64)
        h = _c.c_void_p()
        gpu.call("hymet_mm_index_build", ptr(pool.w2b), ptr(pool.wmask), starts.ctypes.data_as(_c.c_void_p),
                 self.lens.ctypes.data_as(_c.c_void_p), len(self.names), w, k, _c.byref(h))
        self.h = h
        n_pos = _c.c_int64()
        check(gpu.lib.hymet_mm_index_info(self.h, None, None, None, _c.byref(n_pos)), "hymet_mm_index_info")
        self.n_pos = n_pos.value

    def max_occ(self, frac: float = 2e-4) -> int:
        out = _c.c_int32()
        self.gpu.call("hymet_mm_index_max_occ", self.h, _c.c_float(frac), _c.byref(out))
        return out.value

    def export(self):
        hs = np.zeros(self.n_pos, np.uint32)
        pos = np.zeros(self.n_pos, np.uint64)
        self.gpu.call("hymet_mm_index_export", self.h, hs.ctypes.data_as(_c.c_void_p), pos.ctypes.data_as(_c.c_void_p))
        return hs, pos

    def close(self):
        if getattr(self, "h", None):
            self.gpu.lib.hymet_mm_index_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def sketch(gpu, pool: DevicePool, w: int = 10, k: int = 15, rid_mode: int = 0):
    """Minimizers of every sequence of a packed pool -> (x, y) uint64 arrays, sequence-major."""
    ss = pool.ss
    starts = np.ascontiguousarray(ss.starts, dtype=np.int64)
    lens = np.ascontiguousarray(ss.lengths, dtype=np.int64)
    cap = int(lens.sum() // max(1, w // 2) + 1024)
    while True:
        x = np.zeros(cap, np.uint64)
        y = np.zeros(cap, np.uint64)
        n = _c.c_int64()
        rc = gpu.lib.hymet_mm_sketch(gpu.ctx, ptr(pool.w2b), ptr(pool.wmask), starts.ctypes.data_as(_c.c_void_p),
                                     lens.ctypes.data_as(_c.c_void_p), len(lens), w, k, rid_mode,
                                     x.ctypes.data_as(_c.c_void_p), y.ctypes.data_as(_c.c_void_p), cap, _c.byref(n))
        if rc == -3:
            cap = n.value + 16
            continue
        check(rc, "hymet_mm_sketch")
        return x[:n.value], y[:n.value]

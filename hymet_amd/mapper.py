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


class MapOpt(_c.Structure):
    """hymet_mm_opt == minimap2 mm_mapopt_t after mm_set_opt("asm10") (options.c)."""
    _fields_ = [("mid_occ", _c.c_int32), ("q_occ_frac", _c.c_float), ("max_max_occ", _c.c_int32),
                ("occ_dist", _c.c_int32), ("min_cnt", _c.c_int32), ("min_chain_score", _c.c_int32),
                ("bw", _c.c_int32), ("bw_long", _c.c_int32), ("max_gap", _c.c_int32), ("max_chain_skip", _c.c_int32),
                ("rmq_inner_dist", _c.c_int32), ("rmq_size_cap", _c.c_int32), ("rmq_rescue_size", _c.c_int32),
                ("rmq_rescue_ratio", _c.c_float), ("chain_gap_scale", _c.c_float), ("chain_skip_scale", _c.c_float),
                ("mask_level", _c.c_float), ("pri_ratio", _c.c_float), ("mask_len", _c.c_int32), ("best_n", _c.c_int32),
                ("a", _c.c_int32), ("b", _c.c_int32), ("seed", _c.c_int32)]

    # asm presets clamp mid_occ to [50, 500] (options.c mm_set_opt "asm*")
    min_mid_occ = 50
    max_mid_occ = 500
    mid_occ_frac = 2e-4

    @classmethod
    def asm10(cls) -> "MapOpt":
        o = cls()
        o.mid_occ = 0
        o.q_occ_frac = 0.01
        o.max_max_occ, o.occ_dist = 4095, 500
        o.min_cnt, o.min_chain_score = 3, 40
        o.bw, o.bw_long, o.max_gap, o.max_chain_skip = 1000, 100000, 10000, 25
        o.rmq_inner_dist, o.rmq_size_cap, o.rmq_rescue_size = 1000, 100000, 1000
        o.rmq_rescue_ratio = 0.1
        o.chain_gap_scale, o.chain_skip_scale = 0.8, 0.0
        o.mask_level, o.pri_ratio = 0.5, 0.8
        o.mask_len, o.best_n, o.a, o.b, o.seed = 2 ** 31 - 1, 50, 1, 9, 11
        return o

    def resolve_mid_occ(self, part: "IndexPart") -> int:
        """options.c mm_mapopt_update: set once (from the first index part) when <= 0."""
        if self.mid_occ <= 0:
            m = part.max_occ(self.mid_occ_frac)
            if m < self.min_mid_occ:
                m = self.min_mid_occ
            if self.max_mid_occ > self.min_mid_occ and m > self.max_mid_occ:
                m = self.max_mid_occ
            self.mid_occ = m
        if self.bw_long < self.bw:
            self.bw_long = self.bw
        return self.mid_occ


REG_DTYPE = np.dtype([(n, np.int32) for n in ("qs", "qe", "rs", "re", "rid", "rev", "mlen", "blen", "mapq", "cnt", "score",
                                              "subsc", "parent", "id", "n_sub", "strand_retained")]
                     + [("div", np.float32), ("as_", np.int32), ("hash", np.uint32), ("pad", np.int32)])


def x31_hash(name: str) -> int:
    """khash __ac_X31_hash_string (signed char arithmetic, 32-bit wrap)."""
    b = name.encode()
    if not b:
        return 0
    h = b[0] if b[0] < 128 else b[0] - 256
    h &= 0xFFFFFFFF
    for c in b[1:]:
        c = c if c < 128 else c - 256
        h = ((h << 5) - h + c) & 0xFFFFFFFF
    return h


@dataclass
class MapResult:
    off: np.ndarray        # n_q + 1
    rep_len: np.ndarray    # n_q
    regs: np.ndarray       # REG_DTYPE

    def query(self, q):
        return self.regs[self.off[q]:self.off[q + 1]]


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

    @classmethod
    def load(cls, gpu, path: str, offset: int, names, lens, w: int = 10, k: int = 15):
        """A part persisted by save() (hymet_mm_index_load: no sketch, no sort)."""
        self = cls.__new__(cls)
        self.gpu, self.w, self.k = gpu, w, k
        self.names = list(names)
        self.lens = np.ascontiguousarray(lens, dtype=np.int64)
        h = _c.c_void_p()
        end = _c.c_int64()
        gpu.call("hymet_mm_index_load", str(path).encode(), int(offset), _c.byref(h), _c.byref(end))
        self.h = h
        n_pos, n_seq = _c.c_int64(), _c.c_int32()
        check(gpu.lib.hymet_mm_index_info(self.h, None, None, _c.byref(n_seq), _c.byref(n_pos)), "hymet_mm_index_info")
        if n_seq.value != len(self.names):
            self.close()
            raise ValueError(f"{path}: index part has {n_seq.value} sequences, manifest lists {len(self.names)}")
        self.n_pos = n_pos.value
        self.end_offset = end.value
        return self

    def save(self, path: str, append: bool) -> int:
        """Append (or write) this part to a persisted index file; returns the end offset."""
        end = _c.c_int64()
        self.gpu.call("hymet_mm_index_save", self.h, str(path).encode(), int(append), _c.byref(end))
        return end.value

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


INDEX_FORMAT = "hymet-amd-gpu-index/2"


def save_index(path_mmi: str, parts: List["IndexPart"], names, lens, part_first, ref_fasta: str, split: str):
    """Persist the device index beside reference.mmi (minimap2.sh:10-19 caches the index):
    the binary parts go to PATH.hymet (a distinct name, so a CPU minimap2 .mmi is never
    clobbered) and PATH itself holds the manifest -- non-empty, so the script's `[ -s ]`
    cache test keeps its meaning."""
    import json
    import os
    data = str(path_mmi) + ".hymet"
    offs = [0]
    for i, p in enumerate(parts):
        offs.append(p.save(data, append=i > 0))
    st = os.stat(ref_fasta) if ref_fasta and os.path.exists(ref_fasta) else None
    man = {"format": INDEX_FORMAT, "data": os.path.basename(data), "part_offsets": offs[:-1], "part_first": list(part_first),
           "names": list(names), "lens": [int(x) for x in lens], "w": parts[0].w if parts else 10,
           "k": parts[0].k if parts else 15, "split_idx": split,
           "reference": os.path.abspath(ref_fasta) if ref_fasta else None,
           "reference_size": st.st_size if st else None, "reference_mtime": st.st_mtime if st else None}
    tmp = str(path_mmi) + ".tmp"
    with open(tmp, "w") as f:
        json.dump(man, f)
        f.write("\n")
    os.replace(tmp, path_mmi)


def index_mismatch(man: dict, ref_fasta=None, split=None) -> List[str]:
    """The manifest fields that disagree with the current reference FASTA / -I split.
    minimap2.sh:10 reuses any non-empty index (`[ -s ]`), whatever the FASTA, and so does
    load_index: these are reported as warnings, not acted on."""
    import os
    out = []
    if ref_fasta and os.path.exists(ref_fasta) and man.get("reference_size") is not None:
        st = os.stat(ref_fasta)
        if os.path.abspath(ref_fasta) != man.get("reference"):
            out.append(f"reference path {man.get('reference')} -> {os.path.abspath(ref_fasta)}")
        if st.st_size != man.get("reference_size") or st.st_mtime != man.get("reference_mtime"):
            out.append("reference size/mtime changed since the index was built")
    if split is not None and man.get("split_idx") is not None and str(split) != str(man.get("split_idx")):
        out.append(f"-I {man.get('split_idx')} -> {split}")
    return out


def load_index(gpu, path_mmi: str, ref_fasta=None, split=None, warn=None):
    """(parts, names, lens, part_first) of a persisted index, or None when PATH is not one
    of ours (e.g. a real minimap2 .mmi) or its data file is missing.  The manifest's
    reference path / size / mtime and split are checked against ref_fasta / split when
    given; a mismatch is passed to `warn` (stderr by default) and the index is still used,
    as the script's cache test does."""
    import json
    import os
    import sys
    try:
        with open(path_mmi, "r") as f:
            man = json.loads(f.readline())
    except (OSError, ValueError, UnicodeDecodeError):
        return None
    if not isinstance(man, dict) or man.get("format") != INDEX_FORMAT:
        return None
    data = os.path.join(os.path.dirname(os.path.abspath(path_mmi)), man["data"])
    if not os.path.exists(data):
        return None
    for m in index_mismatch(man, ref_fasta, split):
        (warn or (lambda t: print(t, file=sys.stderr)))(f"warning: cached index {path_mmi}: {m} (reused, as minimap2.sh does)")
    names, lens, first = man["names"], np.asarray(man["lens"], np.int64), man["part_first"]
    parts = []
    for i, off in enumerate(man["part_offsets"]):
        b = first[i]
        e = first[i + 1] if i + 1 < len(first) else len(names)
        parts.append(IndexPart.load(gpu, data, off, names[b:e], lens[b:e], man["w"], man["k"]))
    return parts, names, lens, first


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


def map_part(gpu, part: "IndexPart", qpool: DevicePool, opt: MapOpt, name_hash: Optional[np.ndarray] = None) -> MapResult:
    """Map every query of a packed pool against one index part (minimap2 -x asm10)."""
    ss = qpool.ss
    nq = ss.n
    starts = np.ascontiguousarray(ss.starts, dtype=np.int64)
    lens = np.ascontiguousarray(ss.lengths, dtype=np.int64)
    if name_hash is None:
        name_hash = np.array([x31_hash(n) for n in ss.names], dtype=np.uint32)
    name_hash = np.ascontiguousarray(name_hash, dtype=np.uint32)
    h = _c.c_void_p()
    gpu.call("hymet_mm_map", part.h, _c.byref(opt), ptr(qpool.w2b), ptr(qpool.wmask), starts.ctypes.data_as(_c.c_void_p),
             lens.ctypes.data_as(_c.c_void_p), name_hash.ctypes.data_as(_c.c_void_p), nq, _c.byref(h))
    try:
        n = _c.c_int64()
        check(gpu.lib.hymet_mm_result_size(h, _c.byref(n)), "hymet_mm_result_size")
        off = np.zeros(nq + 1, np.int64)
        rl = np.zeros(max(nq, 1), np.int32)
        regs = np.zeros(n.value, REG_DTYPE)
        check(gpu.lib.hymet_mm_result_copy(h, off.ctypes.data_as(_c.c_void_p), rl.ctypes.data_as(_c.c_void_p),
                                           regs.ctypes.data_as(_c.c_void_p)), "hymet_mm_result_copy")
    finally:
        gpu.lib.hymet_mm_result_destroy(h)
    return MapResult(off, rl[:nq], regs)


def paf_lines(qname: str, qlen: int, regs, rep_len: int, tnames, tlens) -> List[str]:
    """format.c mm_write_paf3 + write_tags without CIGAR (no `cg`/`NM` tags)."""
    out = []
    for r in regs:
        prim = r["id"] == r["parent"]
        fields = [qname, str(qlen), str(r["qs"]), str(r["qe"]), "+-"[r["rev"]], tnames[r["rid"]], str(tlens[r["rid"]]),
                  str(r["rs"]), str(r["re"]), str(r["mlen"]), str(r["blen"]), str(r["mapq"]),
                  "tp:A:" + ("P" if prim else "S"), f"cm:i:{r['cnt']}", f"s1:i:{r['score']}"]
        if prim:
            fields.append(f"s2:i:{r['subsc']}")
        d = float(r["div"])
        if 0.0 <= d <= 1.0:
            fields.append("dv:f:" + ("0" if d == 0.0 else "%.4f" % d))
        fields.append(f"rl:i:{rep_len}")
        out.append("\t".join(fields))
    return out

"""TEST INFRASTRUCTURE ONLY -- ctypes bindings for oracle/build/liboracle.so (the CPU
restatements of Mash screen and minimap2).  Imported by tests/, smoke() and bench.py's
cpu_baseline leg only."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_murmur3_x64_128_h0.restype = ctypes.c_uint64
        L.oracle_murmur3_x64_128_h0.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_uint32]
        L.oracle_murmur3_x86_32.restype = ctypes.c_uint32
        L.oracle_murmur3_x86_32.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_uint32]
        L.oracle_screen.restype = ctypes.c_int
        L.oracle_sketch.restype = ctypes.c_int64
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def murmur3_h0(s: bytes, seed: int) -> int:
    return lib().oracle_murmur3_x64_128_h0(s, len(s), seed)


def murmur3_x86_32(s: bytes, seed: int) -> int:
    return lib().oracle_murmur3_x86_32(s, len(s), seed)


def concat(seqs):
    """list of bytes -> (buffer, offsets int64)"""
    off = np.zeros(len(seqs) + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(s) for s in seqs])
    return b"".join(seqs), off


def screen(seqs, k, seed, sketch_size, ref_hashes_list, preserve_case=False):
    buf, off = concat(seqs)
    ref_off = np.zeros(len(ref_hashes_list) + 1, dtype=np.int64)
    ref_off[1:] = np.cumsum([len(h) for h in ref_hashes_list])
    rh = np.ascontiguousarray(np.concatenate(ref_hashes_list) if ref_hashes_list else np.zeros(0), dtype=np.uint64)
    n = len(ref_hashes_list)
    shared = np.zeros(n, dtype=np.uint32)
    median = np.zeros(n, dtype=np.uint32)
    ss = ctypes.c_uint64()
    nk = ctypes.c_uint64()
    rc = lib().oracle_screen(ctypes.c_char_p(buf), _p(off), ctypes.c_int64(len(seqs)), ctypes.c_int(k), ctypes.c_uint32(seed),
                             ctypes.c_int(int(preserve_case)), ctypes.c_int64(sketch_size), _p(rh), _p(ref_off), ctypes.c_int64(n),
                             _p(shared), _p(median), ctypes.byref(ss), ctypes.byref(nk))
    if rc != 0:
        raise ValueError("oracle_screen: unsupported parameters")
    return shared, median, ss.value, nk.value


def sketch(seqs, k, seed, s):
    buf, off = concat(seqs)
    out = np.zeros(s, dtype=np.uint64)
    m = lib().oracle_sketch(ctypes.c_char_p(buf), _p(off), ctypes.c_int64(len(seqs)), ctypes.c_int(k), ctypes.c_uint32(seed),
                            ctypes.c_int64(s), _p(out))
    return out[:m]


# ------------------------------------------------------------------ minimap2 oracle
class MmOpt(ctypes.Structure):
    _fields_ = [(n, t) for n, t in [
        ("mid_occ", ctypes.c_int32), ("mid_occ_frac", ctypes.c_float), ("min_mid_occ", ctypes.c_int32),
        ("max_mid_occ", ctypes.c_int32), ("q_occ_frac", ctypes.c_float), ("max_max_occ", ctypes.c_int32),
        ("occ_dist", ctypes.c_int32), ("min_cnt", ctypes.c_int32), ("min_chain_score", ctypes.c_int32),
        ("bw", ctypes.c_int32), ("bw_long", ctypes.c_int32), ("max_gap", ctypes.c_int32), ("max_chain_skip", ctypes.c_int32),
        ("rmq_inner_dist", ctypes.c_int32), ("rmq_size_cap", ctypes.c_int32), ("rmq_rescue_size", ctypes.c_int32),
        ("rmq_rescue_ratio", ctypes.c_float), ("chain_gap_scale", ctypes.c_float), ("chain_skip_scale", ctypes.c_float),
        ("mask_level", ctypes.c_float), ("pri_ratio", ctypes.c_float), ("alt_drop", ctypes.c_float),
        ("mask_len", ctypes.c_int32), ("best_n", ctypes.c_int32), ("a", ctypes.c_int32), ("b", ctypes.c_int32),
        ("seed", ctypes.c_int32)]]


REG_DTYPE = np.dtype([(n, np.int32) for n in ("qs", "qe", "rs", "re", "rid", "rev", "mlen", "blen", "mapq", "cnt", "score",
                                              "subsc", "parent", "id", "n_sub", "strand_retained")]
                     + [("div", np.float32), ("as_", np.int32), ("hash", np.uint32), ("pad", np.int32)])


def _mm_lib():
    L = lib()
    if not hasattr(L, "_mm_ready"):
        L.mmo_idx_build.restype = ctypes.c_void_p
        L.mmo_idx_build.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.mmo_idx_destroy.argtypes = [ctypes.c_void_p]
        L.mmo_idx_n_keys.restype = ctypes.c_int64
        L.mmo_idx_n_keys.argtypes = [ctypes.c_void_p]
        L.mmo_idx_n_pos.restype = ctypes.c_int64
        L.mmo_idx_n_pos.argtypes = [ctypes.c_void_p]
        L.mmo_idx_export.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.mmo_idx_cal_max_occ.restype = ctypes.c_int32
        L.mmo_idx_cal_max_occ.argtypes = [ctypes.c_void_p, ctypes.c_float]
        L.mmo_opt_asm10.argtypes = [ctypes.POINTER(MmOpt)]
        L.mmo_opt_update_mid_occ.restype = ctypes.c_int32
        L.mmo_opt_update_mid_occ.argtypes = [ctypes.POINTER(MmOpt), ctypes.c_void_p]
        L.mmo_map.restype = ctypes.c_int
        L.mmo_map.argtypes = [ctypes.c_void_p, ctypes.POINTER(MmOpt), ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p,
                              ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.mmo_sketch_seq.restype = ctypes.c_int64
        L.mmo_sketch_seq.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int64]
        L.mmo_debug_anchors.restype = ctypes.c_int64
        L.mmo_debug_anchors.argtypes = [ctypes.c_void_p, ctypes.POINTER(MmOpt), ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p,
                                        ctypes.c_int64, ctypes.POINTER(ctypes.c_int)]
        L.mmo_debug_chain.restype = ctypes.c_int64
        L.mmo_debug_chain.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p]
        L._mm_ready = True
    return L


def mm_sketch(seq: bytes, w=10, k=15, rid=0):
    L = _mm_lib()
    cap = len(seq) + 16
    out = np.zeros((cap, 2), dtype=np.uint64)
    n = L.mmo_sketch_seq(seq, len(seq), w, k, rid, _p(out), cap)
    assert n >= 0
    return out[:n]


def asm10_opt():
    o = MmOpt()
    _mm_lib().mmo_opt_asm10(ctypes.byref(o))
    return o


class MmIndex:
    """One minimap2 index part (k=15, w=10 by default) over the given sequences."""

    def __init__(self, seqs, w=10, k=15, names=None):
        L = _mm_lib()
        buf, off = concat(seqs)
        lens = np.array([len(s) for s in seqs], dtype=np.int64)
        self.names = names or [f"ref{i}" for i in range(len(seqs))]
        self.lens = lens
        self.w, self.k = w, k
        self.h = L.mmo_idx_build(ctypes.c_char_p(buf), _p(off), _p(lens), len(seqs), w, k)

    def export(self):
        L = _mm_lib()
        nk, npos = L.mmo_idx_n_keys(self.h), L.mmo_idx_n_pos(self.h)
        keys = np.zeros(nk, np.uint64)
        koff = np.zeros(nk + 1, np.int64)
        pos = np.zeros(npos, np.uint64)
        L.mmo_idx_export(self.h, _p(keys), _p(koff), _p(pos))
        return keys, koff, pos

    def max_occ(self, f=2e-4):
        return _mm_lib().mmo_idx_cal_max_occ(self.h, f)

    def __del__(self):
        try:
            _mm_lib().mmo_idx_destroy(self.h)
        except Exception:
            pass


def mm_map(idx: MmIndex, opt: MmOpt, qseq: bytes, qname: str):
    L = _mm_lib()
    cap = 256
    while True:
        out = np.zeros(cap, dtype=REG_DTYPE)
        rl = ctypes.c_int()
        n = L.mmo_map(idx.h, ctypes.byref(opt), qseq, len(qseq), qname.encode(), _p(out), cap, ctypes.byref(rl))
        if n >= 0:
            return out[:n], rl.value
        cap = -n + 16


def mm_debug_anchors(idx: MmIndex, opt: MmOpt, qseq: bytes):
    L = _mm_lib()
    cap = max(1024, len(qseq) * 4)
    while True:
        out = np.zeros((cap, 2), dtype=np.uint64)
        rl = ctypes.c_int()
        n = L.mmo_debug_anchors(idx.h, ctypes.byref(opt), qseq, len(qseq), _p(out), cap, ctypes.byref(rl))
        if n >= 0:
            return out[:n], rl.value
        cap = -n + 16


def mm_debug_chain(a: np.ndarray, max_dist, max_dist_inner, bw, max_skip, cap_rmq, pen_gap, pen_skip):
    L = _mm_lib()
    n = len(a)
    f = np.zeros(n + 1, np.int32)
    p = np.zeros(n + 1, np.int64)
    a = np.ascontiguousarray(a, dtype=np.uint64)
    L.mmo_debug_chain(_p(a), n, max_dist, max_dist_inner, bw, max_skip, cap_rmq, pen_gap, pen_skip, _p(f), _p(p))
    return f[:n], p[:n]


def format_paf(qname, qlen, regs, rep_len, tnames, tlens):
    """format.c mm_write_paf3 + write_tags (no CIGAR): one PAF line per region."""
    out = []
    for r in regs:
        typ = "P" if r["id"] == r["parent"] else "S"
        line = (f"{qname}\t{qlen}\t{r['qs']}\t{r['qe']}\t{'+-'[r['rev']]}\t{tnames[r['rid']]}\t{tlens[r['rid']]}\t"
                f"{r['rs']}\t{r['re']}\t{r['mlen']}\t{r['blen']}\t{r['mapq']}\ttp:A:{typ}\tcm:i:{r['cnt']}\ts1:i:{r['score']}")
        if r["parent"] == r["id"]:
            line += f"\ts2:i:{r['subsc']}"
        d = float(r["div"])
        if 0.0 <= d <= 1.0:
            line += "\tdv:f:" + ("0" if d == 0.0 else "%.4f" % d)
        line += f"\trl:i:{rep_len}"
        out.append(line)
    return out


class ScreenOracle:
    """oracle_screen_prepare / _run: the hash table built once for repeated runs."""

    def __init__(self, db):
        L = lib()
        L.oracle_screen_prepare.restype = ctypes.c_void_p
        L.oracle_screen_prepare.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
        L.oracle_screen_free.argtypes = [ctypes.c_void_p]
        L.oracle_screen_run.restype = ctypes.c_int
        L.oracle_screen_run.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                        ctypes.c_uint32, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p]
        self.db = db
        self.h_hashes = np.ascontiguousarray(db.hashes, dtype=np.uint64)
        self.h_off = np.ascontiguousarray(db.offsets, dtype=np.int64)
        self.h = L.oracle_screen_prepare(_p(self.h_hashes), _p(self.h_off), db.n_refs)

    def run(self, seqs):
        buf, off = concat(seqs)
        n = self.db.n_refs
        sh = np.zeros(n, np.uint32)
        md = np.zeros(n, np.uint32)
        ss, nk = ctypes.c_uint64(), ctypes.c_uint64()
        rc = lib().oracle_screen_run(self.h, ctypes.c_char_p(buf), _p(off), len(seqs), self.db.k, self.db.seed, 0,
                                     self.db.sketch_size, _p(sh), _p(md), ctypes.byref(ss), ctypes.byref(nk))
        assert rc == 0
        return sh, md, ss.value, nk.value

    def __del__(self):
        try:
            lib().oracle_screen_free(self.h)
        except Exception:
            pass


def mm_index_from_arrays(hashes_sorted: np.ndarray, pos: np.ndarray, lens, names, w=10, k=15):
    """Build the oracle's index structure from sorted (hash, pos) arrays."""
    L = _mm_lib()
    L.mmo_idx_from_arrays.restype = ctypes.c_void_p
    L.mmo_idx_from_arrays.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_int]
    h = np.asarray(hashes_sorted)
    starts = np.flatnonzero(np.r_[True, h[1:] != h[:-1]]) if len(h) else np.zeros(0, np.int64)
    keys = np.ascontiguousarray(h[starts].astype(np.uint64))
    koff = np.ascontiguousarray(np.r_[starts, len(h)].astype(np.int64))
    pos = np.ascontiguousarray(pos, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.int64)
    idx = MmIndex.__new__(MmIndex)
    idx.names, idx.lens, idx.w, idx.k = list(names), lens, w, k
    idx.h = L.mmo_idx_from_arrays(_p(keys), _p(koff), len(keys), _p(pos), _p(lens), len(lens), w, k)
    return idx

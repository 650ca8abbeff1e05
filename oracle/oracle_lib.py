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
        L.oracle_screen.restype = ctypes.c_int
        L.oracle_sketch.restype = ctypes.c_int64
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def murmur3_h0(s: bytes, seed: int) -> int:
    return lib().oracle_murmur3_x64_128_h0(s, len(s), seed)


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

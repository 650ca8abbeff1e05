"""Mash sketch databases (`data/sketch{1,2,3}.msh`, read by scripts/mash.sh:14).

A .msh file is a Cap'n Proto message (unpacked framing) with Mash's `MinHash` schema.
Mash is third-party and unpinned (environment.yml:9) and no .msh file ships with the
reference, so the schema below is restated from the public Mash 2.x source and is
PARITY-UNPINNED:

    struct MinHash {
      kmerSize @0 :UInt32;  windowSize @1 :UInt32;  minHashesPerWindow @2 :UInt32;
      concatenated @3 :Bool;  error @4 :Float32;  noncanonical @5 :Bool;
      referenceListOld @6 :ReferenceList;  referenceList @7 :ReferenceList;
      locusList @8 :LocusList;  alphabet @9 :Text;  preserveCase @10 :Bool;
      hashSeed @11 :UInt32 = 42;
      struct ReferenceList { references @0 :List(Reference);
        struct Reference { sequence @0 :Text; quality @1 :Text; length @2 :UInt32;
          name @3 :Text; comment @4 :Text; hashes32 @5 :List(UInt32);
          hashes64 @6 :List(UInt64); length64 @7 :UInt64; counts32 @8 :List(UInt32);
          counts32Sorted @9 :Bool; } } }

The ordinals of `referenceList` and `locusList` (@7 / @8) are the one detail this
restatement cannot settle from memory alone; the product reader (csrc/msh.cpp, through
`read_msh`) therefore takes whichever of pointers 1 and 2 holds Reference structs (Locus
structs carry no pointers) and falls back to `referenceListOld` (pointer 0), as Mash does
for old files.  Hand-assembled byte fixtures (tests/golden/msh/, written field by field by
tests/golden/make_msh_fixtures.py, independent of write_msh) pin the reader on both
layouts, multi-segment messages with far and double-far pointers, 32-bit sketches and
unsorted hash lists.

Resulting layouts (Cap'n Proto field-slot allocation): MinHash data = 3 words
{kmerSize@0B, windowSize@4B, minHashesPerWindow@8B, concatenated bit96, noncanonical bit97,
preserveCase bit98, error@16B, hashSeed@20B (xor 42)}, 4 pointers {refListOld, refList,
locusList, alphabet}; Reference data = 2 words {length@0B, counts32Sorted bit32,
length64@8B}, 7 pointers {sequence, quality, name, comment, hashes32, hashes64, counts32}.

Besides .msh, `load_db` accepts the repo's own `.npz` sketch format (same fields).
"""
from __future__ import annotations

import struct
from collections.abc import Sequence
from dataclasses import dataclass, field
from typing import List

import numpy as np


class NulStrings(Sequence):
    """The NUL-separated strings of a byte buffer as a read-only sequence, decoded on access:
    the DB's names and comments are needed only for the references a screen line is printed
    for (a few thousand of 10^5), so read_msh does not build 2 x 10^5 Python strings per run."""

    def __init__(self, buf, n: int, starts=None):
        """buf: bytes or a uint8 array; starts: the n + 1 string starts if known (the native
        reader gives them), else found by a NUL scan."""
        self._buf = buf if isinstance(buf, (bytes, bytearray)) else memoryview(np.ascontiguousarray(buf, np.uint8))
        if starts is not None:
            self._start = np.asarray(starts[:n], np.int64)
            self._end = np.asarray(starts[1:n + 1], np.int64) - 1
            return
        ends = np.flatnonzero(np.frombuffer(buf, np.uint8) == 0)[:n] if n else np.zeros(0, np.int64)
        self._end = ends
        self._start = np.r_[0, ends[:-1] + 1] if n else ends

    def __len__(self):
        return len(self._end)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        if i < 0:
            i += len(self)
        return bytes(self._buf[int(self._start[i]):int(self._end[i])]).decode("utf-8", "replace")

    def __eq__(self, other):
        return list(self) == list(other)

    def __repr__(self):
        return f"NulStrings({len(self)})"


@dataclass
class SketchDB:
    k: int = 21
    seed: int = 42
    sketch_size: int = 1000          # minHashesPerWindow
    alphabet: str = "ACGT"
    preserve_case: bool = False
    noncanonical: bool = False
    window_size: int = 0
    names: List[str] = field(default_factory=list)
    comments: List[str] = field(default_factory=list)
    lengths: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int64))
    offsets: np.ndarray = field(default_factory=lambda: np.zeros(1, np.int64))   # CSR into hashes
    hashes: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint64))   # each ref sorted

    @property
    def n_refs(self):
        return len(self.names)

    def ref_hashes(self, i):
        a, b = int(self.offsets[i]), int(self.offsets[i + 1])
        sl = getattr(self, "dev_slice", None)
        if sl is not None and b > a and (a < sl[0] or b > sl[1]):
            # read_msh(shard=...): the host array holds this rank's slice only; the whole DB
            # exists only in HBM after the ranks' all-gather
            raise RuntimeError(f"SketchDB.ref_hashes({i}): hashes [{a}, {b}) lie outside this rank's "
                               f"host slice [{sl[0]}, {sl[1]})")
        return self.hashes[a:b]


# ------------------------------------------------------------------ capnp reader
class _Msg:
    def __init__(self, data: bytes):
        n = struct.unpack_from("<I", data, 0)[0] + 1
        sizes = struct.unpack_from(f"<{n}I", data, 4)
        off = 4 + 4 * n
        off += (8 - off % 8) % 8
        self.segs = []
        for s in sizes:
            self.segs.append(memoryview(data)[off:off + 8 * s])
            off += 8 * s

    def word(self, seg, w):
        return struct.unpack_from("<Q", self.segs[seg], 8 * w)[0]

    def resolve(self, seg, w):
        """Follow a pointer at (seg, word w). Returns (kind, seg, target_word, ptr_value)."""
        p = self.word(seg, w)
        if p == 0:
            return None
        kind = p & 3
        if kind == 2:  # far
            double = (p >> 2) & 1
            land = (p >> 3) & ((1 << 29) - 1)
            tseg = p >> 32
            if not double:
                return self.resolve(tseg, land)
            pad0 = self.word(tseg, land)
            pad1 = self.word(tseg, land + 1)
            seg2 = pad0 >> 32
            start = (pad0 >> 3) & ((1 << 29) - 1)
            return (pad1 & 3, seg2, start, pad1)
        off = (p >> 2) & ((1 << 30) - 1)
        if off & (1 << 29):
            off -= 1 << 30
        return (kind, seg, w + 1 + off, p)

    def struct_at(self, seg, w):
        r = self.resolve(seg, w)
        if r is None:
            return None
        kind, s, t, p = r
        assert kind == 0, "expected struct pointer"
        return _Struct(self, s, t, (p >> 32) & 0xFFFF, p >> 48)

    def list_at(self, seg, w):
        r = self.resolve(seg, w)
        if r is None:
            return None
        kind, s, t, p = r
        assert kind == 1, "expected list pointer"
        return (s, t, (p >> 32) & 7, p >> 35)


class _Struct:
    def __init__(self, msg, seg, w, dwords, nptrs):
        self.m, self.seg, self.w, self.dw, self.np = msg, seg, w, dwords, nptrs

    def u32(self, byte_off, default=0):
        if byte_off + 4 > 8 * self.dw:
            return default
        return struct.unpack_from("<I", self.m.segs[self.seg], 8 * self.w + byte_off)[0] ^ default

    def u64(self, byte_off):
        if byte_off + 8 > 8 * self.dw:
            return 0
        return struct.unpack_from("<Q", self.m.segs[self.seg], 8 * self.w + byte_off)[0]

    def f32(self, byte_off):
        if byte_off + 4 > 8 * self.dw:
            return 0.0
        return struct.unpack_from("<f", self.m.segs[self.seg], 8 * self.w + byte_off)[0]

    def bit(self, bit):
        if bit >= 64 * self.dw:
            return False
        b = self.m.segs[self.seg][8 * self.w + bit // 8]
        return bool((b >> (bit % 8)) & 1)

    def ptr_word(self, i):
        return self.w + self.dw + i

    def text(self, i):
        if i >= self.np:
            return ""
        l = self.m.list_at(self.seg, self.ptr_word(i))
        if l is None:
            return ""
        s, t, es, n = l
        raw = bytes(self.m.segs[s][8 * t:8 * t + n])
        return raw[:-1].decode("utf-8", "replace") if raw.endswith(b"\0") else raw.decode("utf-8", "replace")

    def prim_list(self, i, dtype):
        if i >= self.np:
            return np.zeros(0, dtype)
        l = self.m.list_at(self.seg, self.ptr_word(i))
        if l is None:
            return np.zeros(0, dtype)
        s, t, es, n = l
        item = np.dtype(dtype).itemsize
        return np.frombuffer(self.m.segs[s], dtype=dtype, count=n, offset=8 * t).copy()

    def struct_list(self, i):
        if i >= self.np:
            return []
        l = self.m.list_at(self.seg, self.ptr_word(i))
        if l is None:
            return []
        s, t, es, n = l
        assert es == 7, "expected composite list"
        tag = self.m.word(s, t)
        cnt = (tag >> 2) & ((1 << 30) - 1)
        dw, npt = (tag >> 32) & 0xFFFF, tag >> 48
        step = dw + npt
        return [_Struct(self.m, s, t + 1 + j * step, dw, npt) for j in range(cnt)]


class _PendingStrings(Sequence):
    """A DB's names / comments before read_msh(defer_meta=True)'s finish_meta() ran: the
    right length, no contents."""

    def __init__(self, n: int):
        self._n = n

    def __len__(self):
        return self._n

    def __getitem__(self, i):
        raise RuntimeError("sketch DB names read before SketchDB.finish_meta()")


def read_msh(path, threads: int = 16, alloc=None, upload=None, shard=None, defer_meta: bool = False) -> SketchDB:
    """.msh -> SketchDB through the library's native reader (hymet_msh_*: mmap, pointer walk
    and a threaded hash gather; S1 of SURVEY.md §8a, on the timed path since `mash screen`
    reads its DB on every call).  alloc(n) may supply the uint64 array the hashes are
    gathered into (e.g. a view of pinned memory, so the table upload is one DMA).
    upload = (gpu, dev_alloc): alloc must then give pinned memory, and the hashes are gathered
    in chunks whose DMAs into dev_alloc(n) (a device int64 tensor) are queued on gpu's stream
    as each chunk is gathered (hymet_msh_upload); the tensor is returned as db.dev_hashes.
    shard = (rank, world), with upload: only this rank's slice of c = ceil(n_hashes / world)
    hashes, [rank * c, (rank + 1) * c), is gathered and uploaded (hymet_msh_upload_range) into
    a device tensor of world * c entries, for Comm.allgather_slices_ to fill in the others;
    db.dev_slice = (lo, hi, c), and db.hashes holds valid hashes only on [lo, hi) (ref_hashes
    raises for a reference outside it).
    defer_meta (with upload): the file stays open and the names / comments are copied only by
    db.finish_meta() -- the caller runs it while the GPU builds the table; until then they
    are placeholders of the right length.
    The library is required, like every product path."""
    import ctypes
    import time
    from ._lib import check, load
    if shard is not None and upload is None:
        raise ValueError("read_msh: shard needs upload (the slices meet in HBM)")
    if defer_meta and upload is None:
        raise ValueError("read_msh: defer_meta needs upload")
    lib = load()
    h = ctypes.c_void_p()
    t0 = time.perf_counter()
    check(lib.hymet_msh_open(str(path).encode(), ctypes.byref(h)), "hymet_msh_open")
    t1 = t2 = time.perf_counter()
    keep_open = False
    try:
        raw = (ctypes.c_int64 * 9)()   # hymet_msh_info: 7 int32 (+4 pad) then 5 int64
        check(lib.hymet_msh_info_get(h, ctypes.byref(raw)), "hymet_msh_info_get")
        b = bytes(raw)
        k, win, ss, seed, nonc, pc, use64 = struct.unpack_from("<iiiIiii", b, 0)
        n_refs, n_hashes, nb, cb, al = struct.unpack_from("<qqqqq", b, 32)
        hashes = alloc(max(n_hashes, 1)) if alloc is not None else np.empty(max(n_hashes, 1), np.uint64)
        offsets = np.empty(n_refs + 1, np.int64)
        lengths = np.empty(max(n_refs, 1), np.int64)
        # uninitialised pools (the reader writes every byte; create_string_buffer zeroes ~10 MB)
        names_a = np.empty(max(nb, 1), np.uint8)
        comments_a = np.empty(max(cb, 1), np.uint8)
        names, comments = (ctypes.c_void_p(a.ctypes.data) for a in (names_a, comments_a))
        alpha = ctypes.create_string_buffer(max(al, 1))
        name_st = np.empty(n_refs + 1, np.int64)
        comment_st = np.empty(n_refs + 1, np.int64)
        check(lib.hymet_msh_text_offsets(h, name_st.ctypes.data_as(ctypes.c_void_p),
                                         comment_st.ctypes.data_as(ctypes.c_void_p)), "hymet_msh_text_offsets")
        dev = None
        if upload is not None:
            # the hashes first: their DMAs run while the metadata is copied below
            g, dev_alloc = upload
            if shard is None:
                lo, hi, c, size = 0, n_hashes, n_hashes, n_hashes
            else:
                r, w = shard
                c = -(-n_hashes // w)
                lo = min(n_hashes, r * c)
                hi, size = min(n_hashes, lo + c), w * c
            dev = dev_alloc(max(size, 1))
            check(lib.hymet_msh_upload_range(g.ctx, h, int(threads), hashes.ctypes.data_as(ctypes.c_void_p),
                                             ctypes.c_void_p(dev.data_ptr()), 8, lo, hi), "hymet_msh_upload_range")
            t2 = time.perf_counter()
            check(lib.hymet_msh_copy(h, int(threads), None, offsets.ctypes.data_as(ctypes.c_void_p),
                                     lengths.ctypes.data_as(ctypes.c_void_p), None if defer_meta else names,
                                     None if defer_meta else comments, alpha), "hymet_msh_copy")
        else:
            check(lib.hymet_msh_copy(h, int(threads), hashes.ctypes.data_as(ctypes.c_void_p),
                                     offsets.ctypes.data_as(ctypes.c_void_p), lengths.ctypes.data_as(ctypes.c_void_p),
                                     names, comments, alpha), "hymet_msh_copy")
        keep_open = defer_meta
    finally:
        if not keep_open:
            lib.hymet_msh_close(h)
    t3 = time.perf_counter()

    def split(buf, n, st):
        return NulStrings(buf, n, st) if n else []

    db = SketchDB(k=k, seed=seed, sketch_size=ss, alphabet=alpha.raw[:al].decode() or "ACGT", preserve_case=bool(pc),
                  noncanonical=bool(nonc), window_size=win,
                  names=_PendingStrings(n_refs) if defer_meta else split(names_a, n_refs, name_st),
                  comments=_PendingStrings(n_refs) if defer_meta else split(comments_a, n_refs, comment_st),
                  lengths=lengths[:n_refs].copy(), offsets=offsets, hashes=hashes[:n_hashes])
    db.dev_hashes = dev
    db.dev_slice = (lo, hi, c) if shard is not None else None
    # with upload: "hashes" = the gather + DMA issue, "meta" = the metadata copy after it;
    # without: one copy of both ("hashes")
    if upload is not None:
        db.load_s = {"open": t1 - t0, "hashes": t2 - t1, "meta": t3 - t2, "wrap": time.perf_counter() - t3}
    else:
        db.load_s = {"open": t1 - t0, "hashes": t3 - t1, "meta": 0.0, "wrap": time.perf_counter() - t3}
    db.finish_meta = None
    if defer_meta:
        def finish_meta():
            tm = time.perf_counter()
            try:
                check(lib.hymet_msh_copy(h, int(threads), None, None, None, names, comments, None), "hymet_msh_copy")
            finally:
                lib.hymet_msh_close(h)
                db.finish_meta = None
            db.names = split(names_a, n_refs, name_st)
            db.comments = split(comments_a, n_refs, comment_st)
            db.load_s["meta"] += time.perf_counter() - tm
        db.finish_meta = finish_meta
    return db


def read_msh_py(path) -> SketchDB:
    """Pure-Python reader of the same format (tests cross-check it against the native one)."""
    data = open(path, "rb").read()
    m = _Msg(data)
    root = m.struct_at(0, 0)
    db = SketchDB()
    db.k = root.u32(0)
    db.window_size = root.u32(4)
    db.sketch_size = root.u32(8)
    db.noncanonical = root.bit(97)
    db.preserve_case = root.bit(98)
    db.seed = root.u32(20, default=42)
    db.alphabet = root.text(3) or "ACGT"
    refs = []
    for pi in (1, 2, 0):   # referenceList (@7 or @8: the list of Reference structs), else referenceListOld
        if pi >= root.np:
            continue
        rl = m.struct_at(root.seg, root.ptr_word(pi))
        lst = rl.struct_list(0) if rl is not None and rl.np > 0 else []
        if lst and lst[0].np > 0:
            refs = lst
            break
    names, comments, lengths, hl = [], [], [], []
    use64 = db.k > 16
    for r in refs:
        names.append(r.text(2))
        comments.append(r.text(3))
        L64 = r.u64(8)
        lengths.append(L64 if L64 else r.u32(0))
        h = r.prim_list(5, np.uint64) if use64 else r.prim_list(4, np.uint32).astype(np.uint64)
        hl.append(np.sort(h))
    db.names, db.comments = names, comments
    db.lengths = np.array(lengths, dtype=np.int64)
    db.offsets = np.zeros(len(hl) + 1, dtype=np.int64)
    if hl:
        db.offsets[1:] = np.cumsum([len(h) for h in hl])
        db.hashes = np.concatenate(hl).astype(np.uint64)
    return db


# ------------------------------------------------------------------ capnp writer
class _Builder:
    """Single-segment Cap'n Proto message builder (enough for the MinHash schema)."""

    def __init__(self):
        self.buf = bytearray()

    def alloc(self, words):
        w = len(self.buf) // 8
        self.buf += b"\0" * (8 * words)
        return w

    def set_ptr(self, at_word, target_word, kind, hi):
        off = target_word - (at_word + 1)
        v = (kind & 3) | ((off & ((1 << 30) - 1)) << 2) | (hi << 32)
        struct.pack_into("<Q", self.buf, 8 * at_word, v)

    def struct_ptr(self, at, target, dw, np_):
        self.set_ptr(at, target, 0, dw | (np_ << 16))

    def text(self, at, s: str):
        b = s.encode() + b"\0"
        w = self.alloc((len(b) + 7) // 8)
        self.buf[8 * w:8 * w + len(b)] = b
        self.set_ptr(at, w, 1, 2 | (len(b) << 3))

    def prim_list(self, at, arr: np.ndarray, es: int):
        b = arr.tobytes()
        w = self.alloc((len(b) + 7) // 8)
        self.buf[8 * w:8 * w + len(b)] = b
        self.set_ptr(at, w, 1, es | (len(arr) << 3))

    def message(self):
        n = len(self.buf) // 8
        return struct.pack("<II", 0, n) + bytes(self.buf)


def write_msh(db: SketchDB, path):
    b = _Builder()
    root_ptr = b.alloc(1)
    root = b.alloc(3 + 4)
    b.struct_ptr(root_ptr, root, 3, 4)
    struct.pack_into("<III", b.buf, 8 * root, db.k, db.window_size, db.sketch_size)
    flags = (int(db.noncanonical) << 1) | (int(db.preserve_case) << 2)
    b.buf[8 * root + 12] = flags
    struct.pack_into("<f", b.buf, 8 * root + 16, 0.0)
    struct.pack_into("<I", b.buf, 8 * root + 20, db.seed ^ 42)
    rl = b.alloc(1)
    b.struct_ptr(root + 3 + 1, rl, 0, 1)
    n = db.n_refs
    DW, NP = 2, 7
    tag = b.alloc(1 + n * (DW + NP))
    b.set_ptr(rl, tag, 1, 7 | ((n * (DW + NP)) << 3))
    struct.pack_into("<Q", b.buf, 8 * tag, (n << 2) | (DW << 32) | (NP << 48))
    for i in range(n):
        e = tag + 1 + i * (DW + NP)
        L = int(db.lengths[i]) if len(db.lengths) > i else 0
        struct.pack_into("<I", b.buf, 8 * e, L & 0xFFFFFFFF)
        struct.pack_into("<Q", b.buf, 8 * e + 8, L)
        p = e + DW
        b.text(p + 2, db.names[i])
        b.text(p + 3, db.comments[i] if i < len(db.comments) else "")
        b.prim_list(p + 5, np.ascontiguousarray(db.ref_hashes(i), dtype=np.uint64), 5)
    b.text(root + 3 + 3, db.alphabet)
    with open(path, "wb") as f:
        f.write(b.message())


def save_npz(db: SketchDB, path):
    np.savez(path, k=db.k, seed=db.seed, sketch_size=db.sketch_size, alphabet=db.alphabet,
             preserve_case=db.preserve_case, noncanonical=db.noncanonical,
             names=np.array(db.names, dtype=object).astype(str), comments=np.array(db.comments, dtype=object).astype(str),
             lengths=db.lengths, offsets=db.offsets, hashes=db.hashes)


def load_db(path) -> SketchDB:
    p = str(path)
    if p.endswith(".npz"):
        z = np.load(p, allow_pickle=False)
        return SketchDB(k=int(z["k"]), seed=int(z["seed"]), sketch_size=int(z["sketch_size"]), alphabet=str(z["alphabet"]),
                        preserve_case=bool(z["preserve_case"]), noncanonical=bool(z["noncanonical"]),
                        names=[str(x) for x in z["names"]], comments=[str(x) for x in z["comments"]],
                        lengths=z["lengths"].astype(np.int64), offsets=z["offsets"].astype(np.int64),
                        hashes=z["hashes"].astype(np.uint64))
    return read_msh(p)

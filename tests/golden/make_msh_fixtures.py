#!/usr/bin/env python3
"""Hand-assembled Mash sketch files (.msh) for the S1 reader.

No .msh file ships with the reference and Mash is not in the image, so these fixtures are
assembled here word by word from the Cap'n Proto encoding rules and Mash's MinHash schema
(both public; restated in hymet_amd/msh.py's docstring) -- deliberately NOT with
hymet_amd.msh.write_msh, so the product reader is pinned by bytes it did not write.  Each
fixture exercises layout choices a real Cap'n Proto writer may make:

  v2_single.msh    one segment, the current reference list in pointer 1 (referenceList @7),
                   k21 64-bit hashes, three references with length64, seed 42 (stored as 0)
  v2_far32.msh     three segments: the reference list in pointer 2 (the other ordinal
                   order, locusList in pointer 1 holding one Locus), reached by a single-far
                   pointer; one hash list behind a double-far pointer; k16 32-bit hashes (one
                   list unsorted), seed 7 (stored 7 ^ 42), preserveCase, 32-bit length only
  old_list.msh     only referenceListOld (pointer 0) set, k25, older struct sizes (the
                   Reference struct without its second data word and last pointer)

expect.json holds the values a correct reader returns (hash lists ascending).
"""
from __future__ import annotations

import json
import struct
from pathlib import Path

OUT = Path(__file__).resolve().parent / "msh"


class Seg:
    def __init__(self):
        self.w = []

    def alloc(self, n):
        i = len(self.w)
        self.w += [0] * n
        return i


def sptr(at, target, dw, np_):
    off = (target - (at + 1)) & ((1 << 30) - 1)
    return (off << 2) | (dw << 32) | (np_ << 48)


def lptr(at, target, es, count):
    off = (target - (at + 1)) & ((1 << 30) - 1)
    return 1 | (off << 2) | (es << 32) | (count << 35)


def far(seg, land, double=False):
    return 2 | (int(double) << 2) | (land << 3) | (seg << 32)


def put_bytes(seg: Seg, data: bytes):
    """data padded to words; returns the first word index"""
    n = (len(data) + 7) // 8
    i = seg.alloc(n)
    pad = data + b"\0" * (8 * n - len(data))
    for k in range(n):
        seg.w[i + k] = struct.unpack_from("<Q", pad, 8 * k)[0]
    return i


def text(seg: Seg, at: int, s: str):
    b = s.encode() + b"\0"
    i = put_bytes(seg, b)
    seg.w[at] = lptr(at, i, 2, len(b))


def u64list(seg: Seg, at: int, vals):
    i = put_bytes(seg, struct.pack(f"<{len(vals)}Q", *vals))
    seg.w[at] = lptr(at, i, 5, len(vals))


def u32list(seg: Seg, at: int, vals):
    i = put_bytes(seg, struct.pack(f"<{len(vals)}I", *vals))
    seg.w[at] = lptr(at, i, 4, len(vals))


def message(segs):
    head = struct.pack("<I", len(segs) - 1) + b"".join(struct.pack("<I", len(s.w)) for s in segs)
    head += b"\0" * ((8 - len(head) % 8) % 8)
    return head + b"".join(struct.pack(f"<{len(s.w)}Q", *s.w) for s in segs)


def root_struct(seg: Seg, k, win, s, flags_bits, seed):
    """MinHash root: data 3 words {kmerSize@0 windowSize@4 minHashesPerWindow@8, bools at
    bits 96.. (concatenated, noncanonical, preserveCase), error f32 @16, hashSeed ^ 42 @20},
    4 pointers {referenceListOld, referenceList/locusList, locusList/referenceList, alphabet}"""
    seg.alloc(1)  # root pointer at word 0
    r = seg.alloc(3 + 4)
    seg.w[0] = sptr(0, r, 3, 4)
    seg.w[r] = k | (win << 32)
    seg.w[r + 1] = s | (flags_bits << 32)
    seg.w[r + 2] = struct.unpack("<I", struct.pack("<f", 0.0))[0] | ((seed ^ 42) << 32)
    return r


def references(seg: Seg, at: int, refs, dw=2, np_=7, use64=True, hash_at=None):
    """ReferenceList struct (0 data words, 1 pointer) -> composite List(Reference).
    hash_at(i, word) may place a reference's hash list elsewhere (returns True if it did)."""
    rl = seg.alloc(1)
    seg.w[at] = sptr(at, rl, 0, 1)
    tag = seg.alloc(1 + len(refs) * (dw + np_))
    seg.w[rl] = lptr(rl, tag, 7, len(refs) * (dw + np_))
    seg.w[tag] = (len(refs) << 2) | (dw << 32) | (np_ << 48)
    for i, ref in enumerate(refs):
        e = tag + 1 + i * (dw + np_)
        L = ref["length"]
        seg.w[e] = L & 0xFFFFFFFF if L < 2 ** 32 else 0  # length @0 (UInt32)
        if dw >= 2:
            seg.w[e + 1] = ref.get("length64", 0)           # length64 @8
        p = e + dw
        text(seg, p + 2, ref["name"])                       # name
        text(seg, p + 3, ref["comment"])                    # comment
        if hash_at and hash_at(i, p + (5 if use64 else 4)):
            continue
        if use64:
            u64list(seg, p + 5, ref["hashes"])              # hashes64
        else:
            u32list(seg, p + 4, ref["hashes"])              # hashes32


def v2_single():
    s0 = Seg()
    r = root_struct(s0, 21, 0, 4, 0, 42)
    refs = [
        {"name": "GCF_000005845.2_ASM584v2_genomic.fna.gz", "comment": "[1 seqs] NC_000913.3 Escherichia coli [...]",
         "length": 4641652, "length64": 4641652, "hashes": [3, 1 << 40, 2 ** 63 + 5, 2 ** 64 - 2]},
        {"name": "b.fna", "comment": "", "length": 0, "length64": 6_000_000_000, "hashes": [7, 8, 9, 10]},
        {"name": "c.fna", "comment": "three words here", "length": 1000, "length64": 1000, "hashes": [11]},
    ]
    references(s0, r + 3 + 1, refs)
    text(s0, r + 3 + 3, "ACGT")
    exp = {"k": 21, "seed": 42, "sketch_size": 4, "preserve_case": False, "noncanonical": False, "alphabet": "ACGT",
           "names": [x["name"] for x in refs], "comments": [x["comment"] for x in refs],
           "lengths": [4641652, 6_000_000_000, 1000], "hashes": [sorted(x["hashes"]) for x in refs]}
    return message([s0]), exp


def v2_far32():
    s0, s1, s2 = Seg(), Seg(), Seg()
    r = root_struct(s0, 16, 0, 5, 0b100, 7)  # preserveCase (bit 98)
    # pointer 1: a LocusList {loci: List(Locus)} with one Locus (3 data words, no pointers)
    ll = s0.alloc(1)
    s0.w[r + 3 + 1] = sptr(r + 3 + 1, ll, 0, 1)
    lt = s0.alloc(1 + 3)
    s0.w[ll] = lptr(ll, lt, 7, 3)
    s0.w[lt] = (1 << 2) | (3 << 32)
    s0.w[lt + 1] = 1 | (2 << 32)
    # pointer 2: referenceList, in segment 1 behind a single-far pointer (landing pad there)
    land = s1.alloc(1)
    s0.w[r + 3 + 2] = far(1, land)
    text(s0, r + 3 + 3, "ACGT")
    refs = [
        {"name": "ref32_a", "comment": "first", "length": 123456, "hashes": [0xFFFFFFFE, 5, 0x80000000, 17, 2]},
        {"name": "ref32_b", "comment": "far away", "length": 99, "hashes": [1, 2, 3]},
    ]

    def hash_at(i, word):
        if i != 1:
            return False
        # ref 1's hashes32 behind a double-far pointer: landing pad (far to the content +
        # list tag) in segment 2, content in segment 0
        content = put_bytes(s0, struct.pack("<3I", *refs[1]["hashes"]))
        pad = s2.alloc(2)
        s2.w[pad] = far(0, content)
        s2.w[pad + 1] = 1 | (4 << 32) | (3 << 35)  # list tag: 4-byte elements, 3 of them, offset 0
        s1.w[word] = far(2, pad, double=True)
        return True

    references(s1, land, refs, use64=False, hash_at=hash_at)
    exp = {"k": 16, "seed": 7, "sketch_size": 5, "preserve_case": True, "noncanonical": False, "alphabet": "ACGT",
           "names": ["ref32_a", "ref32_b"], "comments": ["first", "far away"], "lengths": [123456, 99],
           "hashes": [sorted(refs[0]["hashes"]), [1, 2, 3]]}
    return message([s0, s1, s2]), exp


def old_list():
    s0 = Seg()
    r = root_struct(s0, 25, 0, 3, 0b10, 42)  # noncanonical (bit 97)
    refs = [{"name": "old.fa", "comment": "old format", "length": 5000, "hashes": [9, 4, 6]}]
    references(s0, r + 3 + 0, refs, dw=1, np_=6)
    text(s0, r + 3 + 3, "ACGT")
    exp = {"k": 25, "seed": 42, "sketch_size": 3, "preserve_case": False, "noncanonical": True, "alphabet": "ACGT",
           "names": ["old.fa"], "comments": ["old format"], "lengths": [5000], "hashes": [[4, 6, 9]]}
    return message([s0]), exp


def bad_far_loop():
    """Malformed: the reference list's single-far pointer lands on a far pointer to itself
    (a cycle a recursive decoder would follow until the stack overflows)."""
    s0, s1 = Seg(), Seg()
    r = root_struct(s0, 21, 0, 4, 0, 42)
    land = s1.alloc(1)
    s0.w[r + 3 + 1] = far(1, land)
    s1.w[land] = far(1, land)
    text(s0, r + 3 + 3, "ACGT")
    return message([s0, s1])


def bad_far_to_far():
    """Malformed: a single-far landing pad that is a double-far pointer."""
    s0, s1 = Seg(), Seg()
    r = root_struct(s0, 21, 0, 4, 0, 42)
    land = s1.alloc(1)
    s0.w[r + 3 + 1] = far(1, land)
    s1.w[land] = far(0, 1, double=True)
    text(s0, r + 3 + 3, "ACGT")
    return message([s0, s1])


def main():
    OUT.mkdir(parents=True, exist_ok=True)
    for name, fn in (("bad_far_loop.msh", bad_far_loop), ("bad_far_to_far.msh", bad_far_to_far)):
        (OUT / name).write_bytes(fn())
    expect = {}
    for name, fn in (("v2_single.msh", v2_single), ("v2_far32.msh", v2_far32), ("old_list.msh", old_list)):
        data, exp = fn()
        (OUT / name).write_bytes(data)
        expect[name] = exp
    (OUT / "expect.json").write_text(json.dumps(expect, indent=1) + "\n")
    print("wrote", ", ".join(expect))


if __name__ == "__main__":
    main()

"""FASTA input and the packed on-device sequence pool.

A *pool* is every sequence of a set of FASTA files concatenated with one 'N' separator
between records, so that no k-mer or minimizer window can span two records (the invalid
separator resets every rolling state).  On the device it is held packed: 2-bit codes
(16 bases / uint32) + an invalid-base bitmask (32 bases / uint32) -- 0.375 B per base.
The reference reads FASTA through Mash's and minimap2's kseq readers: a record name is the
first whitespace-delimited token after '>', the rest of the header line is the comment.
"""
from __future__ import annotations

import gzip
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

SEP = b"N"


@dataclass
class SeqSet:
    names: List[str]
    comments: List[str]
    lengths: np.ndarray          # int64 per record
    starts: np.ndarray           # int64 offset of each record inside `buf`
    buf: bytes                   # records joined by SEP
    files: List[str] = field(default_factory=list)
    file_of: Optional[np.ndarray] = None   # record -> file index

    @property
    def n(self) -> int:
        return len(self.names)

    @property
    def total_bases(self) -> int:
        return int(self.lengths.sum())

    def seq(self, i: int) -> bytes:
        s = int(self.starts[i])
        return self.buf[s:s + int(self.lengths[i])]

    def subset(self, idx: Sequence[int]) -> "SeqSet":
        return from_records([(self.names[i], self.comments[i], self.seq(i)) for i in idx])


def _open(path):
    with open(path, "rb") as f:
        magic = f.read(2)
    return gzip.open(path, "rb") if magic == b"\x1f\x8b" else open(path, "rb")


def parse_fasta_bytes(data: bytes):
    out = []
    if not data:
        return out
    if data.startswith(b">"):
        chunks = data[1:].split(b"\n>")
    else:  # tolerate leading junk before the first record (kseq skips to '>')
        i = data.find(b"\n>")
        if i < 0:
            return out
        chunks = data[i + 2:].split(b"\n>")
    for ch in chunks:
        nl = ch.find(b"\n")
        head = ch if nl < 0 else ch[:nl]
        body = b"" if nl < 0 else ch[nl + 1:]
        head = head.rstrip(b"\r")
        parts = head.split(None, 1)
        name = parts[0].decode() if parts else ""
        comment = parts[1].decode() if len(parts) > 1 else ""
        seq = body.replace(b"\n", b"").replace(b"\r", b"")
        out.append((name, comment, seq))
    return out


def from_records(records, files=None, file_of=None) -> SeqSet:
    names = [r[0] for r in records]
    comments = [r[1] for r in records]
    seqs = [r[2] for r in records]
    lengths = np.array([len(s) for s in seqs], dtype=np.int64)
    starts = np.zeros(len(seqs), dtype=np.int64)
    if len(seqs):
        starts[1:] = np.cumsum(lengths[:-1] + len(SEP))
    return SeqSet(names, comments, lengths, starts, SEP.join(seqs), list(files or []),
                  None if file_of is None else np.asarray(file_of, dtype=np.int64))


def read_fasta(paths) -> SeqSet:
    if isinstance(paths, (str, bytes)) or hasattr(paths, "__fspath__"):
        paths = [paths]
    recs, file_of = [], []
    for fi, p in enumerate(paths):
        with _open(p) as f:
            r = parse_fasta_bytes(f.read())
        recs.extend(r)
        file_of.extend([fi] * len(r))
    return from_records(recs, [str(p) for p in paths], file_of)


class DevicePool:
    """A SeqSet resident in HBM, packed for one alphabet (hymet_pack)."""

    ALPHA_MASH, ALPHA_MASH_PRESERVE_CASE, ALPHA_MINIMAP2 = 0, 1, 2

    def __init__(self, gpu, ss: SeqSet, alphabet: int):
        from ._lib import ptr

        torch = gpu.torch
        self.gpu = gpu
        self.ss = ss
        self.alphabet = alphabet
        self.n_bases = len(ss.buf)
        n = self.n_bases
        raw = torch.frombuffer(bytearray(ss.buf) if n else bytearray(b"N"), dtype=torch.uint8)
        d_ascii = raw.to(gpu.dev)
        self.w2b = gpu.zeros((n + 15) // 16 + 4, torch.int32)
        self.wmask = gpu.zeros((n + 31) // 32 + 4, torch.int32)
        if n:
            gpu.call("hymet_pack", ptr(d_ascii), n, alphabet, ptr(self.w2b), ptr(self.wmask))
        del d_ascii
        self.starts = torch.from_numpy(ss.starts).to(gpu.dev)
        self.lengths = torch.from_numpy(ss.lengths).to(gpu.dev)

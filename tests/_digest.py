"""Per-contig digests of a run's outputs, for full-size parity at the CAMI configurations
(tests/golden/make_cami_golden.py writes them from the CPU oracle; the -m gpu tests compute
the same from the GPU run and compare every contig).

* PAF: for every contig (input order), the number of its resultados.paf lines and an
  8-byte BLAKE2b of those lines joined by '\\n' in file order (part-major, as minimap2 -I
  writes them).  ref_abundance counts every line of the run
  (scripts/classification_cami.py:181-208), so a line wrong anywhere shows up here.
* TSV: the SHA-256 of the whole classified_sequences.tsv and an 8-byte BLAKE2b of every
  contig's row (0 for a contig without a row).
* Screen: the shared / median arrays of every DB (all references, decoys included)."""
import hashlib
import json
import os

import numpy as np


def _h8(b: bytes) -> int:
    return int.from_bytes(hashlib.blake2b(b, digest_size=8).digest(), "little")


def name_index(names):
    return {n.encode() if isinstance(n, str) else n: i for i, n in enumerate(names)}


def paf_digests(paf: bytes, index):
    """(line count, digest) per contig of the PAF text; index: name bytes -> contig index."""
    n = len(index)
    per = [[] for _ in range(n)]
    for line in paf.split(b"\n"):
        if line:
            per[index[line[:line.index(b"\t")]]].append(line)
    cnt = np.array([len(x) for x in per], np.uint32)
    dig = np.array([_h8(b"\n".join(x)) if x else 0 for x in per], np.uint64)
    return cnt, dig


def tsv_digests(tsv: bytes, index):
    """(sha256 hex of the file, per-contig row digest, rows in file order as contig indices)."""
    dig = np.zeros(len(index), np.uint64)
    order = []
    for row in tsv.split(b"\r\n")[1:]:
        if row:
            i = index[row[:row.index(b"\t")]]
            dig[i] = _h8(row)
            order.append(i)
    return hashlib.sha256(tsv).hexdigest(), dig, np.array(order, np.int32)


def sha(b) -> str:
    if isinstance(b, np.ndarray):
        b = np.ascontiguousarray(b).tobytes()
    return hashlib.sha256(b).hexdigest()


def save(path, meta, arrays):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    np.savez_compressed(path + ".npz", **arrays)
    with open(path + ".json", "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


def load(path):
    with open(path + ".json") as f:
        meta = json.load(f)
    z = np.load(path + ".npz")
    return meta, {k: z[k] for k in z.files}


def diff_report(name, got, want, limit=8):
    bad = np.flatnonzero(got != want)
    return f"{name}: {len(bad)} of {len(want)} differ, first {bad[:limit].tolist()}"

#!/usr/bin/env python3
"""Known-answer vectors for MurmurHash3_x64_128 (word 0), the hash Mash uses for k>16, and
MurmurHash3_x86_32, the hash it uses for k<=16 (32-bit sketches, hashes32).

The independent implementation is scikit-learn's vendored MurmurHash3.cpp (Austin
Appleby's public-domain code), compiled here with g++ into a temporary directory -- it is
never copied into this repository.  Writes tests/golden/murmur3_kat.json:
  * random ASCII ACGT strings, k = 17..32, seeds {42, 0, 7, 2^32-1}
  * canonical 21-mers (seed 42) from the first 20 kbp of three Zymo genomes present in
    /root/reference/case/truth/zymo_refs/genomes (E. coli, B. subtilis, S. aureus)
  * x86_32: random ACGT strings k = 1..16, the same seeds, and canonical 16-mers (seed 42)
    from the same genome prefixes
"""
import ctypes
import gzip
import json
import os
import random
import subprocess
import tempfile
from pathlib import Path

SK = Path("/usr/local/lib/python3.10/dist-packages/sklearn/utils/src")
REF = Path("/root/reference/case/truth/zymo_refs/genomes")
OUT = Path(__file__).resolve().parent / "murmur3_kat.json"


def build():
    td = tempfile.mkdtemp()
    so = os.path.join(td, "libmm3.so")
    subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-I", str(SK), str(SK / "MurmurHash3.cpp"), "-o", so])
    lib = ctypes.CDLL(so)
    lib.MurmurHash3_x64_128.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p]
    lib.MurmurHash3_x86_32.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p]
    return lib


def h32(lib, s: bytes, seed: int) -> int:
    out = ctypes.c_uint32()
    lib.MurmurHash3_x86_32(s, len(s), seed, ctypes.byref(out))
    return out.value


def h0(lib, s: bytes, seed: int) -> int:
    out = (ctypes.c_uint64 * 2)()
    lib.MurmurHash3_x64_128(s, len(s), seed, out)
    return out[0]


def canon(kmer: str) -> str:
    comp = {"A": "T", "C": "G", "G": "C", "T": "A"}
    rc = "".join(comp[c] for c in reversed(kmer))
    return rc if rc < kmer else kmer


def main():
    lib = build()
    rng = random.Random(1234)
    vecs = []
    for k in range(1, 33):
        for seed in (42, 0, 7, 0xFFFFFFFF):
            for _ in range(4):
                s = "".join(rng.choice("ACGT") for _ in range(k))
                vecs.append({"s": s, "seed": seed, "h0": f"{h0(lib, s.encode(), seed):016x}"})
    genomes = {
        "escherichia_coli/GCF_000005845.2_ASM584v2_genomic.fna.gz": 20000,
        "bacillus_subtilis/GCF_000009045.1_ASM904v1_genomic.fna.gz": 20000,
        "staphylococcus_aureus/GCF_000013425.1_ASM1342v1_genomic.fna.gz": 20000,
    }
    zymo, zymo16 = [], []
    x86 = []
    for k in range(1, 17):
        for seed in (42, 0, 7, 0xFFFFFFFF):
            for _ in range(4):
                s = "".join(rng.choice("ACGT") for _ in range(k))
                x86.append({"s": s, "seed": seed, "h32": f"{h32(lib, s.encode(), seed):08x}"})
    for rel, n in genomes.items():
        seq = []
        with gzip.open(REF / rel, "rt") as f:
            for line in f:
                if line.startswith(">"):
                    if seq:
                        break
                    continue
                seq.append(line.strip().upper())
                if sum(map(len, seq)) >= n:
                    break
        s = "".join(seq)[:n]
        for j in range(0, len(s) - 21 + 1, 97):
            km = s[j:j + 21]
            if set(km) <= set("ACGT"):
                c = canon(km)
                zymo.append({"s": c, "seed": 42, "h0": f"{h0(lib, c.encode(), 42):016x}"})
        for j in range(0, len(s) - 16 + 1, 89):
            km = s[j:j + 16]
            if set(km) <= set("ACGT"):
                c = canon(km)
                zymo16.append({"s": c, "seed": 42, "h32": f"{h32(lib, c.encode(), 42):08x}"})
    OUT.write_text(json.dumps({"source": "sklearn/utils/src/MurmurHash3.cpp (compiled with g++)", "random": vecs,
                               "zymo_canonical_k21_seed42": zymo, "x86_32_random": x86,
                               "x86_32_zymo_canonical_k16_seed42": zymo16}, indent=0))
    print(len(vecs), len(zymo), h0(lib, b"AAAAAAAAAAAAAAAAAAAAC", 42).to_bytes(8, "big").hex())


if __name__ == "__main__":
    main()

"""Seeded synthetic inputs shared by CPU and GPU tests (never reads /root/reference)."""
import numpy as np

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def rand_seq(rng, n, gc=0.5):
    p = [(1 - gc) / 2, gc / 2, gc / 2, (1 - gc) / 2]
    return ACGT[rng.choice(4, size=n, p=p)].tobytes()


def mutate(rng, seq: bytes, rate: float) -> bytes:
    """Substitution model of testdataset/mutationGCF.py:4-18 (uniform position, new base != old)."""
    a = np.frombuffer(seq, dtype=np.uint8).copy()
    n = len(a)
    k = int(round(rate * n))
    if k == 0:
        return seq
    pos = rng.choice(n, size=k, replace=False)
    for p in pos:
        old = a[p]
        choices = [c for c in b"ACGT" if c != old]
        a[p] = choices[rng.integers(len(choices))]
    return a.tobytes()


def revcomp(s: bytes) -> bytes:
    return s[::-1].translate(bytes.maketrans(b"ACGTacgtNn", b"TGCAtgcaNn"))


def add_noise(rng, seq: bytes, n_runs=3, lower_frac=0.05):
    """Sprinkle N runs, IUPAC codes and lower-case stretches (edge cases for every parser)."""
    a = bytearray(seq)
    L = len(a)
    for _ in range(n_runs):
        if L < 10:
            break
        p = int(rng.integers(0, L - 5))
        ln = int(rng.integers(1, 40))
        a[p:p + ln] = b"N" * len(a[p:p + ln])
    for _ in range(3):
        if L:
            a[int(rng.integers(0, L))] = ord(rng.choice(list("RYKMSWBDHV")))
    if L > 100:
        p = int(rng.integers(0, L - 50))
        ln = int(L * lower_frac)
        a[p:p + ln] = bytes(a[p:p + ln]).lower()
    return bytes(a)

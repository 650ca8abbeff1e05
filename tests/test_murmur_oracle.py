"""Pin the oracle's MurmurHash3_x64_128 (k > 16) and x86_32 (k <= 16) against known-answer vectors produced by an
independent implementation (scikit-learn's vendored MurmurHash3.cpp; tests/golden/make_murmur_kat.py)."""
import json
from pathlib import Path

from oracle import oracle_lib

KAT = json.loads((Path(__file__).resolve().parent / "golden" / "murmur3_kat.json").read_text())


def test_murmur_random_vectors():
    for v in KAT["random"]:
        assert oracle_lib.murmur3_h0(v["s"].encode(), v["seed"]) == int(v["h0"], 16), v


def test_murmur_zymo_canonical_kmers():
    for v in KAT["zymo_canonical_k21_seed42"]:
        assert oracle_lib.murmur3_h0(v["s"].encode(), 42) == int(v["h0"], 16)


def test_survey_probe_vector():
    assert oracle_lib.murmur3_h0(b"AAAAAAAAAAAAAAAAAAAAC", 42) == 0x21B7D30F1988618F


def test_murmur_x86_32_vectors():
    for v in KAT["x86_32_random"]:
        assert oracle_lib.murmur3_x86_32(v["s"].encode(), v["seed"]) == int(v["h32"], 16), v
    for v in KAT["x86_32_zymo_canonical_k16_seed42"]:
        assert oracle_lib.murmur3_x86_32(v["s"].encode(), 42) == int(v["h32"], 16)

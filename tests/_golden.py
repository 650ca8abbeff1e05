"""Helpers shared by the golden-fixture tests."""
import hashlib
import json
import os
from pathlib import Path

GOLDEN = Path(__file__).resolve().parent / "golden"
CLS = GOLDEN / "classify"


def classify_cases():
    return json.loads((CLS / "cases.json").read_text())


def big_paf(tmpdir) -> Path:
    """Regenerate the 250k-line stress PAF (zymo x100, renamed queries) exactly as
    tests/golden/make_goldens.py:synth_pafs does."""
    p = Path(tmpdir) / "big_zymo_x100.paf"
    if not p.exists():
        zl = [l.rstrip("\n").split("\t") for l in open(CLS / "zymo.paf")]
        big = []
        for k in range(100):
            for q in zl:
                big.append("\t".join([f"{q[0]}_{k}"] + q[1:]))
        p.write_text("\n".join(big) + "\n")
    return p


def case_paf(case, tmpdir) -> Path:
    if case["paf"] == "big_zymo_x100.paf":
        return big_paf(tmpdir)
    return CLS / case["paf"]


def check_bytes(case, got: bytes):
    if "sha256" in case:
        assert len(got) == case["nbytes"]
        assert hashlib.sha256(got).hexdigest() == case["sha256"]
    else:
        exp = (CLS / case["expect"]).read_bytes()
        assert got == exp

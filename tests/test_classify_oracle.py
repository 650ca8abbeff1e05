"""Pin the classify oracle against the reference classifiers' own outputs
(tests/golden/classify, produced by tests/golden/make_goldens.py)."""
import pytest

from oracle import classify_oracle as co
from tests._golden import CLS, case_paf, check_bytes, classify_cases

CASES = classify_cases()


@pytest.mark.parametrize("case", CASES, ids=[f"{c['variant']}-{c['paf']}-{c['taxonomy']}-{c['hierarchy']}" for c in CASES])
def test_oracle_matches_reference(case, tmp_path_factory):
    paf = case_paf(case, tmp_path_factory.getbasetemp())
    fn = co.classify_cami if case["variant"] == "cami" else co.classify_legacy
    if "error" in case:
        with pytest.raises(Exception) as ei:
            fn(paf, CLS / case["taxonomy"], CLS / case["hierarchy"])
        assert type(ei.value).__name__ == case["error"]
        return
    got = fn(paf, CLS / case["taxonomy"], CLS / case["hierarchy"])
    check_bytes(case, got)


def test_zymo_domain_all_species_level():
    # SURVEY.md §8c probe: domain labels -> 1043/1043 species-level with classification_cami
    got = co.classify_cami(CLS / "zymo.paf", CLS / "zymo_taxonomy.tsv", CLS / "zymo_hierarchy_domain.tsv").decode()
    rows = got.strip("\r\n").split("\r\n")[1:]
    assert len(rows) == 1043
    assert all(r.split("\t")[2] == "species" for r in rows)

"""GPU classifier vs the reference classifiers' own outputs (tests/golden/classify, produced
by running scripts/classification_cami.py and scripts/classification.py): byte-identical TSVs."""
import pytest

from tests._golden import CLS, case_paf, check_bytes, classify_cases

pytestmark = pytest.mark.gpu
CASES = classify_cases()


@pytest.fixture(scope="module")
def gpu():
    from hymet_amd._lib import Gpu
    return Gpu(0)


@pytest.mark.parametrize("case", CASES, ids=[f"{c['variant']}-{c['paf']}-{c['taxonomy']}-{c['hierarchy']}" for c in CASES])
def test_gpu_classifier_matches_reference(gpu, case, tmp_path_factory, tmp_path):
    from hymet_amd import classify
    paf = case_paf(case, tmp_path_factory.getbasetemp())
    variant = classify.CAMI if case["variant"] == "cami" else classify.LEGACY
    out = tmp_path / "out.tsv"
    if "error" in case:
        with pytest.raises(Exception) as ei:
            classify.classify_file(gpu, paf, CLS / case["taxonomy"], CLS / case["hierarchy"], out, variant)
        assert type(ei.value).__name__ == case["error"]
        return
    classify.classify_file(gpu, paf, CLS / case["taxonomy"], CLS / case["hierarchy"], out, variant)
    check_bytes(case, out.read_bytes())

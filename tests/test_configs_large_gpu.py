"""BASELINE.json configs[3] and [4] at full size on one MI355X,
checked against the CPU oracle on a bounded random sample of the same run.

The workloads are bench.py's own (bench.build_cami): C4 CAMI-medium = 12 taxa, 744
candidates / 3.06 Gbp in two -I2g parts, 151k contigs / 1 Gbp, a 1e8-hash sketch DB;
C5 CAMI-high = 14 taxa, the full CAND_MAX of 5,000 candidates / ~20 Gbp in ten parts,
~300k contigs / 2 Gbp, three sketch DBs of 1e8 / 5e7 / 1e7 hashes
(run_hymet_cami.sh:26,83-99).  The whole input runs through the fused GPU path once; then
bench.cpu_baseline_cami maps a random sample of the contigs with the minimap2 restatement
against the same index parts, screens them, and classifies them with the run's global
ref_abundance (classification_cami.py:181-208): every sampled contig's PAF lines and TSV row
must equal the GPU's.  The sample is bounded by time (the CPU restatement is ~300 contigs/s
on 16 threads for C4), not by count."""
import gc
import os

import pytest

pytestmark = pytest.mark.gpu
THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def gpu():
    from hymet_amd._lib import Gpu
    return Gpu(0)


def _run(gpu, workload, budget_s, min_sample):
    import bench
    from hymet_amd.dist import Comm
    args = bench.parse_args(["--workload", workload, "--cpu-threads", str(THREADS), "--cpu-budget", str(budget_s)])
    comm = Comm()
    w, db, pipe, fasta, refs_ss, tax, hier, td = bench.build_cami(args, comm, gpu)
    try:
        res = pipe.run(fasta, with_paf=True)
        assert res.n_queries == len(w.contigs) and res.n_classified >= 0.99 * res.n_queries
        chk = bench.cpu_baseline_cami(args, pipe, res, fasta, db, tax, hier)
        print(workload, chk["sample"], chk["checked"])
        c = chk["checked"]
        assert "error" not in chk
        assert c["contigs"] >= min_sample and c["paf_identical"] == c["contigs"] == c["tsv_rows_identical"]
        return res, pipe
    finally:
        del pipe
        gc.collect()
        gpu.torch.cuda.empty_cache()
        gpu.trim()


@pytest.mark.timeout(900)
def test_config_c4_cami_medium_sampled_oracle(gpu):
    """BASELINE.json configs[3] "CAMI-medium" on one GPU (the 8-GPU sharding is
    tests/test_bench_launch.py + test_pipeline_gpu.py::test_world2_pipeline_equals_world1)."""
    res, _ = _run(gpu, "cami-medium", 8.0, 1000)
    assert len(res.selected) == 744


@pytest.mark.timeout(1200)
def test_config_c5_cami_high_three_dbs_sampled_oracle(gpu):
    """BASELINE.json configs[4] "CAMI-high: all three sketch DBs + full candidate set"."""
    res, pipe = _run(gpu, "cami-high", 8.0, 150)
    assert len(res.selected) == 5000
    assert len(res.screen_rows) == 3

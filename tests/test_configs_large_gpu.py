"""BASELINE.json configs[3] and [4] at full size on one MI355X.

The workloads are bench.py's own (bench.build_cami): C4 CAMI-medium = 12 taxa, 744
candidates / 3.06 Gbp in two -I2g parts, 151k contigs / 1 Gbp, a 1e8-hash sketch DB;
C5 CAMI-high = 14 taxa, the full CAND_MAX of 5,000 candidates / ~20 Gbp in ten parts,
~300k contigs / 2 Gbp, three sketch DBs of 1e8 / 5e7 / 1e7 hashes
(run_hymet_cami.sh:26,83-99).

* C4, every contig: the CPU oracle ran the whole workload once
  (tests/golden/make_cami_golden.py -> tests/golden/cami/cami-medium.{json,npz}); the GPU run
  must give the same screen arrays (shared / median of all 1e5 references), the same
  selected list, every contig's PAF lines (count + digest) and TSV row, and the same TSV
  bytes.  ref_abundance counts every PAF line of the run (classification_cami.py:181-208),
  so the full comparison is what pins the TSV.
* C5, stratified: the three-DB screen in full against the oracle's arrays
  (tests/golden/cami/cami-high-screen), then every contig of >= 90 kbp (a group of > 16,384
  anchors needs >= 16,384 x 5.5 / 0.94 ~ 96 kbp of query at 2/(w+1) minimizers per base and
  <= 5 % divergence, so this set holds every query that reaches the large-group sort, the
  wave backtrack and the long join's biggest groups) plus 5,000 random contigs mapped by the
  oracle on this host's cores against the same index parts (bench.cpu_baseline_cami)."""
import gc
import os
from pathlib import Path

import numpy as np
import pytest

from tests import _digest

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden" / "cami"


@pytest.fixture(scope="module")
def gpu():
    from hymet_amd._lib import Gpu
    return Gpu(0)


def _release(gpu, pipe):
    del pipe
    gc.collect()
    gpu.torch.cuda.empty_cache()
    gpu.trim()


def _check_inputs(meta, fasta, pipe):
    assert _digest.sha(fasta) == meta["fasta_sha256"]
    # the GPU-sketched DBs (read back from the .msh files) hash like the oracle-sketched ones
    assert [_digest.sha(np.ascontiguousarray(d.hashes, np.uint64)) for d in pipe.dbs] == meta["db_hashes_sha256"]


def _check_screen(meta, z, res):
    for d, r in enumerate(res.screen):
        np.testing.assert_array_equal(r.shared, z[f"screen{d}_shared"], err_msg=f"DB {d} shared")
        np.testing.assert_array_equal(r.median, z[f"screen{d}_median"], err_msg=f"DB {d} median")
        assert r.set_size == meta[f"screen{d}_set_size"] and r.n_kmers == meta[f"screen{d}_n_kmers"]
    assert len(res.selected) == meta["selected"]
    assert _digest.sha("".join(n + "\n" for n in res.selected).encode()) == meta["selected_sha256"]


@pytest.mark.timeout(900)
def test_config_c4_cami_medium_every_contig(gpu):
    """BASELINE.json configs[3] "CAMI-medium" on one GPU, every contig against the oracle's
    full run (the 8-GPU sharding: tests/test_bench_launch.py +
    test_pipeline_gpu.py::test_world2_pipeline_equals_world1)."""
    import bench
    from hymet_amd.dist import Comm
    meta, z = _digest.load(str(GOLD / "cami-medium"))
    args = bench.parse_args(["--workload", "cami-medium"])
    w, db, pipe, fasta, refs_ss, tax, hier, td = bench.build_cami(args, Comm(), gpu)
    try:
        _check_inputs(meta, fasta, pipe)
        res = pipe.run(fasta, with_paf=True)
        _check_screen(meta, z, res)
        assert len(res.selected) == 744
        index = _digest.name_index(w.contig_names)
        cnt, dig = _digest.paf_digests(res.paf_bytes, index)
        assert int(cnt.sum()) == meta["paf_lines"] == res.n_paf_lines
        assert np.array_equal(cnt, z["paf_count"]), _digest.diff_report("PAF line counts", cnt, z["paf_count"])
        assert np.array_equal(dig, z["paf_digest"]), _digest.diff_report("PAF lines", dig, z["paf_digest"])
        assert _digest.sha(res.paf_bytes) == meta["paf_sha256"]
        tsv_sha, tdig, order = _digest.tsv_digests(res.tsv, index)
        assert np.array_equal(tdig, z["tsv_digest"]), _digest.diff_report("TSV rows", tdig, z["tsv_digest"])
        assert np.array_equal(order, z["tsv_order"])
        assert tsv_sha == meta["tsv_sha256"] and res.n_queries == meta["tsv_rows"]
        print(f"C4: {len(w.contigs)} contigs, {meta['paf_lines']} PAF lines, {meta['tsv_rows']} TSV rows identical "
              f"to the oracle's full run")
    finally:
        _release(gpu, pipe)


def c5_long_contigs(w, min_len=90_000):
    """Indices of C5's contigs of >= min_len bases, longest first."""
    lens = np.array([len(c) for c in w.contigs], np.int64)
    idx = np.flatnonzero(lens >= min_len)
    return idx[np.argsort(-lens[idx], kind="stable")].tolist()


@pytest.mark.timeout(1200)
def test_config_c5_cami_high_screen_full_and_stratified_sample(gpu):
    """BASELINE.json configs[4] "CAMI-high: all three sketch DBs + full candidate set"."""
    import bench
    from hymet_amd.dist import Comm
    meta, z = _digest.load(str(GOLD / "cami-high-screen"))
    args = bench.parse_args(["--workload", "cami-high", "--cpu-threads", str(bench.cpu_threads_default())])
    w, db, pipe, fasta, refs_ss, tax, hier, td = bench.build_cami(args, Comm(), gpu)
    try:
        _check_inputs(meta, fasta, pipe)
        res = pipe.run(fasta, with_paf=True)
        assert res.n_queries == len(w.contigs) and res.n_classified >= 0.99 * res.n_queries
        _check_screen(meta, z, res)
        assert len(res.selected) == 5000 and len(res.screen_rows) == 3
        must = c5_long_contigs(w)
        assert len(must) >= 100 and len(w.contigs[must[0]]) >= 500_000
        chk = bench.cpu_baseline_cami(args, pipe, res, fasta, db, tax, hier, must=must, n_random=5000)
        print("C5", chk["sample"], chk["checked"])
        c = chk["checked"]
        assert "error" not in chk
        assert c["contigs"] == len(must) + 5000
        assert c["paf_identical"] == c["contigs"] == c["tsv_rows_identical"]
    finally:
        _release(gpu, pipe)

"""The GPU mapping path on the reference's real Zymo genomes (tests/_zymo.py,
tests/test_zymo_real.py): index over the 63 shipped sequences (minimap2 -I2g -d defaults,
scripts/minimap2.sh:12), asm10 mapping of the 322 re-cut contigs (:23).

* against the REAL minimap2 fixture: the same primary- and secondary-agreement bars as the
  CPU restatement (misses diagnosed by the oracle with pri_ratio / best_n relaxed);
* against the restatement (oracle/mm_oracle.c): the PAF text byte for byte on real genomes
  (repeats, plasmids, near-identical strains, a 12 Mbp eukaryote)."""
import os

import pytest

from tests import _zymo as z
from tests.test_zymo_real import check_agreement, check_secondaries, relaxed_opt

pytestmark = pytest.mark.gpu
THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def gpu():
    from hymet_amd._lib import Gpu
    return Gpu(0)


@pytest.mark.timeout(600)
def test_gpu_mapping_real_genomes_vs_minimap2_fixture_and_oracle(gpu):
    from hymet_amd import cli, ingest
    from hymet_amd.seqio import from_records
    from oracle import pipeline_oracle
    seqs = z.sequences()
    refs = from_records([(n, "", s) for n, s in seqs])
    parts, names, lens, first = cli.build_parts(gpu, refs, "2g", 50e6)
    assert len(parts) == 1
    q = z.recut_queries()
    fasta = ingest.to_fasta([n for n, _, _ in q], [s for _, s, _ in q])
    paf = cli.map_paf(gpu, parts, names, lens, first, fasta).decode().splitlines()
    a = z.primary_agreement(q, paf)
    print({k: v for k, v in a.items() if k != "misses"}, a["misses"])
    check_agreement(a)
    o_paf = pipeline_oracle.map_paf([n for n, _ in seqs], [s for _, s in seqs], [(n, s) for n, s, _ in q],
                                    threads=THREADS)
    assert len(paf) == len(o_paf) and paf == o_paf
    relaxed = pipeline_oracle.map_paf([n for n, _ in seqs], [s for _, s in seqs], [(n, s) for n, s, _ in q],
                                      threads=THREADS, opt=relaxed_opt())
    s = z.secondary_agreement(q, paf, relaxed)
    print({k: v for k, v in s.items() if k not in ("misses", "extras")})
    check_secondaries(s)

"""End-to-end: the fused GPU hot path vs the CPU oracle pipeline on a C1-shaped input
(3 taxa, 60 contigs): same selected candidates, same PAF lines, byte-identical TSV."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    from hymet_amd._lib import Gpu
    return Gpu(0)


def _setup(gpu, tmp_path):
    from hymet_amd import screen as scr
    from hymet_amd import synth
    from hymet_amd.msh import SketchDB
    from hymet_amd.seqio import DevicePool, from_records
    rng = np.random.default_rng(7)
    w = synth.make_cami(rng, n_taxa=3, per_taxon=4, genome_mbp=(0.3, 0.5), contig_gbp=0.0006, max_contigs=60, name="tiny")
    refs_ss = from_records([(n, "", s) for n, s in zip(w.ref_names, w.refs)])
    sk = scr.sketch_sequences(gpu, DevicePool(gpu, refs_ss, DevicePool.ALPHA_MASH), 21, 42, 1000)
    dec = synth.decoy_sketches(rng, 40, 1000)
    hl = sk + [d for d in dec]
    off = np.zeros(len(hl) + 1, np.int64)
    off[1:] = np.cumsum([len(h) for h in hl])
    names = [n + ".fna.gz" for n in w.ref_names] + [f"decoy_{i}.fna.gz" for i in range(len(dec))]
    db = SketchDB(names=names, comments=[f"[1 seqs] {n}" for n in names], lengths=np.ones(len(hl), np.int64),
                  offsets=off, hashes=np.concatenate(hl))
    tax = tmp_path / "detailed_taxonomy.tsv"
    tax.write_text(w.taxonomy_tsv())
    hier = tmp_path / "taxonomy_hierarchy.tsv"
    hier.write_text(w.hierarchy_tsv())
    by_name = {n + ".fna.gz": (n, s) for n, s in zip(w.ref_names, w.refs)}
    return w, db, by_name, tax, hier


def test_pipeline_matches_oracle(gpu, tmp_path):
    from hymet_amd import pipeline
    from hymet_amd.seqio import from_records
    from oracle import oracle_lib, pipeline_oracle
    w, db, by_name, tax, hier = _setup(gpu, tmp_path)
    # small -I so that the candidate set spans two index parts (mid_occ from part 1)
    cfg = pipeline.Config(split_idx="2m", index_mini_batch=1e6, map_batch_bases=300_000)

    def ref_lookup(names):
        return from_records([(by_name[n][0], "", by_name[n][1]) for n in names])

    p = pipeline.Pipeline(gpu, [db], ref_lookup, tax, hier, cfg)
    queries = from_records([(n, "", s) for n, s in zip(w.contig_names, w.contigs)])
    res = p.run(queries, with_paf=True)
    o_sel, o_paf, o_tsv = pipeline_oracle.run(list(zip(w.contig_names, w.contigs)), [db],
                                              lambda names: ([by_name[n][0] for n in names], [by_name[n][1] for n in names]),
                                              tax, hier, part_bases=2e6, mini_batch=1e6)
    assert len(p.index_for(res.selected).parts) >= 2
    assert res.selected == o_sel
    assert len(o_sel) == 12
    assert res.paf == o_paf
    assert res.tsv == o_tsv
    assert res.n_classified >= 55

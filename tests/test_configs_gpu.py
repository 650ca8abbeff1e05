"""Parity at configuration size (BASELINE.json configs[0..2]; SURVEY.md §8(d) C1-C3;
C4 / C5 in tests/test_configs_large_gpu.py).

* C1 tiny, main.pl path: 60 contigs cut from three real Zymo chromosomes, legacy
  classifier, no limit step; selected list, PAF and TSV identical to the oracle.
* C2 Zymo screen: the 1,043 fixture contigs at their exact lengths, re-cut from the real
  Zymo genomes (tests/_zymo.py), against the 25 real genome sketches + 99,975 decoys (1e8
  hashes, the sketch1 size of BASELINE.md / SURVEY.md §8(d)).
  Counts, shared, median, set size, screen.tab rows and the mash.sh selection bit-exact vs
  the CPU oracle.
* C3 CAMI-low: 8 taxa, 147 candidate genomes of 3-5 Mbp (0.58 Gbp; bench/results_summary.md:90),
  15,130 contigs / 100 Mbp, one index part, end to end (screen -> select -> limit -> index -> map ->
  classify) vs oracle/pipeline_oracle: selected candidates, PAF lines and TSV bytes
  identical, with one mapping batch and again with many.
* A Pipeline reused on a second, repeat-rich candidate set resolves mid_occ from that set
  (options.c mm_mapopt_update in a fresh minimap2 process) and matches the oracle.
* The run_hymet_cami.sh:182-206 fallback inside the fused path.

C1/C2 use the reference's real genomes; C3 is seeded synthetic (the CAMI data does not
ship).  The oracle restates Mash / minimap2; its minimap2 part is pinned against the real
minimap2 PAF the reference ships (tests/test_zymo_real.py), Mash stays unpinned
(DESIGN.md §4)."""
import functools
import os
from pathlib import Path

import numpy as np
import pytest

from tests import _zymo as z
from tests._data import mutate

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"
THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def gpu():
    from hymet_amd._lib import Gpu
    return Gpu(0)


def zymo_qlens():
    """Query lengths of the reference's Zymo PAF fixture, one per contig, file order."""
    seen, out = set(), []
    for line in (GOLD / "classify" / "zymo.paf").read_text().splitlines():
        p = line.split("\t")
        if len(p) > 1 and p[0] not in seen:
            seen.add(p[0])
            out.append(int(p[1]))
    return out


def _sketch_all(seqs):
    """Mash sketches (k21, seed 42, s1000) of each sequence on the CPU oracle, threaded."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle_lib
    with ThreadPoolExecutor(THREADS) as ex:
        return list(ex.map(lambda g: np.sort(oracle_lib.sketch([g], 21, 42, 1000)), seqs))


def _db(names, sketches, decoys, lengths):
    from hymet_amd.msh import SketchDB
    hl = list(sketches) + list(decoys)
    off = np.zeros(len(hl) + 1, np.int64)
    off[1:] = np.cumsum([len(h) for h in hl])
    names = list(names) + [f"GCF_{900000000 + i:09d}.1_decoy_genomic.fna.gz" for i in range(len(decoys))]
    return SketchDB(names=names, comments=[f"[1 seqs] {n} [...]" for n in names],
                    lengths=np.array(list(lengths) + [4_000_000] * len(decoys), np.int64), offsets=off,
                    hashes=np.concatenate(hl))


@functools.lru_cache(maxsize=1)
def _zymo_sketches():
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle_lib
    with ThreadPoolExecutor(THREADS) as ex:
        return list(ex.map(lambda f: np.sort(oracle_lib.sketch([s for _, s in f[2]], 21, 42, 1000)), z.genome_files()))


def _zymo_db(n_decoys, seed=1):
    """sketch1-shaped DB: one Mash sketch per shipped Zymo genome FILE (mash sketch of a
    multi-record file = one reference, named by the file) + seeded decoy references."""
    from hymet_amd import synth
    files = z.genome_files()
    sk = _zymo_sketches()
    return _db([f[1] for f in files], sk, synth.decoy_sketches(np.random.default_rng(seed), n_decoys, 1000),
               [sum(len(s) for _, s in f[2]) for f in files])


@pytest.mark.timeout(600)
def test_config_c2_zymo_screen_real_contigs(gpu):
    """BASELINE.json configs[1] "Zymo mock contigs: MinHash sketch+Jaccard vs sketch1.msh on 1
    MI355X (screen stage only)" (SURVEY.md §8(d) C2): the 1,043 fixture contigs at their
    exact lengths, re-cut from the real genomes at each contig's primary hit
    (tests/_zymo.py; 726 Cryptococcus contigs from a seeded synthetic genome, that FASTA is
    missing) against the 25 real genome sketches + 99,975 decoys: H = 1e8 hashes, sketch1's
    size."""
    from hymet_amd import screen as scr
    from hymet_amd import select as sel
    from hymet_amd.seqio import DevicePool, from_records
    from oracle import oracle_lib, select_oracle as so
    recs = z.c2_contigs()
    assert len(recs) == 1043 and sum(len(s) for _, s in recs) == 53_805_448
    seqs = [s for _, s in recs]
    db = _zymo_db(99975)
    assert len(db.hashes) == 100_000_000
    pool = DevicePool(gpu, from_records([(n, "", s) for n, s in recs]), DevicePool.ALPHA_MASH)
    res = scr.screen(gpu, pool, [db])[0]
    sh, md, set_size, nk = oracle_lib.ScreenOracle(db).run(seqs)
    assert res.n_kmers == nk
    np.testing.assert_array_equal(res.shared, sh)
    np.testing.assert_array_equal(res.median, md)
    assert res.set_size == set_size
    refs = [(db.names[i], db.comments[i], int(db.offsets[i + 1] - db.offsets[i])) for i in range(db.n_refs)]
    lines = res.lines(v_max=0.9)
    assert lines == so.screen_lines(refs, sh, md, set_size, 21)
    # every shipped species is in the pool: all 25 genome files share hashes with it
    assert sum(1 for x in res.shared[:25] if x > 0) == 25
    rows = sel.sort_gr(sel.sort_unique_k5(lines))
    assert rows == so.sort_gr(so.sort_unique_k5(lines))
    got = sel.threshold_walk(rows, "0.9", 1)
    exp = so.select_threshold(rows, "0.9", 1)
    assert got[:3] == exp[:3] and len(got[2]) >= 5


@pytest.mark.timeout(600)
def test_config_c1_tiny_main_pl_path(gpu, tmp_path):
    """BASELINE.json configs[0] "testdataset/ tiny FASTA via main.pl" (SURVEY.md §8(d) C1):
    60 contigs of U[5k, 50k] cut from three real Zymo chromosomes (E. coli GCF_000005845.2,
    B. subtilis GCF_000009045.1, S. aureus GCF_000013425.1) with 1 % substitutions, seed 0,
    through main.pl's sequence (main.pl:93-113): mash.sh on sketch1 (the 25 genomes) and a
    decoy sketch2, sort -u union WITHOUT limit_candidates, minimap2 -I2g -d / -x asm10 over
    the selected genome files, and the legacy classification.py.  Selected list, PAF and
    TSV bytes identical to the oracle pipeline."""
    from hymet_amd import classify as cls
    from hymet_amd import pipeline, synth
    from hymet_amd.seqio import from_records
    from oracle import pipeline_oracle
    rng = np.random.default_rng(0)
    chrom = {f[1].split("_genomic")[0]: f[2][0] for f in z.genome_files()}
    src = [chrom[k] for k in ("GCF_000005845.2_ASM584v2", "GCF_000009045.1_ASM904v1", "GCF_000013425.1_ASM1342v1")]
    recs = []
    for i in range(60):
        name, g = src[i % 3]
        L = int(rng.integers(5000, 50001))
        st = int(rng.integers(0, len(g) - L))
        recs.append((f"contig_{i + 1}", mutate(rng, g[st:st + L], 0.01)))
    assert 1.0e6 < sum(len(c) for _, c in recs) < 2.2e6
    db1 = _zymo_db(0)
    db2 = _db([], [], synth.decoy_sketches(np.random.default_rng(5), 40, 1000), [])
    by_file = {f[1]: f[2] for f in z.genome_files()}

    def glook(names):
        return from_records([(n, "", s) for f in names for n, s in by_file[f]])

    def olook(names):
        recs_ = [r for f in names for r in by_file[f]]
        return [n for n, _ in recs_], [s for _, s in recs_]

    tax, hier = str(GOLD / "classify" / "zymo_taxonomy.tsv"), str(GOLD / "classify" / "zymo_hierarchy_superkingdom.tsv")
    p = pipeline.Pipeline(gpu, [db1, db2], glook, tax, hier, pipeline.Config(limit=False), variant=cls.LEGACY)
    res = p.run(from_records([(n, "", s) for n, s in recs]), with_paf=True)
    o_sel, o_paf, o_tsv = pipeline_oracle.run(recs, [db1, db2], olook, tax, hier, cand_max=None, threads=THREADS,
                                              legacy=True)
    assert res.selected == o_sel and len(o_sel) >= 3
    assert res.selected == sorted(res.selected, key=lambda n: n.encode())      # the sort -u union, no limit
    assert res.paf == o_paf and len(o_paf) >= 60
    assert res.tsv == o_tsv
    assert res.n_classified >= 55


def _cami_low():
    """147 candidate genomes of 3-5 Mbp (~0.6 Gbp, bench/results_summary.md:90)
    and ~100 Mbp of contigs (~15k at CAMI's lognormal lengths)."""
    from hymet_amd import synth
    rng = np.random.default_rng(2)
    per = [19, 19, 19, 18, 18, 18, 18, 18]
    w = synth.make_cami(rng, n_taxa=8, per_taxon=per, contig_gbp=0.1, max_contigs=20_000, name="cami-low")
    assert len(w.refs) == 147 and 0.5e9 < w.ref_bases < 0.7e9
    assert 0.099e9 <= w.contig_bases < 0.11e9 and len(w.contigs) > 14_000
    return w, rng


def _community_db(w, rng, n_decoys):
    from hymet_amd import synth
    sk = _sketch_all(w.refs)
    return _db([n + ".fna.gz" for n in w.ref_names], sk, synth.decoy_sketches(rng, n_decoys, 1000),
               [len(r) for r in w.refs])


def _write_tax(tmp_path, w, tax_header="GCF\tTaxID\tIdentifiers"):
    tax = tmp_path / "detailed_taxonomy.tsv"
    body = w.taxonomy_tsv().split("\n", 1)[1]
    tax.write_text(tax_header + "\n" + body)
    hier = tmp_path / "taxonomy_hierarchy.tsv"
    hier.write_text(w.hierarchy_tsv())
    return tax, hier


def _lookups(*ws):
    """(GPU, oracle) genome-cache lookups over the candidates of one or more communities
    (downloadDB.py's combined_genomes.fasta in selection order)."""
    from hymet_amd.seqio import from_records
    by_name = {n + ".fna.gz": (n, s) for w in ws for n, s in zip(w.ref_names, w.refs)}

    def gpu_lookup(names):
        return from_records([(by_name[n][0], "", by_name[n][1]) for n in names])

    def oracle_lookup(names):
        return [by_name[n][0] for n in names], [by_name[n][1] for n in names]

    return gpu_lookup, oracle_lookup


@pytest.mark.timeout(900)
def test_config_c3_cami_low_end_to_end(gpu, tmp_path):
    """BASELINE.json configs[2] "CAMI-low subset: full sketch->limit_candidates->
    minimizer-chain->classify on 1 MI355X", at SURVEY.md §8(d)'s shape: 147 candidates /
    0.58 Gbp in one -I2g part, 15,130 contigs / 100 Mbp.  The oracle maps the whole pool on
    the host's cores (~100 s on 8 threads, ~60 s on the GPU box's 16)."""
    from hymet_amd import pipeline
    from hymet_amd.seqio import from_records
    from oracle import pipeline_oracle
    w, rng = _cami_low()
    db = _community_db(w, rng, 300)
    tax, hier = _write_tax(tmp_path, w)
    gpu_lookup, oracle_lookup = _lookups(w)
    queries = from_records([(n, "", s) for n, s in zip(w.contig_names, w.contigs)])
    p = pipeline.Pipeline(gpu, [db], gpu_lookup, str(tax), str(hier), pipeline.Config())
    res = p.run(queries, with_paf=True)
    assert len(p.index_for(res.selected).parts) == 1
    o_sel, o_paf, o_tsv = pipeline_oracle.run(list(zip(w.contig_names, w.contigs)), [db], oracle_lookup, str(tax),
                                              str(hier), threads=THREADS)
    assert len(o_sel) == 147
    assert res.selected == o_sel
    assert len(res.paf) == len(o_paf) and res.paf == o_paf
    assert res.tsv == o_tsv
    assert res.n_classified >= 0.95 * len(w.contigs)
    # the same pool cut into many mapping batches on two streams: identical bytes
    p.cfg.map_batch_bases = 7_000_000
    res2 = p.run(queries, with_paf=True)
    assert res2.paf == o_paf and res2.tsv == o_tsv


@pytest.mark.timeout(300)
def test_reused_pipeline_resolves_mid_occ_per_candidate_set(gpu, tmp_path):
    """First run: 3 taxa x 4 strains (mid_occ clamps to 50).  Second run on the same
    Pipeline: 2 taxa x 60 strains, so every minimizer occurs ~60 times and mid_occ follows
    the new first part; a stale 50 would drop those seeds and change every PAF line."""
    from hymet_amd import pipeline, synth
    from hymet_amd.seqio import from_records
    from oracle import pipeline_oracle
    wa = synth.make_cami(np.random.default_rng(11), n_taxa=3, per_taxon=4, genome_mbp=(0.2, 0.3), contig_gbp=0.0005,
                         max_contigs=40, name="a")
    wb = synth.make_cami(np.random.default_rng(12), n_taxa=2, per_taxon=60, genome_mbp=(0.10, 0.15),
                         contig_gbp=0.0005, max_contigs=40, name="b")
    wb.ref_names = [n.replace("GCF_", "GCA_") for n in wb.ref_names]
    wb.taxids = [500000 + 1000 * t for t in range(2)]
    rng = np.random.default_rng(13)
    da, db_ = _community_db(wa, rng, 20), _community_db(wb, rng, 20)
    # one sketch DB, one taxonomy and one genome cache holding both communities
    from hymet_amd.msh import SketchDB
    both = SketchDB(names=da.names + db_.names, comments=da.comments + db_.comments,
                    lengths=np.r_[da.lengths, db_.lengths], offsets=np.r_[da.offsets[:-1], db_.offsets + da.offsets[-1]],
                    hashes=np.r_[da.hashes, db_.hashes])
    ta, ha = _write_tax(tmp_path, wa)
    tb_text = wb.taxonomy_tsv().split("\n", 1)[1]
    (tmp_path / "detailed_taxonomy.tsv").write_text(ta.read_text() + tb_text)
    hb = wb.hierarchy_tsv().replace("Species", "Other")
    (tmp_path / "taxonomy_hierarchy.tsv").write_text(ha.read_text() + hb.split("\n", 1)[1])
    glook, olook = _lookups(wa, wb)
    tax, hier = str(tmp_path / "detailed_taxonomy.tsv"), str(tmp_path / "taxonomy_hierarchy.tsv")
    p = pipeline.Pipeline(gpu, [both], glook, tax, hier, pipeline.Config())
    p.run(from_records([(n, "", s) for n, s in zip(wa.contig_names, wa.contigs)]))
    mid_a = p.opt.mid_occ
    res = p.run(from_records([(n, "", s) for n, s in zip(wb.contig_names, wb.contigs)]), with_paf=True)
    assert p.opt.mid_occ != mid_a
    o_sel, o_paf, o_tsv = pipeline_oracle.run(list(zip(wb.contig_names, wb.contigs)), [both], olook, tax, hier,
                                              threads=THREADS)
    assert res.selected == o_sel and res.paf == o_paf and res.tsv == o_tsv


def test_fused_fallback_when_classifier_cannot_load(gpu, tmp_path):
    """classification_cami.py dies on a taxonomy without a TaxID column (:75-76), leaving an
    empty TSV; run_hymet_cami.sh then runs build_id_map (positional columns) + mini_classify."""
    from hymet_amd import pipeline, synth
    from hymet_amd.seqio import from_records
    from oracle import classify_oracle, pipeline_oracle
    w = synth.make_cami(np.random.default_rng(21), n_taxa=2, per_taxon=3, genome_mbp=(0.2, 0.3), contig_gbp=0.0003,
                        max_contigs=30, name="fb")
    db = _community_db(w, np.random.default_rng(22), 10)
    tax, hier = _write_tax(tmp_path, w, tax_header="GCF\tTaxonomyID\tIdentifiers")
    gl, ol = _lookups(w)
    p = pipeline.Pipeline(gpu, [db], gl, str(tax), str(hier), pipeline.Config())
    assert p.classifier is None
    res = p.run(from_records([(n, "", s) for n, s in zip(w.contig_names, w.contigs)]), with_paf=True)
    sel, _ = pipeline_oracle.select(list(w.contigs), [db])
    assert res.selected == sel
    names, seqs = ol(sel)
    o_paf = pipeline_oracle.map_paf(names, seqs, list(zip(w.contig_names, w.contigs)))
    paf_file = tmp_path / "resultados.paf"
    paf_file.write_text("".join(l + "\n" for l in o_paf))
    assert res.paf == o_paf
    assert res.tsv == classify_oracle.fallback_classify(str(paf_file), str(tax))
    assert res.tsv.count(b"\tunknown\tunknown\t1.0000\n") >= 25

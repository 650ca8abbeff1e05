"""Parity at configuration size (BASELINE.json configs[1] and [2]).

* C2 Zymo screen: 1,043 contigs with the exact query-length multiset of the reference's
  Zymo PAF fixture (case/truth/zymo_mc/zymo_mc_vs_refs.paf col 2, committed as
  tests/golden/classify/zymo.paf; 53.8 Mbp) against a sketch1-shaped DB of 2,000
  references x 1,000 hashes (25 genome sketches + decoys, 2e6 hashes).  Counts, shared,
  median, set size, screen.tab rows and the mash.sh selection must be bit-exact vs the CPU
  oracle.
* C3 CAMI-low: 8 taxa, 147 candidate genomes (bench/results_summary.md:90), 2,100 contigs,
  one index part, end to end (screen -> select -> limit -> index -> map -> classify) vs
  oracle/pipeline_oracle: selected candidates, PAF lines and TSV bytes identical, with one
  mapping batch and again with seven.
* A Pipeline reused on a second, repeat-rich candidate set resolves mid_occ from that set
  (options.c mm_mapopt_update in a fresh minimap2 process) and matches the oracle.
* The run_hymet_cami.sh:182-206 fallback inside the fused path.

Sequences are seeded synthetic stand-ins (the Zymo contig FASTA is absent from the
reference); the oracle restates Mash / minimap2 (parity unpinned against the
real tools)."""
import os
from pathlib import Path

import numpy as np
import pytest

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


def test_c2_zymo_screen_config_size(gpu):
    from hymet_amd import screen as scr
    from hymet_amd import select as sel
    from hymet_amd import synth
    from hymet_amd.seqio import DevicePool, from_records
    from oracle import oracle_lib, select_oracle as so
    qlens = zymo_qlens()
    assert len(qlens) == 1043 and abs(sum(qlens) - 53.8e6) < 0.1e6
    rng = np.random.default_rng(1)
    sizes = [7_000_000] + [int(rng.uniform(2e6, 4.5e6)) for _ in range(9)]
    base = [synth.random_codes(rng, n, gc=0.38 + 0.03 * i) for i, n in enumerate(sizes)]
    genomes = base + [synth.mutate_codes(rng, base[i % 10], 0.002 + 0.002 * i) for i in range(15)]   # 25 "Zymo" refs
    recs = []
    for i, L in enumerate(qlens):
        ok = [g for g in range(10) if len(base[g]) > L]
        g = base[ok[int(rng.integers(len(ok)))]]
        st = int(rng.integers(0, len(g) - L))
        c = synth.mutate_codes(rng, g[st:st + L], 0.01)
        if rng.random() < 0.5:
            c = (3 - c)[::-1]
        recs.append((f"ctg{i + 1}", "", synth.to_ascii(c)))
    seqs = [r[2] for r in recs]
    ref_ascii = [synth.to_ascii(g) for g in genomes]
    sk = _sketch_all(ref_ascii)
    db = _db([f"GCF_{i:09d}.1_zymo{i}_genomic.fna.gz" for i in range(25)], sk,
             synth.decoy_sketches(rng, 1975, 1000), [len(g) for g in genomes])
    assert len(db.hashes) >= 1_000_000
    pool = DevicePool(gpu, from_records(recs), DevicePool.ALPHA_MASH)
    res = scr.screen(gpu, pool, [db])[0]
    sh, md, set_size, nk = oracle_lib.ScreenOracle(db).run(seqs)
    assert res.n_kmers == nk
    np.testing.assert_array_equal(res.shared, sh)
    np.testing.assert_array_equal(res.median, md)
    assert res.set_size == set_size
    refs = [(db.names[i], db.comments[i], int(db.offsets[i + 1] - db.offsets[i])) for i in range(db.n_refs)]
    lines = res.lines(v_max=0.9)
    assert lines == so.screen_lines(refs, sh, md, set_size, 21)
    assert sum(1 for x in res.shared[:25] if x > 0) == 25
    rows = sel.sort_gr(sel.sort_unique_k5(lines))
    assert rows == so.sort_gr(so.sort_unique_k5(lines))
    got = sel.threshold_walk(rows, "0.9", 1)
    exp = so.select_threshold(rows, "0.9", 1)
    assert got[:3] == exp[:3] and len(got[2]) >= 5


def _cami_low():
    from hymet_amd import synth
    rng = np.random.default_rng(2)
    per = [19, 19, 19, 18, 18, 18, 18, 18]
    w = synth.make_cami(rng, n_taxa=8, per_taxon=per, genome_mbp=(0.6, 1.0), contig_gbp=0.05, max_contigs=2100,
                        name="cami-low")
    assert len(w.refs) == 147 and len(w.contigs) == 2100
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


@pytest.mark.timeout(600)
def test_c3_cami_low_end_to_end(gpu, tmp_path):
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
    assert res.n_classified >= 2000
    # the same pool cut into seven mapping batches: identical bytes
    p.cfg.map_batch_bases = 2_000_000
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

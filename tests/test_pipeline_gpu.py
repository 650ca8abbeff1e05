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


def _fasta_text(w, quote_name=True):
    """FASTA bytes as an assembler writes them: 60-column lines, some records with CRLF, a
    comment on the header, junk before the first record, one name holding a quote."""
    out = [b"# assembly k141\n"]
    for i, (n, s) in enumerate(zip(w.contig_names, w.contigs)):
        name = n + ('"x' if quote_name and i == 3 else "")
        eol = b"\r\n" if i % 5 == 1 else b"\n"
        out.append(b">" + name.encode() + b" flag=1 multi=2.0 len=" + str(len(s)).encode() + eol)
        out.append(eol.join(s[j:j + 60] for j in range(0, len(s), 60)) + eol)
    return b"".join(out)


def test_fasta_bytes_path_matches_oracle(gpu, tmp_path):
    """The bench's input form: FASTA text in host memory -> native record table -> one H2D
    copy -> device line-break compaction; and csv quoting of a query name and a lineage
    label holding '"' (written by the GPU TSV writer)."""
    from hymet_amd import pipeline
    from hymet_amd.seqio import from_records, parse_fasta_bytes
    from oracle import pipeline_oracle
    w, db, by_name, tax, hier = _setup(gpu, tmp_path)
    hier.write_text(hier.read_text().replace("SpeciesA synthetica", 'SpeciesA "synthetica"'))
    data = _fasta_text(w)
    recs = [(n, s) for n, _, s in parse_fasta_bytes(data)]
    assert len(recs) == len(w.contigs) and recs[3][0].endswith('"x')

    def ref_lookup(names):
        return from_records([(by_name[n][0], "", by_name[n][1]) for n in names])

    p = pipeline.Pipeline(gpu, [db], ref_lookup, str(tax), str(hier), pipeline.Config(map_batch_bases=400_000))
    res = p.run(data, with_paf=True)
    o_sel, o_paf, o_tsv = pipeline_oracle.run(recs, [db],
                                              lambda names: ([by_name[n][0] for n in names], [by_name[n][1] for n in names]),
                                              str(tax), str(hier))
    assert res.selected == o_sel
    assert res.paf == o_paf
    assert res.tsv == o_tsv
    assert b'"SpeciesA ""synthetica""' in res.tsv or b'""synthetica""' in res.tsv
    assert b'"k141_3""x"' in res.tsv or not any(l.startswith('k141_3"x') for l in o_paf)


def test_legacy_variant_fused_matches_oracle(gpu, tmp_path):
    """main.pl's classifier (classification.py) on the device PAF: superkingdom-labelled
    hierarchy, and one contig that IS a candidate genome (same name, full length) so the
    exact-match shortcut (:141-151) fires."""
    from hymet_amd import classify as cls
    from hymet_amd import pipeline
    from hymet_amd.seqio import from_records
    from oracle import classify_oracle, pipeline_oracle
    w, db, by_name, tax, hier = _setup(gpu, tmp_path)
    hier.write_text(hier.read_text().replace("domain:", "superkingdom:"))
    names = list(w.contig_names) + [w.ref_names[0]]
    seqs = list(w.contigs) + [w.refs[0]]

    def ref_lookup(ns):
        return from_records([(by_name[n][0], "", by_name[n][1]) for n in ns])

    p = pipeline.Pipeline(gpu, [db], ref_lookup, str(tax), str(hier), pipeline.Config(), variant=cls.LEGACY)
    res = p.run(from_records([(n, "", s) for n, s in zip(names, seqs)]), with_paf=True)
    sel, _ = pipeline_oracle.select(seqs, [db])
    assert res.selected == sel
    o_paf = pipeline_oracle.map_paf([by_name[n][0] for n in sel], [by_name[n][1] for n in sel], list(zip(names, seqs)))
    assert res.paf == o_paf
    pf = tmp_path / "resultados.paf"
    pf.write_text("".join(l + "\n" for l in o_paf))
    exp = classify_oracle.classify_legacy(str(pf), str(tax), str(hier))
    assert res.tsv == exp
    assert (w.ref_names[0] + "\t").encode() in exp and b"\t1.0000\r\n" in exp


def test_emit_tsv_confidence_rounding(gpu):
    """'%.4f' on the device == Python's correctly rounded formatting, ties to even included
    (x/32 values are exact binary ties at 4 decimals)."""
    import csv
    import io
    import ctypes
    from hymet_amd._lib import ptr
    torch = gpu.torch
    rng = np.random.default_rng(4)
    conf = [0.0, 1.0, 0.03125, 0.28125, 0.59375, 0.96875, 5e-5, 0.99995, 0.12345, 0.5, 1e-300, 0.99999999]
    conf += [j / 32 for j in range(33)] + rng.random(2000).tolist() + (rng.random(300) ** 8).tolist()
    R = len(conf)
    qn = [f"q{i}" for i in range(R)]
    pool = "".join(qn).encode()
    off = np.zeros(R + 1, np.int64)
    np.cumsum([len(x) for x in qn], out=off[1:])

    def dev(a):
        return torch.from_numpy(np.ascontiguousarray(a)).to(gpu.dev)

    names = np.full((R, 8), -1, np.int32)
    names[:, 0] = 0
    d = {"q": dev(np.arange(R, dtype=np.int32)), "depth": dev(np.ones(R, np.int32)), "names": dev(names.reshape(-1)),
         "conf": dev(np.array(conf, np.float64)), "tax": dev(np.zeros(R, np.int32))}
    lab, lab_off = dev(np.frombuffer(b"Bacteria", np.uint8).copy()), dev(np.array([0, 8], np.int64))
    out = gpu.empty(1 << 20, torch.uint8)
    nb = ctypes.c_int64()
    d_pool, d_off = dev(np.frombuffer(pool, np.uint8).copy()), dev(off)   # kept alive across the call
    gpu.call("hymet_emit_tsv", 0, R, ptr(d["q"]), ptr(d["depth"]), ptr(d["names"]), ptr(d["conf"]), ptr(d["tax"]),
             ptr(d_pool), ptr(d_off), ptr(lab), ptr(lab_off), None, None, None, None, ptr(out), 1 << 20, ctypes.byref(nb))
    got = out[:nb.value].cpu().numpy().tobytes()
    buf = io.StringIO(newline="")
    wr = csv.writer(buf, delimiter="\t")
    wr.writerows([q, "superkingdom:Bacteria", "superkingdom", f"{c:.4f}"] for q, c in zip(qn, conf))
    assert got == buf.getvalue().encode()


def _world2_worker(rank, port, data_path, msh_path, tax, hier, q, db_gather="loader"):
    import os
    import traceback
    try:
        os.environ["HYMET_DB_GATHER"] = db_gather
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        from hymet_amd import pipeline
        from hymet_amd._lib import Gpu
        from hymet_amd.dist import Comm
        gpu = Gpu(0)
        comm = Comm(rank, 2).init_backend(gpu, "gloo")
        w, db, by_name = _w2_setup(gpu)
        from hymet_amd.seqio import from_records
        # the DB by path, re-read every run: run 2 loads one slice of its hashes per rank and
        # all-gathers the other (Pipeline._join_slices)
        p = pipeline.Pipeline(gpu, [msh_path], lambda ns: from_records([(by_name[n][0], "", by_name[n][1]) for n in ns]),
                              tax, hier, pipeline.Config(map_batch_bases=300_000, map_streams=2, reload_inputs=True), comm)
        data = open(data_path, "rb").read()
        out = []
        for _ in range(2):
            res = p.run(data, with_paf=True)
            out.append((res.tsv, res.paf_bytes, res.selected))
        sliced = p.timings.get("msh_allgather_s") is not None
        comm.close()
        q.put((rank, "ok", (out, sliced)))
    except Exception:
        q.put((rank, "err", traceback.format_exc()))


def _w2_setup(gpu):
    import tempfile
    from pathlib import Path
    w, db, by_name, _, _ = _setup(gpu, Path(tempfile.mkdtemp()))
    return w, db, by_name


def _world2_input(w, shape):
    """FASTA bytes for the world-2 test.  halves: the 60 contigs (the byte cut lands mid-file,
    both ranks get records).  one_record: a single contig (rank 0's byte range is the whole
    file, rank 1's is empty).  big_last: the contigs and then one record longer than all of
    them together -- two candidate genomes joined -- so the cut at len/2 falls inside it and
    rank 0 again takes every record.  The last two are the shapes where a rank-local test of
    the byte range would send the ranks down different collective paths."""
    if shape == "halves":
        return _fasta_text(w, quote_name=False)
    if shape == "one_record":
        i = int(np.argmax([len(s) for s in w.contigs]))
        return b">" + w.contig_names[i].encode() + b" len=" + str(len(w.contigs[i])).encode() + b"\n" + w.contigs[i] + b"\n"
    if shape == "big_last":
        big = w.refs[0] + w.refs[1]
        assert len(big) > sum(len(s) for s in w.contigs)
        return _fasta_text(w, quote_name=False) + b">chimera_0_1\n" + big + b"\n"
    raise ValueError(shape)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("db_gather,shape", [("loader", "halves"), ("main", "halves"), ("loader", "one_record"),
                                             ("loader", "big_last")])
def test_world2_pipeline_equals_world1(gpu, tmp_path, db_gather, shape):
    """Two ranks (two processes on this GPU, gloo staging the collectives through the host):
    each takes its byte range of the same FASTA; rank 0's TSV equals the one-rank TSV and
    the ranks' PAF texts concatenate to the one-rank PAF (one index part).  The ranks read the
    DB from its .msh path on every run; the second run loads it as per-rank hash slices
    all-gathered between the ranks (the loader thread holding the communicator), and must give
    the same bytes.  One-record and big-last-record inputs leave rank 1 with no records."""
    from hymet_amd.msh import write_msh
    import multiprocessing as mpc
    import socket
    from hymet_amd import pipeline
    from hymet_amd.ingest import shard_bytes
    from hymet_amd.seqio import from_records
    w, db, by_name, tax, hier = _setup(gpu, tmp_path)
    data = _world2_input(w, shape)
    if shape != "halves":
        assert shard_bytes(data, 0, 2) == (0, len(data)) and shard_bytes(data, 1, 2) == (len(data), len(data))
    dp = tmp_path / "pool.fna"
    dp.write_bytes(data)
    mp_ = tmp_path / "sketch.msh"
    write_msh(db, str(mp_))
    p = pipeline.Pipeline(gpu, [db], lambda ns: from_records([(by_name[n][0], "", by_name[n][1]) for n in ns]),
                          str(tax), str(hier), pipeline.Config(map_batch_bases=300_000))
    one = p.run(data, with_paf=True)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mpc.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_world2_worker, args=(r, port, str(dp), str(mp_), str(tax), str(hier), q, db_gather)) for r in range(2)]
    for x in ps:
        x.start()
    got = {}
    for _ in range(2):
        r, st, out = q.get(timeout=240)
        assert st == "ok", out
        got[r] = out
    for x in ps:
        x.join(timeout=60)
    assert got[0][1] and got[1][1]           # run 2 took the sliced DB load on both ranks
    for k in range(2):
        r0, r1 = got[0][0][k], got[1][0][k]
        assert r0[2] == one.selected == r1[2]
        assert r0[0] == one.tsv
        assert r1[0] == b""
        assert r0[1] + r1[1] == one.paf_bytes
    assert one.n_queries >= 1


def test_map_streams_one_and_two_identical(gpu, tmp_path):
    """The default two-stream mapping (worker contexts, per-worker accumulators re-ordered
    part-major by hymet_paf_acc_append) must give the same PAF and TSV bytes as one stream,
    on an input of several index parts and several query batches per worker."""
    from hymet_amd import pipeline
    from hymet_amd.seqio import from_records
    w, db, by_name, tax, hier = _setup(gpu, tmp_path)

    def ref_lookup(names):
        return from_records([(by_name[n][0], "", by_name[n][1]) for n in names])

    queries = from_records([(n, "", s) for n, s in zip(w.contig_names, w.contigs)])
    out = {}
    for ms in (1, 2):
        cfg = pipeline.Config(split_idx="2m", index_mini_batch=1e6, map_batch_bases=60_000, map_streams=ms)
        p = pipeline.Pipeline(gpu, [db], ref_lookup, tax, hier, cfg)
        res = p.run(queries, with_paf=True)
        assert len(p.index_for(res.selected).parts) >= 2
        out[ms] = res
    assert out[1].selected == out[2].selected
    assert out[1].paf == out[2].paf
    assert out[1].tsv == out[2].tsv
    assert len(out[1].paf) > 50


def test_msh_pipeline_three_runs_keep_results(gpu, tmp_path):
    """The bench's own configuration on a small input: a Pipeline built from .msh PATHS
    (reload_inputs: every run re-parses the DB files on the loader thread and builds the
    screen tables on the idle mapping stream), two mapping streams, FASTA bytes in, PAF text
    in the alternating pinned buffers.  Run three times while the FIRST result's PAF text is
    still referenced: its bytes must survive runs 2 and 3 (copy-on-reuse), and every run's
    screen arrays, PAF and TSV must equal the first run's."""
    from hymet_amd import pipeline
    from hymet_amd.msh import write_msh
    from hymet_amd.seqio import from_records
    w, db, by_name, tax, hier = _setup(gpu, tmp_path)
    msh = tmp_path / "sketch1.msh"
    write_msh(db, str(msh))
    data = _fasta_text(w, quote_name=False)

    def ref_lookup(names):
        return from_records([(by_name[n][0], "", by_name[n][1]) for n in names])

    cfg = pipeline.Config(map_batch_bases=200_000, map_streams=2, reload_inputs=True)
    p = pipeline.Pipeline(gpu, [str(msh)], ref_lookup, str(tax), str(hier), cfg)
    first = p.run(data, with_paf=True)
    first_view = first.paf_text.view()      # zero-copy while `first` is alive
    first_copy = bytes(first_view)
    sh0 = [r.shared.copy() for r in first.screen]
    md0 = [r.median.copy() for r in first.screen]
    assert len(first_copy) > 1000 and first.tsv.count(b"\r\n") > 50
    for _ in range(2):
        r = p.run(data, with_paf=True)
        assert r.paf_bytes == first_copy
        assert r.tsv == first.tsv and r.selected == first.selected
        for a, b, res in zip(sh0, md0, r.screen):
            np.testing.assert_array_equal(res.shared, a)
            np.testing.assert_array_equal(res.median, b)
        assert first.paf_bytes == first_copy       # the held result was copied out before reuse

"""Stage drop-ins under scripts/ (SURVEY.md §8b): argv, output files, stdout and exit codes.

CPU: scripts/limit_candidates.py run as a subprocess against the reference-generated goldens
(output bytes, stdout, rc); every wrapper script reaches its subcommand (usage errors).
GPU: the screen / map / classify subcommands behind scripts/mash.sh, scripts/minimap2.sh and
scripts/classification*.py, called in-process (the test process already holds the GPU) on
small inputs and compared with the oracle."""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
SCRIPTS = ROOT / "scripts"
LIM = ROOT / "tests" / "golden" / "limit"
LCASES = json.loads((LIM / "cases.json").read_text())


def _run(args, timeout=240, **kw):
    env = dict(os.environ)
    env.pop("PYTHONPATH", None)
    try:
        return subprocess.run(args, capture_output=True, text=True, env=env, timeout=timeout, **kw)
    except subprocess.TimeoutExpired as e:
        raise AssertionError(f"{args[:3]} timed out; stdout={e.stdout!r} stderr={e.stderr!r}") from None


@pytest.mark.parametrize("case", LCASES, ids=[Path(c["expect"]).stem for c in LCASES])
def test_limit_dropin_matches_reference(case, tmp_path):
    out = tmp_path / "limited.txt"
    args = [sys.executable, str(SCRIPTS / "limit_candidates.py"), "--selected", str(LIM / "selected.txt"),
            "--output", str(out), "--max", str(case["max"])]
    for t in case["tabs"]:
        args += ["--score-file", str(LIM / t)]
    if case["dedupe"]:
        args += ["--dedupe", "--no-download", "--assembly-dir", str(tmp_path / "none")]
    r = _run(args)
    assert r.returncode == case["rc"], r.stderr
    assert r.stdout == case["stdout"]
    assert out.read_bytes() == (LIM / case["expect"]).read_bytes()


def test_limit_dropin_errors(tmp_path):
    empty = tmp_path / "empty.txt"
    empty.write_text("\n")
    r = _run([sys.executable, str(SCRIPTS / "limit_candidates.py"), "--selected", str(empty), "--output",
              str(tmp_path / "o")])
    assert r.returncode != 0 and "No candidates found" in r.stderr
    r = _run([sys.executable, str(SCRIPTS / "limit_candidates.py"), "--selected", str(LIM / "selected.txt"),
              "--output", str(tmp_path / "o"), "--max", "0"])
    assert r.returncode != 0 and "--max value must be greater than zero" in r.stderr


def test_limit_dropin_log_append(tmp_path):
    log = tmp_path / "logs" / "limit.log"
    for _ in range(2):
        r = _run([sys.executable, str(SCRIPTS / "limit_candidates.py"), "--selected", str(LIM / "selected.txt"),
                  "--output", str(tmp_path / "o"), "--max", "3", "--log", str(log)])
        assert r.returncode == 0
    assert log.read_text().splitlines() == [r.stdout.rstrip("\n")] * 2


@pytest.mark.parametrize("script", ["mash.sh", "minimap2.sh"])
def test_shell_wrappers_reach_subcommand(script, tmp_path):
    r = _run(["bash", str(SCRIPTS / script), "only-one-arg"])
    assert r.returncode == 2 and "usage:" in r.stderr


@pytest.mark.parametrize("script", ["classification_cami.py", "classification.py"])
def test_python_wrappers_reach_subcommand(script):
    r = _run([sys.executable, str(SCRIPTS / script), "--paf", "x"])
    assert r.returncode == 2 and "--taxonomy" in r.stderr


# ---------------------------------------------------------------------------- GPU
def _fasta(path, recs):
    with open(path, "w") as f:
        for n, s in recs:
            f.write(f">{n}\n")
            for i in range(0, len(s), 80):
                f.write(s[i:i + 80].decode() + "\n")


@pytest.mark.gpu
def test_screen_map_classify_dropins_match_oracle(tmp_path, capsys):
    from hymet_amd.cli import main as cli
    from hymet_amd import synth
    from hymet_amd.msh import SketchDB, write_msh
    from oracle import classify_oracle, oracle_lib, pipeline_oracle, select_oracle
    rng = np.random.default_rng(11)
    w = synth.make_cami(rng, n_taxa=2, per_taxon=3, genome_mbp=(0.2, 0.3), contig_gbp=0.0002, max_contigs=20,
                        name="dropin")
    hl = [np.sort(oracle_lib.sketch([r], 21, 42, 1000)) for r in w.refs]
    hl += list(synth.decoy_sketches(rng, 10, 1000))
    names = [n + ".fna.gz" for n in w.ref_names] + [f"decoy_{i}.fna.gz" for i in range(len(hl) - len(w.refs))]
    off = np.zeros(len(hl) + 1, np.int64)
    off[1:] = np.cumsum([len(h) for h in hl])
    db = SketchDB(names=names, comments=[f"[1 seqs] {n}" for n in names], lengths=np.full(len(hl), 250_000, np.int64),
                  offsets=off, hashes=np.concatenate(hl))
    msh = tmp_path / "sketch1.msh"
    write_msh(db, msh)
    inp = tmp_path / "input"
    inp.mkdir()
    recs = list(zip(w.contig_names, w.contigs))
    _fasta(inp / "contigs.fna", recs)
    # ---- mash.sh
    outs = [tmp_path / f for f in ("screen.tab", "filtered.tab", "sorted.tab", "top_hits.tab", "selected.txt")]
    assert cli(["screen", str(inp), str(msh)] + [str(o) for o in outs] + ["0.90"]) == 0
    stdout = capsys.readouterr().out
    rows = pipeline_oracle.screen_rows([s for _, s in recs], db)
    assert outs[0].read_text().splitlines() == rows
    srt = select_oracle.sort_gr(select_oracle.sort_unique_k5(rows))
    assert outs[2].read_text().splitlines() == srt
    t, top, sel_names, _ = select_oracle.select_threshold(srt, "0.90", 1)
    assert outs[3].read_text().splitlines() == top
    assert outs[4].read_text().splitlines() == sel_names
    assert f"Final threshold used: {t}" in stdout
    # ---- minimap2.sh over the selected genomes
    by_name = {n + ".fna.gz": (n, s) for n, s in zip(w.ref_names, w.refs)}
    chosen = [by_name[n] for n in sel_names if n in by_name]
    assert chosen
    ref_fa = tmp_path / "combined_genomes.fasta"
    _fasta(ref_fa, chosen)
    paf = tmp_path / "resultados.paf"
    mmi = tmp_path / "reference.mmi"
    assert cli(["map", str(inp), str(ref_fa), str(mmi), str(paf)]) == 0
    assert "Creating index with minimap2..." in capsys.readouterr().out and mmi.stat().st_size > 0
    o_paf = pipeline_oracle.map_paf([n for n, _ in chosen], [s for _, s in chosen], recs)
    assert paf.read_text().splitlines() == o_paf
    assert (tmp_path / "reference.mmi.hymet").stat().st_size > 0
    # warm call: the persisted device index is loaded; like minimap2 with a prebuilt .mmi it
    # never reads the reference FASTA again (moved away here)
    ref_fa.rename(tmp_path / "moved.fasta")
    assert cli(["map", str(inp), str(ref_fa), str(mmi), str(paf)]) == 0
    assert "Using cached minimap2 index" in capsys.readouterr().out
    assert paf.read_text().splitlines() == o_paf
    (tmp_path / "moved.fasta").rename(ref_fa)
    # ---- classification_cami.py / classification.py
    tax = tmp_path / "detailed_taxonomy.tsv"
    tax.write_text(w.taxonomy_tsv())
    hier = tmp_path / "taxonomy_hierarchy.tsv"
    hier.write_text(w.hierarchy_tsv())
    for sub, fn in (("classify", classify_oracle.classify_cami), ("classify-legacy", classify_oracle.classify_legacy)):
        out = tmp_path / f"{sub}.tsv"
        assert cli([sub, "--paf", str(paf), "--taxonomy", str(tax), "--hierarchy", str(hier), "--output", str(out),
                    "--processes", "2"]) == 0
        assert out.read_bytes() == fn(str(paf), str(tax), str(hier))


@pytest.mark.gpu
def test_persisted_multipart_index_round_trip(tmp_path, capsys, monkeypatch):
    """SPLIT_IDX small enough for three -I parts: the persisted parts reload to the same
    PAF as the fresh build and as the oracle (minimap2 -I300k -d ; -x asm10)."""
    from hymet_amd.cli import main as cli
    from hymet_amd import synth
    from oracle import pipeline_oracle
    w = synth.make_cami(np.random.default_rng(31), n_taxa=3, per_taxon=2, genome_mbp=(0.15, 0.25), contig_gbp=0.0003,
                        max_contigs=30, name="parts")
    inp = tmp_path / "input"
    inp.mkdir()
    recs = list(zip(w.contig_names, w.contigs))
    _fasta(inp / "a.fna", recs[:12])
    _fasta(inp / "b.fna", recs[12:])
    chosen = list(zip(w.ref_names, w.refs))
    ref_fa = tmp_path / "combined_genomes.fasta"
    _fasta(ref_fa, chosen)
    monkeypatch.setenv("SPLIT_IDX", "300k")
    monkeypatch.setenv("HYMET_INDEX_MINI_BATCH", "1e5")
    paf, mmi = tmp_path / "resultados.paf", tmp_path / "reference.mmi"
    assert cli(["map", str(inp), str(ref_fa), str(mmi), str(paf)]) == 0
    cold = paf.read_bytes()
    assert cli(["map", str(inp), str(ref_fa), str(mmi), str(paf)]) == 0
    assert "Using cached minimap2 index" in capsys.readouterr().out
    assert paf.read_bytes() == cold
    o_paf = pipeline_oracle.map_paf([n for n, _ in chosen], [s for _, s in chosen], recs, part_bases=3e5, mini_batch=1e5)
    assert cold.decode().splitlines() == o_paf
    import json
    assert len(json.loads(mmi.read_text())["part_offsets"]) >= 3

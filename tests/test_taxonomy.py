"""§8(f) rows 1 and 3: the taxonomy_hierarchy.tsv builder and the hymet2cami CAMI export,
against goldens the reference scripts generated (tests/golden/make_taxonomy_goldens.py):
scripts/taxonomy_hierarchy.py on a synthetic taxdump with its edge cases, and
tools/hymet2cami.py's own logic (lineage parsing, per-rank counts, ordering, '%.6f') given
fixed taxonkit answers.  The taxonkit restatement itself is parity-unpinned (taxonkit is
absent from the image); it is checked for consistency with those answers."""
import json
import subprocess
import sys
from pathlib import Path

from hymet_amd import taxonomy as tx

G = Path(__file__).resolve().parent / "golden" / "taxonomy"
ROOT = Path(__file__).resolve().parents[1]


def test_hierarchy_builder_matches_reference():
    assert tx.hierarchy_tsv(str(G / "names.dmp"), str(G / "nodes.dmp")) == (G / "expect_hierarchy.tsv").read_bytes()


def test_cami_profile_logic_matches_reference():
    inp = json.loads((G / "cami_inputs.json").read_text())
    recs = tx.load_records((G / "classified.tsv").read_text())
    t2p = {k: tuple(v) for k, v in inp["taxid2path"].items()}
    assert tx.cami_profile(recs, inp["name2taxid"], t2p) == (G / "expect_cami.txt").read_text()


def test_taxonkit_restatement_consistent_with_fixture_answers():
    inp = json.loads((G / "cami_inputs.json").read_text())
    d = tx.TaxDump(str(G / "names.dmp"), str(G / "nodes.dmp"), all_names=True)
    recs = tx.load_records((G / "classified.tsv").read_text())
    names = {n for p in recs for n in p.values() if n}
    n2t = tx.name2taxid(d, names)
    assert n2t == inp["name2taxid"]
    assert tx.name2taxid(d, ["bacillus SUBTILIS"]) == {"bacillus SUBTILIS": "1423"}   # case-insensitive
    t2p = tx.reformat(d, sorted(set(n2t.values())))
    assert {k: list(v) for k, v in t2p.items()} == inp["taxid2path"]


def test_hymet2cami_dropin(tmp_path):
    r = subprocess.run([sys.executable, str(ROOT / "scripts" / "hymet2cami.py"), str(G / "classified.tsv")],
                       capture_output=True, text=True, env={"TAXONKIT_DB": str(G), "PATH": "/usr/bin:/bin"})
    assert r.returncode == 0, r.stderr
    assert r.stdout == (G / "expect_cami.txt").read_text()
    assert "[hymet2cami] parsed 8 lineages" in r.stderr and "[hymet2cami] done" in r.stderr


def test_taxonomy_hierarchy_dropin(tmp_path):
    (tmp_path / "taxonomy_files").mkdir()
    for f in ("names.dmp", "nodes.dmp"):
        (tmp_path / "taxonomy_files" / f).write_bytes((G / f).read_bytes())
    r = subprocess.run([sys.executable, str(ROOT / "scripts" / "taxonomy_hierarchy.py")], cwd=tmp_path,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "data" / "taxonomy_hierarchy.tsv").read_bytes() == (G / "expect_hierarchy.tsv").read_bytes()
    assert "File generated successfully" in r.stdout

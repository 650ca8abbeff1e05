"""tools/eval_cami.py restated (hymet_amd/evaluate.py).

Parity unpinned: the reference ships no fixtures for eval_cami and depends on taxonkit, which
is absent; running the reference here was refused.  The expected metrics
below are computed by hand from eval_cami.py's formulas (:369-385, :530-547) on the
synthetic taxdump of tests/golden/taxonomy (Bacillus subtilis 1423 under domain 2,
Escherichia coli 562 / genus 561, Methanobrevibacter smithii 2173 under superkingdom 2157).
"""
import os
import subprocess
import sys

import pytest

from hymet_amd import evaluate as ev

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TAXDB = os.path.join(REPO, "tests", "golden", "taxonomy")

CLASSIFIED = ("Query\tLineage\tTaxonomic Level\tConfidence\r\n"
              "c1\tsuperkingdom:Bacteria; species:Bacillus subtilis\tspecies\t0.9\r\n"
              "c2\tdomain:Bacteria;g:Escherichia\tgenus\t0.8\r\n"
              "c3\tUnknown\troot\t0.0\r\n"
              "c4\tspecies:Nomen nudum\tspecies\t0.3\r\n")
PAF = ("c3\t100\t0\t100\t+\tNC_000913.3\t4641652\t10\t110\t100\t100\t60\n"
       "c3\t100\t0\t100\t+\tNC_000964.3\t4215606\t10\t110\t90\t100\t0\n")
TAXMAP = "GCF\tTaxID\tIdentifiers\nGCF_000005845.2\t562\tNC_000913.3\nGCF_000009045.1\t1423\tNC_000964.3;NZ_PLASMID1.1\n"
GSA = ("#anonymous_contig_id\tgenome_id\ttax_id\tcontig_id\n"
       "c1\tg1\t1423\tx1\nc2\tg2\t562\tx2\nc3\tg2\t562\tx3\nc4\tg3\t2173\tx4\n")
PRED_PROFILE = ("@SampleID:x\n@@TAXID\tRANK\tTAXPATH\tTAXPATHSN\tPERCENTAGE\n"
                "2\tsuperkingdom\t2\tBacteria\t100.0\n"
                "1423\tspecies\t2|1239|91061|1385|186817|1386|1423\tBacteria|...\t60.0\n"
                "562\tspecies\t2|1224|1236|91347|543|561|562\tBacteria|...\t40.0\n")
TRUTH_PROFILE = ("@@TAXID\tRANK\tTAXPATH\tTAXPATHSN\tPERCENTAGE\n"
                 "2\tsuperkingdom\t2\tBacteria\t70\n2157\tsuperkingdom\t2157\tArchaea\t30\n"
                 "1423\tspecies\t.\t.\t50\n2173\tspecies\t.\t.\t50\n")


@pytest.fixture
def files(tmp_path):
    p = {}
    for name, text in (("classified.tsv", CLASSIFIED), ("resultados.paf", PAF), ("taxmap.tsv", TAXMAP),
                       ("gsa.tsv", GSA), ("pred.cami", PRED_PROFILE), ("truth.cami", TRUTH_PROFILE)):
        (tmp_path / name).write_text(text)
        p[name] = str(tmp_path / name)
    p["out"] = str(tmp_path / "eval")
    return p


def test_metrics_by_hand():
    assert ev.l1_and_braycurtis({"a": 60, "b": 40}, {"a": 50, "c": 50}) == (50.0, 50.0)
    l1, bc = ev.l1_and_braycurtis({"2": 100.0}, {"2": 70.0, "2157": 30.0})
    assert l1 == 30.0 and abs(bc - 30.0) < 1e-12
    assert ev.prf_presence({"2": 100.0}, {"2": 70.0, "2157": 30.0}) == (100.0, 50.0, pytest.approx(66.6666666), 1, 0, 1)
    assert ev.l1_and_braycurtis({}, {}) == (0.0, 0.0)
    assert ev.parse_lineage_string("sk:Bacteria; strain:X y; bogus:1; s:") == {"superkingdom": "Bacteria", "species": "X y"}
    assert ev.normalize_taxid("taxid:562.1") == "562" and not ev.is_num("1e5") and ev.is_num("12.5")


def test_contig_resolution(files):
    tax = ev.Taxonomy(TAXDB)
    idmap = ev.load_id_map(files["taxmap.tsv"])
    assert idmap["NC_000913"] == "562" and idmap["GCF_000009045"] == "1423"
    got = ev.preds_taxid_from_classified(files["classified.tsv"], tax, idmap, files["resultados.paf"])
    # c1: species name; c2: genus name; c3: first PAF hit through the id map; c4: unknown name
    assert got == {"c1": "1423", "c2": "561", "c3": "562"}
    assert ev.load_gt_contigs(files["gsa.tsv"]) == {"c1": "1423", "c2": "562", "c3": "562", "c4": "2173"}


def test_main_outputs(files, capsys):
    rc = ev.main(["--pred-profile", files["pred.cami"], "--truth-profile", files["truth.cami"],
                  "--pred-contigs", files["classified.tsv"], "--truth-contigs", files["gsa.tsv"],
                  "--pred-fasta", "", "--truth-fasta", "", "--taxdb", TAXDB, "--taxmap", files["taxmap.tsv"],
                  "--paf", files["resultados.paf"], "--outdir", files["out"]])
    assert rc == 0
    out = capsys.readouterr().out
    summary = open(os.path.join(files["out"], "profile_summary.tsv")).read().splitlines()
    assert summary[0].split("\t")[:3] == ["rank", "L1_total_variation_pctpts", "BrayCurtis_pct"]
    rows = {r.split("\t")[0]: r.split("\t")[1:] for r in summary[1:]}
    assert rows["superkingdom"] == ["30.0000", "30.0000", "100.00", "50.00", "66.67", "1", "0", "1"]
    assert rows["species"] == ["50.0000", "50.0000", "50.00", "50.00", "50.00", "1", "1", "1"]
    assert rows["genus"] == ["0.0000", "0.0000", "0.00", "0.00", "0.00", "0", "0", "0"]
    # contigs: pairs c1 (1423/1423), c2 (561/562), c3 (562/562); 561 has no species id
    exact = open(os.path.join(files["out"], "contigs_exact.tsv")).read().splitlines()
    assert exact[1:3] == ["usable_pairs\t3", "exact_taxid_matches\t2"]
    per = {r.split("\t")[0]: r.split("\t")[1:] for r in open(os.path.join(files["out"], "contigs_per_rank.tsv")).read().splitlines()[1:]}
    assert per["genus"] == ["3", "3", "100.0000"] and per["species"] == ["3", "2", "66.6667"]
    assert per["superkingdom"] == ["3", "3", "100.0000"]
    assert "Exact TaxID: 2/3 (66.67%)" in out
    assert "superkingdom    L1=30.000  BC=30.000%  P/R/F1=100.0/50.0/66.7% (TP=1, FP=0, FN=1)" in out


def test_profile_rebuilt_from_contigs(files):
    """No usable profiles: both are rebuilt from contig TaxIDs weighted by FASTA length."""
    fa = os.path.join(os.path.dirname(files["out"]), "contigs.fna")
    with open(fa, "w") as f:
        f.write(">c1\nACGT\nAC\n>c2\nAAAA\n>c3\nAA\n>c4\nA\n")
    out = files["out"]
    rc = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "eval_cami.py"), "--pred-profile", "/nonexistent",
                         "--truth-profile", "/nonexistent", "--pred-contigs", files["classified.tsv"],
                         "--truth-contigs", files["gsa.tsv"], "--pred-fasta", fa, "--truth-fasta", "",
                         "--taxdb", TAXDB, "--taxmap", files["taxmap.tsv"], "--paf", files["resultados.paf"],
                         "--outdir", out], capture_output=True, text=True)
    assert rc.returncode == 0, rc.stderr
    rows = {r.split("\t")[0]: r.split("\t")[1:] for r in open(os.path.join(out, "profile_summary.tsv")).read().splitlines()[1:]}
    # pred species weights: c1 6 bp -> 1423, c3 2 bp -> 562 (c2's 561 has an empty species id,
    # counted under '' as the reference does); truth: 1423 6, 562 4 + 2, 2173 1
    pred = {"1423": 6, "": 4, "562": 2}
    truth = {"1423": 6, "562": 6, "2173": 1}
    a = {k: 100.0 * v / 12 for k, v in pred.items()}
    b = {k: 100.0 * v / 13 for k, v in truth.items()}
    l1, bc = ev.l1_and_braycurtis(a, b)
    assert rows["species"][:2] == [f"{l1:.4f}", f"{bc:.4f}"]

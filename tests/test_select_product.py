"""hymet_amd.select (product host code) vs the reference-pinned goldens and the oracle."""
import json
import random
from pathlib import Path

import pytest

from hymet_amd import select as sel
from oracle import select_oracle as so

LIM = Path(__file__).resolve().parent / "golden" / "limit"
LCASES = json.loads((LIM / "cases.json").read_text())


@pytest.mark.parametrize("case", LCASES, ids=[Path(c["expect"]).stem for c in LCASES])
def test_limit_matches_reference_goldens(case):
    names = [l.strip() for l in (LIM / "selected.txt").read_text().splitlines() if l.strip()]
    scores = sel.read_scores([str(LIM / t) for t in case["tabs"]])
    got = sel.limit(names, scores, case["max"], dedupe=case["dedupe"])
    assert ("".join(n + "\n" for n in got)).encode() == (LIM / case["expect"]).read_bytes()


def _rows(rng, n):
    rows = []
    for i in range(n):
        ident = rng.choice(["1", "0.95", "0.9", "0.899999", "%g" % rng.random(), "0.88", "0.7", "0.71", "0.69"])
        name = rng.choice([f"GCF_{rng.randrange(50):06d}.1_x", "plain", "zz", "A b"])
        rows.append(f"{ident}\t{rng.randrange(1000)}/1000\t{rng.randrange(9)}\t{rng.random():g}\t{name}\t[1 seqs] c {i}")
    return rows


def test_selection_text_stages_match_oracle():
    rng = random.Random(5)
    for trial in range(300):
        rows = _rows(rng, rng.randrange(0, 40))
        a = sel.sort_gr(sel.sort_unique_k5(rows))
        b = so.sort_gr(so.sort_unique_k5(rows))
        assert a == b
        init = rng.choice(["0.9", "0.90", "0.8", "0.95"])
        nf = rng.randrange(1, 4)
        t1, top1, n1, log1 = sel.threshold_walk(a, init, nf)
        t2, top2, n2, trace = so.select_threshold(b, init, nf)
        assert (t1, top1, n1) == (t2, top2, n2)
        # mash.sh's stdout from the walk on: one Testing/Candidates pair per threshold tried
        # (:35-36), the fallback note (:50), the summary (:57-60)
        exp = [l for t, c in trace for l in (f"Testing threshold: {t}", f"Candidates found: {c}")]
        found = bool(trace) and trace[-1][1] >= sel.min_candidates(nf)
        if not found:
            exp.append("No suitable threshold found. Using 0.70.")
        exp += ["=" * 36, f"Final threshold used: {t2}", f"Candidates found: {trace[-1][1] if found else len(top2)}", "=" * 36]
        assert log1 == exp
    assert sel.union_sorted(["b", "a"], ["B"]) == so.union_sorted(["b", "a"], ["B"])


def test_threshold_walk_log_known_answer():
    """scripts/mash.sh:32-60 on a table where 0.90 and 0.88 fail and .86 succeeds (bc prints .88)."""
    rows = [f"0.87{i}\t900/1000\t1\t0\tG{i}\tc" for i in range(5)] + ["0.95\t990/1000\t3\t0\tTOP\tc"]
    best, top, names, log = sel.threshold_walk(sel.sort_gr(rows), "0.9", 1)
    assert best == ".86" and len(top) == 6 and names[0] == "TOP"
    assert log[:6] == ["Testing threshold: 0.9", "Candidates found: 1", "Testing threshold: .88", "Candidates found: 1",
                       "Testing threshold: .86", "Candidates found: 6"]
    assert log[-3:-1] == ["Final threshold used: .86", "Candidates found: 6"]
    best, top, _, log = sel.threshold_walk(rows[:2], "0.9", 1)
    assert best == "0.71" and "No suitable threshold found. Using 0.70." in log and log[-2] == "Candidates found: 2"


def _summary_rows(rows):
    return "".join("\t".join(r) + "\n" for r in rows)


def test_species_dedupe_from_local_assembly_summaries(tmp_path):
    """limit_candidates.py:163-185 + 198-233 with real-shaped assembly_summary files
    (hand-derived expectations): the species key is species_taxid (column 6), else taxid
    (column 5), else the accession; rows with fewer than 8 columns and '#' lines are
    skipped; genbank is read after refseq, so its row for an accession wins; candidates are
    keyed by the accession part of the file name (GCF_x.y) and the best-scoring one per
    species is kept."""
    from hymet_amd import cli
    from hymet_amd import select as sel
    head = "#   See ftp://ftp.ncbi.nlm.nih.gov/genomes/README_assembly_summary.txt\n"
    cols = ["#assembly_accession", "bioproject", "biosample", "wgs_master", "refseq_category", "taxid",
            "species_taxid", "organism_name", "infraspecific_name"]
    acc = [f"GCF_00000000{i}.1" for i in range(1, 7)]
    (tmp_path / "assembly_summary_refseq.txt").write_text(
        head + _summary_rows([cols,
        [acc[0], "P1", "S1", "", "reference genome", "511145", "562", "Escherichia coli K-12", "x"],
        [acc[1], "P2", "S2", "", "na", "562", "", "Escherichia coli", "x"],            # species_taxid empty -> taxid
        [acc[2], "P3", "S3", "", "na", "93061", "1280", "Staphylococcus aureus", "x"],
        [acc[3], "P4", "S4", "", "na"],                                                # < 8 columns: skipped
        [acc[4], "P5", "S5", "", "na", "", "", "", "x"],                               # no ids: keyed by accession
        [acc[5], "P6", "S6", "", "na", "158878", "1280", "Staphylococcus aureus Mu50", "x"]]))
    (tmp_path / "assembly_summary_genbank.txt").write_text(_summary_rows([
        [acc[2], "P3", "S3", "", "na", "224308", "1423", "Bacillus subtilis 168", "x"]]))   # read last: wins
    smap = sel.species_map(str(tmp_path))
    assert smap[acc[0]] == ("562", "Escherichia coli K-12")
    assert smap[acc[1]] == ("562", "Escherichia coli")
    assert smap[acc[2]] == ("1423", "Bacillus subtilis 168")
    assert acc[3] not in smap
    assert smap[acc[4]] == (acc[4], acc[4])
    names = [f"{a}_ASM{i}v1_genomic.fna.gz" for i, a in enumerate(acc)]
    scores = dict(zip(names, [0.95, 0.99, 0.97, 0.96, 0.93, 0.98]))
    # score order: acc2 (562), acc6 (1280), acc3 (1423), acc4 (its accession), acc1 (562: dup), acc5
    assert sel.limit(names, scores, 10, True, smap) == [names[1], names[5], names[2], names[3], names[4]]
    assert sel.limit(names, scores, 3, True, smap) == [names[1], names[5], names[2]]
    assert sel.limit(names, scores, 10, False, smap) == [names[i] for i in (1, 5, 2, 3, 0, 4)]
    # without the genbank row acc3 is S. aureus (1280) again and loses to acc6
    (tmp_path / "assembly_summary_genbank.txt").unlink()
    assert sel.limit(names, scores, 10, True, sel.species_map(str(tmp_path))) == [names[1], names[5], names[3], names[4]]
    # the drop-in CLI end to end
    selected = tmp_path / "selected_genomes.txt"
    selected.write_text("".join(n + "\n" for n in names))
    tab = tmp_path / "screen.tab"
    tab.write_text("".join(f"{scores[n]}\t1/1000\t1\t0\t{n}\t[1 seqs]\n" for n in names))
    out = tmp_path / "limited.txt"
    assert cli.cmd_limit(["--selected", str(selected), "--output", str(out), "--score-file", str(tab), "--dedupe",
                          "--assembly-dir", str(tmp_path), "--max", "10"]) == 0
    assert out.read_text().split() == [names[1], names[5], names[3], names[4]]

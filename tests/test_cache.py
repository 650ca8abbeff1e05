"""Offline reference-cache builder (hymet_amd/cache.py) against
scripts/downloadDB.py:78-222.

Parity unpinned: the reference ships no fixtures for this stage and running its class here
was refused, so the expected files below are derived by hand from
downloadDB.py's code on a small synthetic genome directory.  Compared modulo the orders the
reference takes from Python sets and os.listdir (rows, identifiers, genome concatenation).
"""
import os
import subprocess
import sys

import pytest

from hymet_amd import cache

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

GENOMES = {
    "GCF_000005845.2_ASM584v2_genomic.fna": ">NC_000913.3 Escherichia coli K-12\nACGTACGTAC\nGGTT\n",
    "GCF_000009045.1_ASM904v1_genomic.fna": ">NC_000964.3 Bacillus subtilis 168\nTTGACA\n>NZ_PLASMID1.1 plasmid\nGGGCCC\n",
    "GCA_900000001.1_X_genomic.fna": ">CAAAAA010000001.1 contig 1\nAAAA\n>CAAAAA010000002.1 contig 2\nCCCC\n"
                                     ">CAAAAA010000001.1 duplicate header\nGG\n",
    "GCF_999999999.1_unlisted_genomic.fna": ">NZ_UNLISTED.1 no summary row\nGATTACA\n",
}


def _row(acc, name, taxid, organism, ftp):
    cols = [""] * 23
    cols[0], cols[1], cols[5], cols[7], cols[19] = acc, name, taxid, organism, ftp
    return "\t".join(cols) + "\n"


SUMMARIES = {
    "assembly_summary_refseq.txt": "#   See README\n# assembly_accession\tbioproject\n"
    + _row("GCF_000005845.2", "ASM584v2_genomic", "511145", "Escherichia coli K-12", "ftp://ftp.ncbi/GCF_000005845.2")
    + _row("GCF_000009045.1", "ASM904v1_genomic", "224308", "Bacillus subtilis 168", "ftp://ftp.ncbi/GCF_000009045.1")
    + _row("GCF_555555555.1", "noftp", "1", "no ftp path", ""),
    "assembly_summary_genbank.txt": "# genbank\n"
    + _row("GCA_900000001.1", "X_genomic", "1423", "Bacillus subtilis", "ftp://ftp.ncbi/GCA_900000001.1")
    + _row("GCF_000009045.1", "ASM904v1_genomic", "1423", "override from genbank", "ftp://ftp.ncbi/GCF_000009045.1b"),
}
SELECTED = "GCF_000005845.2_ASM584v2\nGCF_000009045.1\nGCA_900000001.1_X\nGCF_123456789.1_missing\nGCF_555555555.1\n\n"

# downloadDB.py by hand: taxid from the last summary holding the GCF (genbank overrides
# refseq, :83-96); the row without ftp_path is dropped (:89); every .fna in the directory
# gets a row, "Unknown TaxID" without a summary row (:182,195); identifiers = first header
# field, a set (:191-192); genomes with a summary row and a file succeed (:137-140).
EXPECT_ROWS = {
    ("GCF_000005845.2", "511145", frozenset({"NC_000913.3"})),
    ("GCF_000009045.1", "1423", frozenset({"NC_000964.3", "NZ_PLASMID1.1"})),
    ("GCA_900000001.1", "1423", frozenset({"CAAAAA010000001.1", "CAAAAA010000002.1"})),
    ("GCF_999999999.1", "Unknown TaxID", frozenset({"NZ_UNLISTED.1"})),
}
EXPECT_OK = {"GCF_000005845.2_ASM584v2_genomic.fna", "GCF_000009045.1_ASM904v1_genomic.fna",
             "GCA_900000001.1_X_genomic.fna"}
EXPECT_FAILED = {"GCF_123456789.1", "GCF_555555555.1"}


@pytest.fixture
def tree(tmp_path):
    g = tmp_path / "genomes"
    c = tmp_path / "cache"
    g.mkdir()
    c.mkdir()
    for n, t in GENOMES.items():
        (g / n).write_text(t)
    (g / "README.txt").write_text("not a genome\n")
    for n, t in SUMMARIES.items():
        (c / n).write_text(t)
    (tmp_path / "selected.txt").write_text(SELECTED)
    return tmp_path


def _rows(path):
    lines = open(path, newline="").read().split("\r\n")
    assert lines[0] == "GCF\tTaxID\tIdentifiers" and lines[-1] == ""
    out = set()
    for ln in lines[1:-1]:
        gcf, taxid, ids = ln.split("\t")
        out.add((gcf, taxid, frozenset(ids.split(";"))))
    return out


def _records(text):
    recs = text.strip("\n").split("\n>")
    return sorted((r if r.startswith(">") else ">" + r).strip("\n") for r in recs if r)


def test_extract_gcf_and_summaries(tree):
    assert cache.extract_gcf("GCF_000005845.2_ASM584v2_genomic.fna") == "GCF_000005845.2"
    assert cache.extract_gcf("GCF_000009045.1") == "GCF_000009045.1"
    data = cache.load_assembly_summaries(cache.summary_paths(str(tree / "cache")))
    assert set(data) == {"GCF_000005845.2", "GCF_000009045.1", "GCA_900000001.1"}
    assert data["GCF_000009045.1"]["taxid"] == "1423"  # genbank read last
    assert data["GCF_000009045.1"]["ftp_path"] == "https://ftp.ncbi/GCF_000009045.1b"
    assert data["GCF_000005845.2"]["file_name"] == "GCF_000005845.2_ASM584v2_genomic.fna"


def test_build_cache_matches_reference_semantics(tree):
    tax = tree / "detailed_taxonomy.tsv"
    res = cache.build_cache(str(tree / "selected.txt"), str(tree / "genomes"), str(tax), str(tree / "cache"),
                            log=lambda m: None)
    assert _rows(tax) == EXPECT_ROWS
    assert set(res["ok"]) == EXPECT_OK and set(res["failed"]) == EXPECT_FAILED
    combined = open(res["combined"]).read()
    want = "".join(GENOMES[n] for n in sorted(EXPECT_OK))
    assert len(combined) == len(want) and _records(combined) == _records(want)
    # deterministic order here: selection order
    assert combined == "".join(GENOMES[n] for n in res["ok"])


def test_dropin_script(tree):
    tax = tree / "t.tsv"
    r = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "downloadDB.py"), str(tree / "selected.txt"),
                        str(tree / "genomes"), str(tax), str(tree / "cache")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert _rows(tax) == EXPECT_ROWS
    assert os.path.exists(tree / "genomes" / "combined_genomes.fasta")
    assert " - Successfully downloaded: 3" in r.stderr and " - Failed downloads: 2" in r.stderr
    r = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "downloadDB.py"), "x"], capture_output=True, text=True)
    assert r.returncode == 1 and "Usage" in r.stdout


def test_failed_downloads_counted_once_and_text_mode_line_ends(tmp_path):
    """failed_downloads is a set (downloadDB.py:124,127): a GCF listed twice fails once.
    concatenate_genomes copies through text-mode files (:215-218): CRLF / lone CR -> LF,
    also across the 16 MiB chunk boundary."""
    g = tmp_path / "g"
    g.mkdir()
    ok, failed = cache.resolve_downloads(["GCF_1.1", "GCF_2.1", "GCF_1.1"], {}, str(g))
    assert ok == [] and failed == ["GCF_1.1", "GCF_2.1"]
    big = b"A" * ((1 << 24) - 1) + b"\r\nCC\rGG\r"
    (g / "a.fna").write_bytes(b">x\r\nACGT\r\n")
    (g / "b.fna").write_bytes(big)
    out = tmp_path / "c.fasta"
    assert cache.concatenate_genomes(str(g), ["a.fna", "missing.fna", "b.fna"], str(out)) == ["a.fna", "b.fna"]
    assert out.read_bytes() == b">x\nACGT\n" + b"A" * ((1 << 24) - 1) + b"\nCC\nGG\n"

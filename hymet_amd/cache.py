"""Reference cache materialisation, offline.

`scripts/downloadDB.py` downloads the selected genomes and then writes the two files the
rest of HYMET consumes (`run_hymet_cami.sh:135-164`):

* `detailed_taxonomy.tsv` -- one row per downloaded genome: GCF, TaxID (from the NCBI
  assembly summaries, "Unknown TaxID" when absent) and the genome's FASTA identifiers joined
  by ';' (`downloadDB.py:178-207`);
* `combined_genomes.fasta` -- the downloaded genome files concatenated
  (`downloadDB.py:209-222`), read and written in text mode, so CRLF and lone CR line ends
  become LF (Python's universal newlines); other bytes are copied unchanged.

This module builds both from files already on disk (no network: a genome that is not in
the genome directory counts as a failed download).  Order: the reference iterates Python
sets and `os.listdir`, so its row, identifier and genome orders vary between runs; here
they are fixed -- .fna files in sorted name order, identifiers in first-appearance order,
genomes in the selection file's order.  Parity with the reference is defined modulo those
orders.  The builder is unpinned: running the reference's class to write fixtures was refused
(DESIGN.md §4), so tests/test_cache.py checks expectations derived by hand from
`downloadDB.py:78-222`.
"""
from __future__ import annotations

import csv
import os
from typing import Dict, Iterable, List, Optional, Tuple

UNKNOWN_TAXID = "Unknown TaxID"


def extract_gcf(filename: str) -> str:
    """`downloadDB.py:106-111`: the first two '_' fields ("GCF_000005845.2_ASM584v2.fna" ->
    "GCF_000005845.2")."""
    parts = filename.split("_")
    return f"{parts[0]}_{parts[1]}"


def load_assembly_summaries(paths: Iterable[str]) -> Dict[str, dict]:
    """`downloadDB.py:78-97`: rows of the NCBI assembly_summary files with a non-empty
    ftp_path (column 20); later files override earlier ones (refseq, then genbank)."""
    data: Dict[str, dict] = {}
    for path in paths:
        with open(path, "r") as f:
            for line in f:
                if line.startswith("#"):
                    continue
                parts = line.strip().split("\t")
                if len(parts) > 19 and parts[19]:
                    data[parts[0]] = {
                        "ftp_path": parts[19].replace("ftp://", "https://"),
                        "organism_name": parts[7],
                        "taxid": parts[5],
                        "file_name": f"{parts[0]}_{parts[1]}.fna",
                    }
    return data


def summary_paths(cache_dir: str) -> List[str]:
    """The cached summaries the reference reads (`downloadDB.py:37-53`), those present."""
    out = []
    for key in ("refseq", "genbank"):
        p = os.path.join(cache_dir, f"assembly_summary_{key}.txt")
        if os.path.exists(p):
            out.append(p)
    return out


def read_selection(genomes_file: str) -> List[str]:
    """`downloadDB.py:99-104`: GCF identifiers of the non-empty lines."""
    with open(genomes_file) as f:
        return [extract_gcf(line.strip()) for line in f if line.strip()]


def resolve_downloads(gcfs: Iterable[str], assembly: Dict[str, dict], genome_dir: str) -> Tuple[List[str], List[str]]:
    """The reference's download step without the network (`downloadDB.py:113-142`): a GCF with
    summary metadata whose file is already in `genome_dir` succeeds, every other one fails.
    Returns (file names in selection order, failed GCFs).  The reference collects failures in
    a set (`failed_downloads.add`, :124,127), so a GCF listed twice counts once; first-seen
    order is kept here."""
    ok: List[str] = []
    failed: List[str] = []
    seen = set()
    seen_failed = set()
    for gcf in gcfs:
        meta = assembly.get(gcf)
        if meta and os.path.exists(os.path.join(genome_dir, meta["file_name"])):
            if meta["file_name"] not in seen:
                seen.add(meta["file_name"])
                ok.append(meta["file_name"])
        elif gcf not in seen_failed:
            seen_failed.add(gcf)
            failed.append(gcf)
    return ok, failed


def fasta_identifiers(path: str) -> List[str]:
    """Header identifiers of a FASTA file: the first whitespace field after '>'."""
    out: List[str] = []
    with open(path, "r") as f:
        for line in f:
            if line.startswith(">"):
                out.append(line.split()[0][1:])
    return out


def detailed_taxonomy_rows(genome_dir: str, assembly: Dict[str, dict]) -> List[Tuple[str, str, str]]:
    """`downloadDB.py:178-195`: every *.fna file in the directory, grouped by GCF."""
    rows: Dict[str, dict] = {}
    for name in sorted(os.listdir(genome_dir)):
        if not name.endswith(".fna"):
            continue
        gcf = extract_gcf(name)
        ent = rows.setdefault(gcf, {"taxid": UNKNOWN_TAXID, "ids": {}})
        for ident in fasta_identifiers(os.path.join(genome_dir, name)):
            ent["ids"].setdefault(ident, None)
        ent["taxid"] = assembly.get(gcf, {}).get("taxid", UNKNOWN_TAXID)
    return [(gcf, e["taxid"], ";".join(e["ids"])) for gcf, e in rows.items()]


def write_detailed_taxonomy(path: str, rows: Iterable[Tuple[str, str, str]]) -> None:
    """`downloadDB.py:197-205`: csv.writer, tab-delimited, header GCF/TaxID/Identifiers."""
    with open(path, "w", newline="") as f:
        w = csv.writer(f, delimiter="\t")
        w.writerow(["GCF", "TaxID", "Identifiers"])
        for r in rows:
            w.writerow(list(r))


def concatenate_genomes(genome_dir: str, file_names: Iterable[str], output_file: str) -> List[str]:
    """`downloadDB.py:209-222`: the files appended in order; a missing file is skipped.
    The reference copies through text-mode file objects, so line ends are normalised to LF
    (CRLF and lone CR, as universal newlines read them); the copy streams 16 MiB chunks and
    carries a chunk-final CR into the next chunk.  Returns the names actually written."""
    written = []
    with open(output_file, "wb") as out:
        for name in file_names:
            p = os.path.join(genome_dir, name)
            try:
                src = open(p, "rb")
            except FileNotFoundError:
                continue
            with src:
                carry = b""
                while True:
                    chunk = src.read(1 << 24)
                    if not chunk:
                        break
                    chunk = carry + chunk
                    carry = b""
                    if chunk.endswith(b"\r"):
                        chunk, carry = chunk[:-1], b"\r"
                    out.write(chunk.replace(b"\r\n", b"\n").replace(b"\r", b"\n"))
                if carry:
                    out.write(b"\n")
            written.append(name)
    return written


def build_cache(genomes_file: str, genome_dir: str, taxonomy_file: str, cache_dir: str,
                combined: Optional[str] = None, log=print) -> dict:
    """The whole `downloadDB.py` main (`:224-249`) offline."""
    os.makedirs(genome_dir, exist_ok=True)
    os.makedirs(cache_dir, exist_ok=True)
    assembly = load_assembly_summaries(summary_paths(cache_dir))
    gcfs = read_selection(genomes_file)
    log(f"Starting download of {len(gcfs)} genomes...")
    ok, failed = resolve_downloads(gcfs, assembly, genome_dir)
    for gcf in failed:
        log(f"Failed to download {gcf}: not in {genome_dir} (offline)")
    write_detailed_taxonomy(taxonomy_file, detailed_taxonomy_rows(genome_dir, assembly))
    log(f"Detailed taxonomy file saved to: {taxonomy_file}")
    combined = combined or os.path.join(genome_dir, "combined_genomes.fasta")
    log("Concatenating genomes...")
    concatenate_genomes(genome_dir, ok, combined)
    log(f"Genomes concatenated into {combined}")
    log("\nSummary:")
    log(f" - Successfully downloaded: {len(ok)}")
    log(f" - Failed downloads: {len(failed)}")
    log(f" - Combined file: {combined}")
    return {"ok": ok, "failed": failed, "combined": combined}

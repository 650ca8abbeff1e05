"""Stage drop-ins with the reference scripts' argv / file / exit-code contracts.

    python -m hymet_amd.cli screen  INPUT_DIR DB.msh SCREEN_TAB FILTERED SORTED TOP_HITS SELECTED THRESH
        == scripts/mash.sh:4-55 (mash screen -p 8 -v 0.9, sort -u -k5,5, sort -gr, threshold walk)
    python -m hymet_amd.cli limit --selected F --output F [--score-file F]... [--max N] [--dedupe] ...
        == scripts/limit_candidates.py:47-89,249-289
    python -m hymet_amd.cli map     INPUT_DIR REFERENCE_FASTA INDEX_PATH PAF_OUT
        == scripts/minimap2.sh:4-33 (minimap2 -I2g -d, minimap2 -x asm10)
    python -m hymet_amd.cli classify        --paf P --taxonomy T --hierarchy H --output O [--processes N]
        == scripts/classification_cami.py:345-354
    python -m hymet_amd.cli classify-legacy (same flags)
        == scripts/classification.py:184-200
    python -m hymet_amd.cli build-id-map detailed_taxonomy.tsv out_map.tsv
        == tools/build_id_map.py (classification fallback, run_hymet_cami.sh:191)
    python -m hymet_amd.cli mini-classify input.paf id_to_taxid.tsv out.tsv
        == tools/mini_classify.py (classification fallback, run_hymet_cami.sh:192)
    python -m hymet_amd.cli hymet2cami classified_sequences.tsv
        == tools/hymet2cami.py (CAMI profile export, run_hymet_cami.sh:214-218)
    python -m hymet_amd.cli taxonomy-hierarchy [NAMES_DMP NODES_DMP OUT]
        == scripts/taxonomy_hierarchy.py (taxdump -> taxonomy_hierarchy.tsv)
    python -m hymet_amd.cli download-db GENOMES_FILE OUTPUT_DIR TAXONOMY_FILE CACHE_DIR
        == scripts/downloadDB.py:178-249 offline (detailed_taxonomy.tsv, combined_genomes.fasta)
    python -m hymet_amd.cli eval-cami [--pred-profile ... --outdir D]
        == tools/eval_cami.py (CAMI profile and contig metrics)

The thin wrappers under scripts/ call these, so run_hymet_cami.sh / main.pl can use them
in place of the reference stage scripts unchanged.  All device work goes through
libhymet_gpu.so; without it (or without a GPU) every GPU subcommand fails loudly.
"""
from __future__ import annotations

import argparse
import glob
import logging
import os
import sys
from typing import List, Optional, Sequence

import numpy as np


def _fna_files(input_dir: str) -> List[str]:
    # bash expands "$INPUT_DIR"/*.fna in collation order; LC_ALL=C byte order here
    return sorted(glob.glob(os.path.join(input_dir, "*.fna")), key=lambda p: p.encode())


def _write_lines(path: str, lines: Sequence[str]):
    with open(path, "w", encoding="utf-8", newline="") as f:
        for l in lines:
            f.write(l + "\n")


# ------------------------------------------------------------------ screen (mash.sh)
def cmd_screen(argv: Sequence[str]) -> int:
    if len(argv) != 8:
        print("usage: screen INPUT_DIR DB.msh SCREEN_TAB FILTERED SORTED TOP_HITS SELECTED THRESH", file=sys.stderr)
        return 2
    input_dir, msh_path, screen_tab, filtered, sorted_p, top_hits, selected, thresh = argv
    from . import screen as scr
    from . import select as sel
    from ._lib import Gpu
    from .msh import load_db
    from .seqio import DevicePool, read_fasta
    files = _fna_files(input_dir)
    db = load_db(msh_path)
    gpu = Gpu(int(os.environ.get("HYMET_DEVICE", "0")))
    rows: List[str] = []
    if files:
        ss = read_fasta(files)
        res = scr.screen(gpu, DevicePool(gpu, ss, DevicePool.ALPHA_MASH), [db])[0]
        rows = res.lines(v_max=0.9)
    _write_lines(screen_tab, rows)
    f_rows = sel.sort_unique_k5(rows)
    _write_lines(filtered, f_rows)
    s_rows = sel.sort_gr(f_rows)
    _write_lines(sorted_p, s_rows)
    n_files = len(files)
    need = sel.min_candidates(n_files)
    print("====================================")
    print(f"Number of input sequences: {n_files}")
    print(f"Minimum expected candidates: {need}")
    print("====================================")
    best, top, names, log = sel.threshold_walk(s_rows, thresh, n_files)
    _write_lines(top_hits, top)
    _write_lines(selected, names)
    print("\n".join(log))     # mash.sh:35-36,50,57-60: per-threshold lines, fallback note, summary
    return 0


# ------------------------------------------------------------ limit (limit_candidates.py)
def cmd_limit(argv: Sequence[str]) -> int:
    from . import select as sel
    p = argparse.ArgumentParser(prog="limit", description="Limit Mash candidate genomes (limit_candidates.py).")
    p.add_argument("--selected", required=True)
    p.add_argument("--output", required=True)
    p.add_argument("--score-file", action="append", default=[], dest="score_files")
    p.add_argument("--assembly-dir", default=None)
    p.add_argument("--max", type=int, default=5000)
    p.add_argument("--dedupe", action="store_true")
    p.add_argument("--log", default=None)
    p.add_argument("--no-download", action="store_true")
    a = p.parse_args(argv)
    if a.max <= 0:
        raise SystemExit("The --max value must be greater than zero.")
    with open(a.selected, "r", encoding="utf-8") as f:
        cands = [l.strip() for l in f if l.strip()]
    if not cands:
        raise SystemExit(f"No candidates found in {a.selected}")
    scores = sel.read_scores([s for s in a.score_files if os.path.exists(s)])
    # never downloads: without local assembly summaries the species key is the accession.
    # Default directory as limit_candidates.py:259-263 resolves it (repo/data/...).
    adir = a.assembly_dir or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data",
                                          "downloaded_genomes", "assembly_summaries")
    smap = sel.species_map(adir) if a.dedupe else {}
    chosen = sel.limit(cands, scores, a.max, a.dedupe, smap)
    tmp = a.output + ".tmp"
    _write_lines(tmp, chosen)
    os.replace(tmp, a.output)
    kept = len(chosen)
    summary = (f"[limit_candidates] kept {kept} / {len(cands)} candidates ({kept} unique keys) "
               f"{'(species dedupe)' if a.dedupe else ''}")
    print(summary)
    if a.log:
        os.makedirs(os.path.dirname(os.path.abspath(a.log)), exist_ok=True)
        with open(a.log, "a", encoding="utf-8") as f:
            f.write(summary.rstrip("\n") + "\n")
    return 0


# ------------------------------------------------------------------ map (minimap2.sh)
def build_parts(gpu, refs, split_idx: str = "2g", mini_batch: float = 50e6, w: int = 10, k: int = 15):
    """minimap2 -I<split_idx> -d: the device index, one part per <= split_idx bases."""
    from . import mapper as mp
    parts_idx = mp.split_parts(refs.lengths, float(mp.parse_num(split_idx)), mini_batch)
    parts, first = [], []
    for p in parts_idx:
        sub = refs.subset(p) if len(parts_idx) > 1 else refs
        parts.append(mp.IndexPart(gpu, sub, w, k))
        first.append(int(p[0]))
    return parts, list(refs.names), refs.lengths, first


def read_query_files(paths: Sequence[str]) -> bytes:
    """The pooled input/*.fna as one FASTA text, file order kept; bytes before a file's
    first record are skipped (kseq does) and files are joined on a line break."""
    out = []
    for p in paths:
        with open(p, "rb") as f:
            d = f.read()
        if p.endswith(".gz") or d[:2] == b"\x1f\x8b":
            import gzip
            d = gzip.decompress(d)
        if not d.startswith(b">"):
            i = d.find(b"\n>")
            d = d[i + 1:] if i >= 0 else b""
        if d and not d.endswith(b"\n"):
            d += b"\n"
        out.append(d)
    return b"".join(out)


def map_paf(gpu, parts, names, lens, first, query_fasta: bytes, batch_bases: int = 40_000_000) -> bytes:
    """`-x asm10` mapping of the pooled queries against the index parts -> resultados.paf
    bytes in minimap2's order (part by part; queries in input order within a part), through
    the fused path's device kernels (records accumulated in HBM, text written on the GPU)."""
    from . import pipeline
    from .ingest import FastaIndex, QueryShard
    ix = pipeline.make_index_set(gpu, names, lens, parts, first)
    fx = FastaIndex(query_fasta)
    sh = QueryShard.from_fasta(gpu, fx, 0, fx.n, batch_bases)
    acc = pipeline.PafAcc(gpu)
    pipeline.map_shard(gpu, ix, sh, acc)
    return pipeline.emit_paf_bytes(gpu, ix, sh, acc, {})


def cmd_map(argv: Sequence[str]) -> int:
    """scripts/minimap2.sh: build the index unless INDEX_PATH is non-empty (:10-19), then map
    input/*.fna with asm10 (:23).  The device index is persisted as INDEX_PATH.hymet beside a
    manifest in INDEX_PATH, so a warm call only loads it (no sketching, no sorting)."""
    if len(argv) != 4:
        print("usage: map INPUT_DIR REFERENCE_FASTA INDEX_PATH PAF_OUT", file=sys.stderr)
        return 2
    input_dir, ref_fasta, index_path, paf_out = argv
    from . import mapper as mp
    from ._lib import Gpu
    from .seqio import read_fasta
    split = os.environ.get("SPLIT_IDX", "2g")
    cached = os.path.exists(index_path) and os.path.getsize(index_path) > 0
    try:
        gpu = Gpu(int(os.environ.get("HYMET_DEVICE", "0")))
        loaded = None
        if not cached:
            print("Creating index with minimap2...")
        else:
            print(f"Using cached minimap2 index: {index_path}")
            loaded = mp.load_index(gpu, index_path, ref_fasta, split)
        if loaded is None:   # fresh, or a CPU minimap2 .mmi we keep untouched: build in HBM
            # HYMET_INDEX_MINI_BATCH: the index reader's mini-batch (minimap2's 50 Mbp chunking)
            mini = float(os.environ.get("HYMET_INDEX_MINI_BATCH", "50e6"))
            parts, names, lens, first = build_parts(gpu, read_fasta([ref_fasta]), split, mini)
            if not cached:
                mp.save_index(index_path, parts, names, lens, first, ref_fasta, split)
        else:
            parts, names, lens, first = loaded
    except Exception as e:  # minimap2.sh:13-16
        print(f"Error creating index with minimap2. ({e})")
        return 1
    print("Running alignment with minimap2...")
    try:
        data = map_paf(gpu, parts, names, lens, first, read_query_files(_fna_files(input_dir)))
        with open(paf_out, "wb") as f:
            f.write(data)
    except Exception as e:  # minimap2.sh:25-29
        print(f"Error running alignment with minimap2. ({e})")
        return 1
    print(f"Alignment completed successfully! Results saved to {paf_out}.")
    return 0


# --------------------------------------------------- classify (classification*.py)
def cmd_classify(argv: Sequence[str], legacy: bool = False) -> int:
    from . import classify as cls
    from ._lib import Gpu
    p = argparse.ArgumentParser(prog="classify")
    p.add_argument("--paf", required=True)
    p.add_argument("--taxonomy", required=True)
    p.add_argument("--hierarchy", required=True)
    p.add_argument("--output", required=True)
    p.add_argument("--processes", type=int, default=4)   # accepted; the GPU does the fan-out
    a = p.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(levelname)s - %(message)s")
    gpu = Gpu(int(os.environ.get("HYMET_DEVICE", "0")))
    variant = cls.LEGACY if legacy else cls.CAMI
    c = cls.Classifier(gpu, a.taxonomy, a.hierarchy, variant)
    paf = cls.read_paf(a.paf, variant)
    if legacy and len(paf.queries) == 0:
        raise ZeroDivisionError("division by zero")  # classification.py:182 on an empty PAF
    res = c.run(paf)
    rows = c.rows(res)
    with open(a.output, "wb") as f:
        f.write(c.tsv_bytes(res, rows))
    n = len(rows)
    k = sum(1 for r in rows if r[1] != "Unknown")
    logging.info(f"Classification complete. Results saved to {a.output}")
    logging.info(f"Classified: {k}/{n} ({(k / n if n else 0):.1%})")
    return 0


# ------------------------------------------- CAMI export / taxdump
def cmd_hymet2cami(argv: Sequence[str]) -> int:
    """tools/hymet2cami.py <classified_sequences.tsv>: CAMI profile on stdout, progress on
    stderr; names.dmp / nodes.dmp from TAXONKIT_DB (default <repo>/taxonomy_files)."""
    from pathlib import Path
    from .taxonomy import hymet2cami
    if len(argv) != 1:
        print("Usage: hymet2cami.py <classified_sequences.tsv>", file=sys.stderr)
        return 1
    path = Path(argv[0]).resolve()
    if not path.is_file():
        print(f"Missing classified_sequences TSV: {path}", file=sys.stderr)
        return 1
    taxdb = os.environ.get("TAXONKIT_DB", str(Path(__file__).resolve().parents[1] / "taxonomy_files"))
    sys.stdout.write(hymet2cami(str(path), taxdb))
    return 0


def cmd_taxonomy_hierarchy(argv: Sequence[str]) -> int:
    """scripts/taxonomy_hierarchy.py: taxonomy_files/{names,nodes}.dmp -> data/taxonomy_hierarchy.tsv
    (paths relative to the working directory, as the reference; or NAMES NODES OUT)."""
    from .taxonomy import hierarchy_tsv
    if argv and len(argv) != 3:
        print("usage: taxonomy-hierarchy [NAMES_DMP NODES_DMP OUT_TSV]", file=sys.stderr)
        return 2
    names, nodes, out = argv if argv else (os.path.join(".", "taxonomy_files", "names.dmp"),
                                           os.path.join(".", "taxonomy_files", "nodes.dmp"),
                                           os.path.join(".", "data", "taxonomy_hierarchy.tsv"))
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    for p in (names, nodes):
        if not os.path.exists(p):
            raise FileNotFoundError(f"File {p} not found.")
    print("Loading data from files...")
    data = hierarchy_tsv(names, nodes)
    print("Generating taxonomy_hierarchy.tsv...")
    with open(out, "wb") as f:
        f.write(data)
    print(f"File generated successfully: {out}")
    return 0


def cmd_download_db(argv: Sequence[str]) -> int:
    """scripts/downloadDB.py <genomes_file> <output_dir> <taxonomy_file> <cache_dir>, offline
    (SURVEY.md §8f-2): genomes already in output_dir, summaries cached in cache_dir."""
    from .cache import build_cache
    if len(argv) != 4:
        print("Usage: python3 download_genomes.py <genomes_file> <output_dir> <taxonomy_file> <cache_dir>")
        return 1
    build_cache(argv[0], argv[1], argv[2], argv[3], log=lambda m: print(m, file=sys.stderr))
    return 0


def main(argv: Optional[Sequence[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        print(__doc__, file=sys.stderr)
        return 2
    cmd, rest = argv[0], argv[1:]
    if cmd == "screen":
        return cmd_screen(rest)
    if cmd == "limit":
        return cmd_limit(rest)
    if cmd == "map":
        return cmd_map(rest)
    if cmd == "classify":
        return cmd_classify(rest)
    if cmd == "classify-legacy":
        return cmd_classify(rest, legacy=True)
    if cmd == "build-id-map":
        from .fallback import main_build_id_map
        return main_build_id_map(rest)
    if cmd == "mini-classify":
        from .fallback import main_mini_classify
        return main_mini_classify(rest)
    if cmd == "hymet2cami":
        return cmd_hymet2cami(rest)
    if cmd == "taxonomy-hierarchy":
        return cmd_taxonomy_hierarchy(rest)
    if cmd == "download-db":
        return cmd_download_db(rest)
    if cmd == "eval-cami":
        from .evaluate import main as eval_main
        return eval_main(rest)
    print(f"unknown subcommand {cmd!r}", file=sys.stderr)
    return 2


if __name__ == "__main__":
    sys.exit(main())

"""TEST INFRASTRUCTURE ONLY -- the whole hot path on the CPU oracle restatements, stage by
stage as run_hymet_cami.sh drives the reference (steps 1-5):

  mash screen x DBs (mash_oracle.c) -> mash.sh selection (select_oracle) -> union sort -u
  -> limit_candidates (select_oracle) -> minimap2 -I2g -d + -x asm10 (mm_oracle.c)
  -> PAF text -> classification_cami.py restatement (classify_oracle)

Used as the checker in tests/test_pipeline_gpu.py and as bench.py's cpu_baseline leg."""
from __future__ import annotations

import ctypes
import os
import tempfile

import numpy as np

from oracle import classify_oracle, oracle_lib, select_oracle


def screen_rows(pool_seqs, db, mm=None):
    sh, md, ss, nk = oracle_lib.screen(pool_seqs, db.k, db.seed, db.sketch_size, [db.ref_hashes(i) for i in range(db.n_refs)])
    refs = [(db.names[i], db.comments[i], int(db.offsets[i + 1] - db.offsets[i])) for i in range(db.n_refs)]
    return select_oracle.screen_lines(refs, sh, md, ss, db.k)


def select(pool_seqs, dbs, thresh="0.9", cand_max=5000, n_files=1):
    sorted_tabs, sels = [], []
    for db in dbs:
        rows = select_oracle.sort_gr(select_oracle.sort_unique_k5(screen_rows(pool_seqs, db)))
        t, top, names, _ = select_oracle.select_threshold(rows, thresh, n_files)
        sorted_tabs.append(rows)
        sels.append(names)
    selected = select_oracle.union_sorted(*sels)
    scores = {}
    for rows in sorted_tabs:
        for line in rows:
            p = line.split("\t")
            try:
                s = float(p[0])
            except ValueError:
                continue
            if p[4] not in scores or s > scores[p[4]]:
                scores[p[4]] = s
    if cand_max is None:        # main.pl:94-104: no limit_candidates step, the sort -u union is used
        return selected, sorted_tabs
    limited, _ = select_oracle.limit_candidates(selected, scores, cand_max)
    return limited, sorted_tabs


def split_parts(lengths, batch=2e9, mini=50e6):
    parts, cur, plen, i = [], [], 0, 0
    while i < len(lengths):
        if plen > batch:
            parts.append(cur)
            cur, plen = [], 0
        mb = 0
        while i < len(lengths):
            cur.append(i)
            mb += int(lengths[i])
            plen += int(lengths[i])
            i += 1
            if mb >= mini:
                break
    if cur:
        parts.append(cur)
    return parts


def map_paf(ref_names, ref_seqs, queries, part_bases=2e9, mini_batch=50e6, threads=1, opt=None):
    """minimap2 -I<part_bases> -d ; minimap2 -x asm10 : PAF lines in minimap2's order.
    threads > 1 maps queries concurrently (the C mapper releases the GIL; its state is
    per call), then emits them in input order like minimap2's ordered output."""
    from concurrent.futures import ThreadPoolExecutor
    lens = [len(s) for s in ref_seqs]
    parts = split_parts(lens, part_bases, mini_batch)
    out = []
    resolved = False
    for p in parts:
        idx = oracle_lib.MmIndex([ref_seqs[i] for i in p], names=[ref_names[i] for i in p])
        if not resolved:
            opt = opt if opt is not None else oracle_lib.asm10_opt()
            oracle_lib._mm_lib().mmo_opt_update_mid_occ(ctypes.byref(opt), idx.h)
            resolved = True

        def one(q):
            qn, qs = q
            regs, rl = oracle_lib.mm_map(idx, opt, qs, qn)
            return oracle_lib.format_paf(qn, len(qs), regs, rl, idx.names, idx.lens)

        if threads > 1:
            with ThreadPoolExecutor(threads) as ex:
                for lines in ex.map(one, queries, chunksize=16):
                    out.extend(lines)
        else:
            for q in queries:
                out.extend(one(q))
    return out


def run(queries, dbs, ref_lookup, taxonomy, hierarchy, thresh="0.9", cand_max=5000, part_bases=2e9, mini_batch=50e6,
        threads=1, legacy=False):
    """queries: list of (name, seq bytes).  Returns (selected, paf lines, tsv bytes).
    cand_max=None, legacy=True: the main.pl path (no limit step, classification.py)."""
    selected, _ = select([q[1] for q in queries], dbs, thresh, cand_max)
    names, seqs = ref_lookup(selected)
    paf = map_paf(names, seqs, queries, part_bases, mini_batch, threads)
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "resultados.paf")
        with open(p, "w") as f:
            f.write("".join(l + "\n" for l in paf))
        tsv = (classify_oracle.classify_legacy(p, taxonomy, hierarchy) if legacy
               else classify_oracle.classify_cami(p, taxonomy, hierarchy))
    return selected, paf, tsv

"""The fused, device-resident hot path of `bin/hymet run` (run_hymet_cami.sh steps 1-5):

    screen (3 sketch DBs, one hash pass)  -> mash.sh selection per DB -> union (sort -u)
    -> limit_candidates -> [candidate-keyed index cache, as run_hymet_cami.sh:135-171]
    -> minimap2 asm10 mapping per -I2g part -> classification_cami weighted LCA -> TSV

Everything between the input pool and the TSV stays in HBM except the small host-side
text steps (screen rows, candidate lists) and the region records that become PAF lines.
Multi-GPU: every rank holds its own contig shard; the screen counts and
the per-target PAF line counts are all-reduced; rank 0 assembles the TSV in the
reference's query order.
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import classify as cls
from . import mapper as mp
from . import screen as scr
from . import select as sel
from .msh import SketchDB
from .seqio import DevicePool, SeqSet, from_records


@dataclass
class Config:
    mash_thresh: str = "0.9"          # MASH_THRESH (run_hymet_cami.sh:31)
    cand_max: int = 5000              # CAND_MAX (run_hymet_cami.sh:26)
    dedupe: bool = False              # SPECIES_DEDUP
    split_idx: str = "2g"             # SPLIT_IDX / minimap2 -I
    index_mini_batch: float = 50e6    # minimap2 indexing mini-batch (bseq reader chunk)
    w: int = 10                       # minimap2 -d defaults
    k: int = 15
    map_batch_bases: int = 40_000_000  # query bases per device mapping batch (HBM budget)
    n_input_files: int = 1            # run_hymet_cami.sh copies one FASTA into input/


@dataclass
class IndexSet:
    names: List[str]
    lens: np.ndarray
    parts: List[mp.IndexPart]
    part_first: List[int]             # global target index of each part's rid 0
    opt: mp.MapOpt                    # asm10 options, mid_occ resolved on this set's first part


@dataclass
class RunResult:
    selected: List[str]
    screen_rows: List[List[str]]      # per DB, rows after sort -u -k5,5 | sort -gr
    thresholds: List[str]
    tsv: bytes
    n_queries: int
    n_classified: int
    n_paf_lines: int
    paf: Optional[List[str]] = None


class Pipeline:
    def __init__(self, gpu, dbs: Sequence[SketchDB], ref_lookup, taxonomy, hierarchy, cfg: Config = None, comm=None,
                 variant: int = cls.CAMI):
        """ref_lookup(names) -> SeqSet of the candidate genomes in combined_genomes.fasta
        order (the download cache; scripts/downloadDB.py is outside the accelerated path)."""
        self.gpu, self.cfg, self.comm = gpu, cfg or Config(), comm
        self.dbs = list(dbs)
        self.tables = [scr.ScreenTable(gpu, db) for db in self.dbs]
        self.ref_lookup = ref_lookup
        self.taxonomy, self.variant = taxonomy, variant
        # classification_cami.py runs as `... || true` (run_hymet_cami.sh:175-180): a
        # classifier that cannot load its inputs leaves an empty TSV, and the fallback runs
        try:
            self.classifier = cls.Classifier(gpu, taxonomy, hierarchy, variant)
            self.classifier_error = None
        except Exception as e:  # noqa: BLE001 -- any failure of the reference script
            self.classifier, self.classifier_error = None, e
        self.index_cache: Dict[str, IndexSet] = {}
        self.opt: Optional[mp.MapOpt] = None

    # ------------------------------------------------------------------ stages
    def screen_select(self, pool: DevicePool):
        res = scr.screen(self.gpu, pool, self.dbs, self.tables, self.comm)
        rows, thr, selections = [], [], []
        for r in res:
            s = sel.sort_gr(sel.sort_unique_k5(r.lines(v_max=0.9)))
            t, top, names = sel.select_threshold(s, self.cfg.mash_thresh, self.cfg.n_input_files)
            rows.append(s)
            thr.append(t)
            selections.append(names)
        selected = sel.union_sorted(*selections) if len(selections) > 1 else sel.union_sorted(selections[0])
        scores = sel.best_scores(rows)
        limited = sel.limit(selected, scores, self.cfg.cand_max, self.cfg.dedupe)
        return limited, rows, thr

    def index_for(self, selected: List[str]) -> IndexSet:
        key = hashlib.sha1(("".join(n + "\n" for n in selected)).encode()).hexdigest()
        if key in self.index_cache:
            return self.index_cache[key]
        refs: SeqSet = self.ref_lookup(selected)
        parts_idx = mp.split_parts(refs.lengths, float(mp.parse_num(self.cfg.split_idx)), self.cfg.index_mini_batch)
        parts, first = [], []
        for p in parts_idx:
            sub = refs.subset(p) if len(parts_idx) > 1 else refs
            parts.append(mp.IndexPart(self.gpu, sub, self.cfg.w, self.cfg.k))
            first.append(int(p[0]))
        # a fresh `minimap2 -x asm10` process per run: mm_mapopt_update resolves mid_occ from
        # the first part of THIS index (options.c), so the options live with the index set
        opt = mp.MapOpt.asm10()
        opt.resolve_mid_occ(parts[0])
        ix = IndexSet(list(refs.names), np.asarray(refs.lengths, np.int64), parts, first, opt)
        self.index_cache = {key: ix}  # one cached candidate set, like the sha1 cache dir
        return ix

    def prepare(self, queries: SeqSet) -> "Prepared":
        """Make the query set resident in HBM: one Mash-alphabet pool for the screen and
        minimap2-alphabet pools cut into mapping batches (sized for the anchor working set)."""
        pq = Prepared(queries, DevicePool(self.gpu, queries, DevicePool.ALPHA_MASH), [])
        for b0, b1 in _batches(queries.lengths, self.cfg.map_batch_bases):
            sub = queries if (b0 == 0 and b1 == queries.n) else queries.subset(range(b0, b1))
            names_hash = np.array([mp.x31_hash(n) for n in sub.names], np.uint32)
            pq.batches.append((b0, DevicePool(self.gpu, sub, DevicePool.ALPHA_MINIMAP2), names_hash))
        return pq

    def map_all(self, ix: IndexSet, pq: "Prepared"):
        """Per part, per query batch -> list of (part, query offset, MapResult)."""
        self.opt = ix.opt
        out = []
        for pi, part in enumerate(ix.parts):
            for b0, qp, nh in pq.batches:
                out.append((pi, b0, mp.map_part(self.gpu, part, qp, self.opt, nh)))
        return out

    def paf_table(self, ix: IndexSet, queries: SeqSet, results, with_text=False):
        """PAF lines in minimap2's output order (part-major, query order) as classifier arrays."""
        qnames = queries.names
        lq, lt, lb, lp, text = [], [], [], [], ([] if with_text else None)
        for pi, b0, res in results:
            first = ix.part_first[pi]
            regs = res.regs
            if len(regs) == 0:
                continue
            nper = np.diff(res.off)
            lq.append(np.repeat(np.arange(len(nper), dtype=np.int64) + b0, nper))
            lt.append(regs["rid"].astype(np.int32) + np.int32(first))
            lb.append(regs["blen"].astype(np.int64))
            lp.append(np.full(len(regs), pi, np.int32))
            if with_text:
                for q in np.flatnonzero(nper):
                    g = int(q) + b0
                    text.extend(mp.paf_lines(qnames[g], int(queries.lengths[g]), res.query(int(q)), int(res.rep_len[q]),
                                             ix.names[first:], ix.lens[first:]))
        if lq:
            all_q = np.concatenate(lq)
            uq, first_pos = np.unique(all_q, return_index=True)
            order_q = uq[np.argsort(first_pos, kind="stable")]      # queries by first appearance
            pos = np.empty(int(all_q.max()) + 1, np.int64)
            pos[order_q] = np.arange(len(order_q))
            line_q = pos[all_q].astype(np.int32)
            line_t, line_b = np.concatenate(lt), np.concatenate(lb)
            line_l = np.asarray(queries.lengths, np.int64)[all_q]
            fp = np.sort(first_pos)
            self.last_qkey = (np.concatenate(lp)[fp], order_q.astype(np.int64))  # (part of first line, query)
        else:
            self.last_qkey = (np.zeros(0, np.int32), np.zeros(0, np.int64))
            order_q = np.zeros(0, np.int64)
            line_q, line_t = np.zeros(0, np.int32), np.zeros(0, np.int32)
            line_b, line_l = np.zeros(0, np.int64), np.zeros(0, np.int64)
        exact = np.zeros(len(line_q), np.uint8)
        if self.variant == cls.LEGACY and len(line_q):
            # classification.py:141-151: query == target and coverage >= 0.99
            same = np.asarray(qnames, dtype=object)[all_q] == np.asarray(ix.names, dtype=object)[line_t]
            cov = np.where(line_l > 0, line_b / np.maximum(line_l, 1), 0.0)
            exact = (same & (cov >= 0.99)).astype(np.uint8)
        table = cls.PafTable([qnames[q] for q in order_q], line_q, list(ix.names), line_t, line_b, line_l, exact)
        return table, text

    # ------------------------------------------------------------------- run
    def run(self, queries, with_paf=False, query_ids=None) -> RunResult:
        """queries: a SeqSet, or a Prepared (already resident in HBM).  With several ranks,
        query_ids gives each local query's index in the whole input (default: the shards
        are consecutive slices in rank order); rank 0's RunResult.tsv is the whole TSV."""
        pq = queries if isinstance(queries, Prepared) else self.prepare(queries)
        queries = pq.queries
        selected, rows, thr = self.screen_select(pq.mash_pool)
        if not selected:
            raise RuntimeError("candidate list empty after applying limit")  # run_hymet_cami.sh:126
        ix = self.index_for(selected)
        results = self.map_all(ix, pq)
        table, text = self.paf_table(ix, queries, results, with_paf)
        part, q = self.last_qkey
        multi = self.comm is not None and self.comm.world > 1
        gid = None
        if multi:
            gid = (np.asarray(query_ids, np.int64)[q] if query_ids is not None
                   else (np.int64(self.comm.rank) << np.int64(32)) + q)
        rws, tsv = [], b""
        if self.classifier is not None:
            res = self.classifier.run(table, comm=self.comm)
            rws = self.classifier.rows(res)
            if multi:
                rws = gather_rows(self.comm, rws, part, gid)
            tsv = self.classifier.tsv_bytes(res, rws)
        n_rows = len(rws)
        if multi:
            n_rows = self.comm.broadcast_obj(n_rows)
        if n_rows < 1:  # fewer than 2 TSV lines: run_hymet_cami.sh:182-206
            tsv = self._fallback(table, part, gid)
            rws = []
        return RunResult(selected, rows, thr, tsv, len(rws), sum(1 for r in rws if r[1] != "Unknown"), table.n_lines, text)

    def _fallback(self, table, part, gid) -> bytes:
        """build_id_map + mini_classify over the PAF lines (first mapped hit per query), then
        the awk rewrite; dies like the script when even that leaves no row."""
        from . import fallback
        pairs = [(table.queries[int(a)], table.targets[int(b)]) for a, b in zip(table.line_q, table.line_t)]
        if self.comm is not None and self.comm.world > 1:
            # lines of a query sit together per part; queries sort by (part, input index)
            key = {table.queries[i]: (int(part[i]), int(gid[i])) for i in range(len(table.queries))}
            got = self.comm.gather_obj([(key[a], j, a, b) for j, (a, b) in enumerate(pairs)])
            if self.comm.rank != 0:
                return b""
            pairs = [(a, b) for _, _, a, b in sorted(x for g in got for x in g)]
        tsv = fallback.fallback_tsv(pairs, self.taxonomy)
        if tsv.count(b"\n") < 2:
            raise RuntimeError("classification still empty after fallback")  # run_hymet_cami.sh:205
        return tsv


def gather_rows(comm, rows, part: np.ndarray, qid: np.ndarray, dst: int = 0):
    """Rank `dst` assembles the classified_sequences.tsv rows of every contig shard
    (SURVEY.md §8e step 7).  minimap2 prints the pooled input's PAF index part by part, and
    within a part query by query in input order; the reference writes one row per query in
    order of first PAF appearance.  So rows sort by (part of the query's first line, the
    query's index in the whole input).  Other ranks get []."""
    got = comm.gather_obj((rows, np.asarray(part, np.int64), np.asarray(qid, np.int64)), dst)
    if comm.rank != dst:
        return []
    all_rows = [r for rw, _, _ in got for r in rw]
    if not all_rows:
        return []
    kp = np.concatenate([p for _, p, _ in got])
    kq = np.concatenate([q for _, _, q in got])
    order = np.lexsort((kq, kp))
    return [all_rows[i] for i in order]


@dataclass
class Prepared:
    queries: SeqSet
    mash_pool: DevicePool
    batches: list


def _batches(lengths: np.ndarray, max_bases: int):
    out, b0, acc = [], 0, 0
    for i, L in enumerate(lengths):
        if acc and acc + int(L) > max_bases:
            out.append((b0, i))
            b0, acc = i, 0
        acc += int(L)
    if b0 < len(lengths) or not out:
        out.append((b0, len(lengths)))
    return out

"""The fused, device-resident hot path of `bin/hymet run` (run_hymet_cami.sh steps 1-5):

    FASTA bytes (host) -> one H2D copy -> ASCII pool + packed alphabets (HBM)
    -> screen (sketch DBs, one hash pass) -> mash.sh selection per DB -> union (sort -u)
    -> limit_candidates -> [candidate-keyed index cache, as run_hymet_cami.sh:135-171]
    -> minimap2 asm10 mapping per -I2g part into a device-resident PAF (hymet_paf_acc)
    -> classification_cami weighted LCA over that PAF in HBM -> TSV (and PAF) text written
       on the device, copied out once.

Host work per run is the short text logic of selection and a few dozen library calls; no
per-contig or per-line Python.  Multi-GPU: every rank takes a contiguous
byte range of the same FASTA (ingest.shard_bytes); the DB hash slices are all-gathered, the
screen hit counts (by canonical DB index) and the per-target PAF line counts all-reduced;
fixed-size LCA row records and the name pools are all-gathered and rank 0 writes the TSV in
the reference's query order.  One host thread issues collectives at a time (dist.Comm).
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import classify as cls
from . import mapper as mp
from . import screen as scr
from . import select as sel
from ._lib import check, ptr
from .ingest import FastaIndex, QueryShard, shard_bytes
from .msh import SketchDB, read_msh
from .seqio import SeqSet

_c = ctypes
TSV_HEADER = b"Query\tLineage\tTaxonomic Level\tConfidence\r\n"


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
    map_streams: int = 2              # concurrent mapping batches (library contexts / HIP streams)
    n_input_files: int = 1            # run_hymet_cami.sh copies one FASTA into input/
    limit: bool = True                # run_hymet_cami.sh:101-126; main.pl has no limit step (False)
    # Every run re-reads its inputs, as the reference's stage processes do: `mash screen`
    # loads each sketch DB (S1, when the DBs are given as .msh paths) and
    # classification_cami.py loads detailed_taxonomy.tsv + taxonomy_hierarchy.tsv (C1-C2).
    # False: load once at construction (a resident service).
    reload_inputs: bool = True


@dataclass
class IndexSet:
    names: List[str]
    lens: np.ndarray
    parts: List[mp.IndexPart]
    part_first: List[int]             # global target index of each part's rid 0
    opt: mp.MapOpt                    # asm10 options, mid_occ resolved on this set's first part
    dev: Dict[str, object] = field(default_factory=dict)   # target name pool / lengths in HBM


class HostText:
    """Text the device wrote, landed by one DMA in a pinned host buffer of the pipeline (no
    host-side copy into a fresh bytes object, which cost ~80 ms per GB of PAF mostly in page
    faults).  The buffers alternate between runs; before a buffer is reused, the text still
    referenced from an earlier result is copied out (copy-on-reuse), so a result stays valid
    for as long as it is referenced."""

    def __init__(self, buf, n: int):
        self._buf, self.n, self._bytes = buf, int(n), None

    def view(self) -> memoryview:
        """A zero-copy view of the text.  It stays valid only while this HostText (or the
        RunResult holding it) is referenced: copy-on-reuse tracks the HostText, not views of
        it, so a view kept past the HostText's lifetime may see a later run's text.  Use
        bytes() for a copy that lives on its own."""
        if self._bytes is not None:
            return memoryview(self._bytes)
        return memoryview(self._buf)[:self.n]

    def bytes(self) -> bytes:
        if self._bytes is None:
            self._bytes = bytes(memoryview(self._buf)[:self.n])
            self._buf = None
        return self._bytes

    detach = bytes   # called by the pipeline before it reuses the buffer


@dataclass
class RunResult:
    selected: List[str]
    screen_rows: List[List[str]]      # per DB, rows after sort -u -k5,5 | sort -gr
    thresholds: List[str]
    tsv: bytes
    n_queries: int                    # TSV rows (queries with >= 1 PAF line)
    n_classified: int                 # rows with a lineage other than Unknown
    n_paf_lines: int                  # this rank's PAF lines
    paf_text: Optional[object] = None  # this rank's resultados.paf text (with_paf): bytes or HostText
    screen: Optional[list] = None      # per DB, the ScreenResult (shared / median arrays)

    @property
    def paf_bytes(self) -> Optional[bytes]:
        t = self.paf_text
        return t.bytes() if isinstance(t, HostText) else t

    @property
    def paf(self) -> Optional[List[str]]:
        if self.paf_bytes is None:
            return None
        return self.paf_bytes.decode().split("\n")[:-1] if self.paf_bytes else []


class PafAcc:
    """hymet_paf_acc: the run's resultados.paf as records in HBM."""

    def __init__(self, gpu):
        self.gpu = gpu
        h = _c.c_void_p()
        check(gpu.lib.hymet_paf_acc_create(gpu.ctx, _c.byref(h)), "hymet_paf_acc_create")
        self.h = h

    def reset(self):
        check(self.gpu.lib.hymet_paf_acc_reset(self.h), "hymet_paf_acc_reset")

    @property
    def n(self) -> int:
        n = _c.c_int64()
        check(self.gpu.lib.hymet_paf_acc_info(self.h, _c.byref(n), None, None, None, None, None), "hymet_paf_acc_info")
        return n.value

    def columns(self):
        """(query, part, target) index of every line in PAF order (host; the rare fallback)."""
        n = self.n
        q, part, t = (np.zeros(max(n, 1), np.int32) for _ in range(3))
        check(self.gpu.lib.hymet_paf_acc_copy(self.gpu.ctx, self.h, q.ctypes.data_as(_c.c_void_p),
                                              part.ctypes.data_as(_c.c_void_p), t.ctypes.data_as(_c.c_void_p)),
              "hymet_paf_acc_copy")
        return q[:n], part[:n], t[:n]

    def close(self):
        if getattr(self, "h", None):
            self.gpu.lib.hymet_paf_acc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def make_index_set(gpu, names, lens, parts, first) -> IndexSet:
    """An index set ready to map: a fresh `minimap2 -x asm10` process per run resolves
    mid_occ from the first part of THIS index (options.c mm_mapopt_update), so the options
    live with the set; target names and lengths go to HBM for the PAF writer."""
    torch = gpu.torch
    opt = mp.MapOpt.asm10()
    opt.resolve_mid_occ(parts[0])
    ix = IndexSet(list(names), np.asarray(lens, np.int64), list(parts), list(first), opt)
    tb = [n.encode() for n in ix.names]
    toff = np.zeros(len(tb) + 1, np.int64)
    np.cumsum([len(b) for b in tb], out=toff[1:])
    ix.dev = {"tname": torch.frombuffer(bytearray(b"".join(tb) or b"\0"), dtype=torch.uint8).to(gpu.dev),
              "tname_off": torch.from_numpy(toff).to(gpu.dev),
              "tlen": torch.from_numpy(ix.lens.copy()).to(gpu.dev)}
    return ix


def map_shard(gpu, ix: IndexSet, sh: QueryShard, acc: PafAcc) -> int:
    """minimap2 -x asm10 of every query batch against every part, appended to the device
    PAF in minimap2's order (part-major, queries in input order)."""
    acc.reset()
    starts = np.ascontiguousarray(sh.starts, np.int64)
    lens = np.ascontiguousarray(sh.lengths, np.int64)
    hbase = sh.name_hash.data_ptr()
    for pi, part in enumerate(ix.parts):
        for b0, b1 in sh.batches:
            n = b1 - b0
            if n <= 0:
                continue
            gpu.call("hymet_mm_map_acc", part.h, _c.byref(ix.opt), ptr(sh.mm.w2b), ptr(sh.mm.wmask),
                     _c.c_void_p(starts.ctypes.data + 8 * b0), _c.c_void_p(lens.ctypes.data + 8 * b0),
                     _c.c_void_p(hbase + 4 * b0), n, b0, pi, ix.part_first[pi], acc.h)
    return acc.n


def map_shard_streams(gpus, accs, ix: IndexSet, sh: QueryShard, acc: PafAcc) -> int:
    """map_shard with the part x batch calls spread over several library contexts, each on
    its own HIP stream and host thread (ctypes releases the GIL): one batch's host
    synchronisations, small kernels and chaining tail overlap another batch's kernels.  Each
    worker appends to its own accumulator; the segments are then concatenated into `acc`
    in minimap2's order (part-major, batch order)."""
    import threading
    tasks = [(pi, b0, b1) for pi in range(len(ix.parts)) for b0, b1 in sh.batches if b1 > b0]
    segs = [None] * len(tasks)
    errs = []
    starts = np.ascontiguousarray(sh.starts, np.int64)
    lens = np.ascontiguousarray(sh.lengths, np.int64)
    hbase = sh.name_hash.data_ptr()

    def work(w):
        g, a = gpus[w], accs[w]
        try:
            a.reset()
            for ti in range(w, len(tasks), len(gpus)):
                pi, b0, b1 = tasks[ti]
                before = a.n
                g.call("hymet_mm_map_acc", ix.parts[pi].h, _c.byref(ix.opt), ptr(sh.mm.w2b), ptr(sh.mm.wmask),
                       _c.c_void_p(starts.ctypes.data + 8 * b0), _c.c_void_p(lens.ctypes.data + 8 * b0),
                       _c.c_void_p(hbase + 4 * b0), b1 - b0, b0, pi, ix.part_first[pi], a.h)
                segs[ti] = (w, before, a.n)
        except Exception as e:  # noqa: BLE001 -- re-raised on the calling thread
            errs.append(e)

    th = [threading.Thread(target=work, args=(w,)) for w in range(len(gpus))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    acc.reset()
    g0 = acc.gpu
    for w, b, e in segs:
        g0.call("hymet_paf_acc_append", acc.h, accs[w].h, b, e)
    return acc.n


def _dev_buf(gpu, bufs, key, nbytes):
    """A reusable device byte buffer of at least nbytes."""
    b = bufs.get(key)
    if b is None or b.numel() < nbytes:
        bufs.pop(key, None)
        b = gpu.empty(max(int(nbytes), 16), gpu.torch.uint8)
        bufs[key] = b
    return b


_bytes_new = _c.pythonapi.PyBytes_FromStringAndSize
_bytes_new.restype = _c.py_object
_bytes_new.argtypes = [_c.c_void_p, _c.c_ssize_t]


def _to_host(gpu, bufs, key, dev, n, prefix: bytes = b"") -> bytes:
    """prefix + n bytes of device memory, as a new bytes object filled through the library's
    double-buffered pinned staging (16 host copy threads): no torch pinned buffer and no
    extra bytes copy (a copy cost ~0.35 s per GB of PAF text; prefix + text would be one)."""
    if n == 0:
        return bytes(prefix)
    m = len(prefix)
    b = _bytes_new(None, int(n) + m)  # uninitialised, filled below before anyone sees it
    addr = _c.cast(_c.c_char_p(b), _c.c_void_p).value
    if m:
        _c.memmove(addr, prefix, m)
    check(gpu.lib.hymet_copy_to_host(gpu.ctx, addr + m, ptr(dev), int(n), 16), "hymet_copy_to_host")
    return b


def emit_paf_bytes(gpu, ix: IndexSet, sh: QueryShard, acc: PafAcc, bufs) -> bytes:
    """resultados.paf text of the accumulator (written on the device, copied out once)."""
    n = acc.n
    if n == 0:
        return b""
    nb = _c.c_int64()
    cap = 200 * n
    while True:
        out = _dev_buf(gpu, bufs, "paf", cap)
        rc = gpu.lib.hymet_emit_paf(gpu.ctx, acc.h, ptr(sh.qname), ptr(sh.qname_off), ptr(sh.qlen), ptr(ix.dev["tname"]),
                                    ptr(ix.dev["tname_off"]), ptr(ix.dev["tlen"]), ptr(out), cap, _c.byref(nb), None)
        if rc == -3:
            cap = nb.value
            continue
        check(rc, "hymet_emit_paf")
        break
    return _to_host(gpu, bufs, "paf_h", out, nb.value)


def run_beside(loader, main):
    """main() on this thread while loader() (or nothing, when None) runs on a second host
    thread; the loader is joined before main's result is returned, and an exception of either
    is re-raised here (main's first).  Pipeline.run's placement of the per-run input loads:
    the loader may issue collectives (holding the communicator, Comm.owned); main may not --
    the caller issues its collectives after this returns."""
    if loader is None:
        return main()
    import threading
    err = []

    def body():
        try:
            loader()
        except BaseException as e:  # noqa: BLE001 -- re-raised on the calling thread
            err.append(e)
    th = threading.Thread(target=body, name="hymet-inputs")
    th.start()
    try:
        out = main()
    finally:
        th.join()
    if err:
        raise err[0]
    return out


class Pipeline:
    def __init__(self, gpu, dbs: Sequence[SketchDB], ref_lookup, taxonomy, hierarchy, cfg: Config = None, comm=None,
                 variant: int = cls.CAMI):
        """ref_lookup(names) -> SeqSet of the candidate genomes in combined_genomes.fasta
        order (the download cache; scripts/downloadDB.py is outside the accelerated path)."""
        """dbs: SketchDB objects (tables built once) or .msh paths (read by the native
        reader and rebuilt into HBM tables on every run when cfg.reload_inputs, as `mash
        screen` reads its DB per call)."""
        self.gpu, self.cfg, self.comm = gpu, cfg or Config(), comm
        self.db_paths = [str(d) for d in dbs] if dbs and all(isinstance(d, (str, os.PathLike)) for d in dbs) else None
        self.dbs = [] if self.db_paths else list(dbs)
        self.tables = [scr.ScreenTable(gpu, db) for db in self.dbs]
        self.ref_lookup = ref_lookup
        self.taxonomy, self.hierarchy, self.variant = taxonomy, hierarchy, variant
        self.timings: Dict[str, float] = {}   # host wall seconds of the last run's input loads
        self._pin: Dict[int, object] = {}     # pinned host buffers of the DB hashes (S1 upload)
        self._load_classifier()
        if self.db_paths:
            self._load_dbs()
        self.index_cache: Dict[str, IndexSet] = {}
        self.opt: Optional[mp.MapOpt] = None
        self.acc = PafAcc(gpu)
        self.map_gpus = [gpu.fork() for _ in range(self.cfg.map_streams)] if self.cfg.map_streams > 1 else []
        self.map_accs = [PafAcc(g) for g in self.map_gpus]
        self._bufs: Dict[str, object] = {}
        self._paf_pin = [None, None]          # pinned host buffers of the PAF text, alternating per run
        self._paf_holders = [None, None]      # weak refs to the HostText living in each
        self._ran = False   # the constructor's loads serve the first run

    def _pinned_hashes(self, i, n):
        """Reusable pinned host buffer for DB i's hashes (grown, never shrunk)."""
        torch = self.gpu.torch
        b = self._pin.get(i)
        if b is None or b.numel() < n:
            b = torch.empty(int(n), dtype=torch.int64, pin_memory=True)
            self._pin[i] = b
        return b

    def _load_dbs(self):
        """S1: each sketch DB file parsed (csrc/msh.cpp), its hashes gathered into pinned
        memory and uploaded by DMA, and its hash table built in HBM.  The pinned buffers are
        reused run after run, so the SketchDB.hashes of a path-built Pipeline (and of its
        RunResult.screen) are valid until the next run.  The previous tables are released
        before the new ones are built (no second copy of the tables in HBM)."""
        self._read_dbs()
        self._build_tables()

    def _read_dbs(self, side=None):
        """S1 host part: the .msh files parsed and their hashes gathered into pinned memory
        (run() does it on a second host thread while the contigs are ingested).  With `side`
        (an idle mapping context) the gather goes in chunks whose DMAs into HBM are queued on
        side's stream as each chunk is gathered (hymet_msh_upload), so the table build that
        follows finds the hashes in HBM instead of uploading them after the gather."""
        self.tables, self.dbs = [], []
        t0 = time.perf_counter()
        dbs = []
        # more than one rank: this rank gathers and uploads only its slice of each DB's
        # hashes; run() all-gathers the slices over xGMI (_join_slices) before the tables
        shard = (self.rank, self.world) if side is not None and self.world > 1 else None
        for i, p in enumerate(self.db_paths):
            pin = lambda n, i=i: self._pinned_hashes(i, n).numpy().view(np.uint64)[:n]   # noqa: E731
            if side is None:
                dbs.append(read_msh(p, alloc=pin))
            else:
                with self.gpu.torch.cuda.stream(side.stream):
                    dbs.append(read_msh(p, alloc=pin, upload=(side, lambda n: side.empty(n, side.torch.int64)),
                                        shard=shard, defer_meta=True))
        self.dbs = dbs
        self.timings["msh_read_s"] = time.perf_counter() - t0
        for k in ("open", "meta", "hashes"):    # read_msh's own phases, summed over the DBs
            self.timings[f"msh_{k}_s"] = sum(getattr(db, "load_s", {}).get(k, 0.0) for db in dbs)

    def _build_tables(self, side=None):
        """S1 device part: the pinned hashes uploaded by DMA and the HBM tables built -- on
        this context's stream, or on `side` (an idle mapping context, from the loader thread,
        overlapping the ingest; that thread waits for side's stream before run() joins it)."""
        t1 = time.perf_counter()
        if side is None:
            self._finish_meta()
            self.tables = [scr.ScreenTable(self.gpu, db, pinned=self._pin[i]) for i, db in enumerate(self.dbs)]
            self.gpu.sync()
        else:
            with self.gpu.torch.cuda.stream(side.stream):
                self.tables = [scr.ScreenTable(side, db, pinned=self._pin[i]) for i, db in enumerate(self.dbs)]
            self.timings["screen_table_enqueue_s"] = time.perf_counter() - t1
            self._finish_meta()        # the DBs' names copied while the GPU inserts the hashes
            side.stream.synchronize()
        self.timings["screen_table_s"] = time.perf_counter() - t1

    def _finish_meta(self):
        """Names / comments of DBs read with defer_meta (closes their files)."""
        for db in self.dbs:
            if getattr(db, "finish_meta", None) is not None:
                db.finish_meta()

    def _read_inputs(self, side=None):
        """The run's input loads for a second host thread: .msh parse (+ the HBM tables on
        `side`'s stream when given), and the taxonomy tables on a third thread beside them
        (the .msh gather runs in native code without the GIL, so the two overlap)."""
        import threading
        err = []

        def classifier():
            try:
                self._load_classifier(side)
            except BaseException as e:  # noqa: BLE001 -- re-raised below
                err.append(e)
        th = threading.Thread(target=classifier, name="hymet-taxonomy")
        th.start()
        try:
            if self.db_paths:
                self._read_dbs(side)
                if side is not None and self._sliced():
                    if not self._db_gather_main():
                        self._join_slices(side)
                elif side is not None:
                    self._build_tables(side)
        finally:
            self._finish_meta()        # (a no-op unless an error cut the build short)
            th.join()
        if err:
            raise err[0]

    def _sliced(self):
        return any(getattr(db, "dev_slice", None) is not None for db in self.dbs)

    @staticmethod
    def _db_gather_main() -> bool:
        """HYMET_DB_GATHER=main: all-gather the DB slices and build the tables on the calling
        thread after the ingest (one thread issuing every collective) instead of on the loader
        thread beside it -- the fallback if concurrent collectives on two communicators ever
        misbehave on a multi-GPU node (about 8 ms more per rank step at N = 8)."""
        return os.environ.get("HYMET_DB_GATHER", "loader") == "main"

    def _join_slices(self, side):
        """The DBs' hash slices all-gathered on side's stream (behind this rank's DMAs), then
        the tables built there -- on the loader thread, overlapping the contigs' ingest (or,
        with HYMET_DB_GATHER=main, on the calling thread after it).  The all-gathers go over
        the communicator Comm keeps for the DB load alone (Comm.db_group), and this thread holds
        the communicator (Comm.owned) until they have completed on the GPU: run() issues no
        collective before it has joined the loader thread (ingest() defers its record-count
        all-gather), so every rank's collectives form one sequence."""
        t0 = time.perf_counter()
        with self.comm.owned():
            with self.gpu.torch.cuda.stream(side.stream):
                for i, db in enumerate(self.dbs):
                    if db.dev_slice is not None and db.dev_hashes is not None:
                        self.comm.allgather_slices_(db.dev_hashes, db.dev_slice[2], key=i)
            self.timings["msh_allgather_s"] = time.perf_counter() - t0
            self._build_tables(side)          # ends in side.stream.synchronize(): the gathers are done

    def _load_classifier(self, side=None):
        """C1-C2: detailed_taxonomy.tsv and taxonomy_hierarchy.tsv.  classification_cami.py
        runs as `... || true` (run_hymet_cami.sh:175-180): a classifier that cannot load its
        inputs leaves an empty TSV, and the fallback runs."""
        t0 = time.perf_counter()
        try:
            self.classifier = cls.Classifier(self.gpu, self.taxonomy, self.hierarchy, self.variant)
            self.classifier_error = None
        except Exception as e:  # noqa: BLE001 -- any failure of the reference script
            self.classifier, self.classifier_error = None, e
        if self.classifier is not None and side is not None:
            # the taxonomy's HBM tables (labels, name ids, hierarchy flags) on this loader
            # thread, on the idle mapping stream, rather than in the run's classification
            # step.  No stream of its own: a process's streams share a few hardware queues
            # (GPU_MAX_HW_QUEUES, 4), and one more stream shifted the round-robin so that the
            # two mapping streams landed on one queue and ran one after the other (C4 step
            # 1,298 -> 1,388 ms)
            torch = self.gpu.torch
            with torch.cuda.stream(side.stream):
                self.classifier.device_tables(None)
            side.stream.synchronize()
        self.timings["classifier_load_s"] = time.perf_counter() - t0

    def load_inputs(self):
        """The per-run input loads of the reference's stage processes (Config.reload_inputs)."""
        if self.db_paths:
            self._load_dbs()
        self._load_classifier()

    @property
    def world(self) -> int:
        return self.comm.world if self.comm is not None else 1

    @property
    def rank(self) -> int:
        return self.comm.rank if self.comm is not None else 0

    # ------------------------------------------------------------------ stages
    def ingest(self, queries, defer_base: bool = False) -> QueryShard:
        """FASTA bytes / FastaIndex (this rank's contiguous record range) or a SeqSet (one
        rank) -> QueryShard resident in HBM.  defer_base (run(), while the loader thread may
        hold the communicator): a byte-range shard's first query index is left pending
        (q_base None) for shard_base() to all-gather once the loader has been joined."""
        if isinstance(queries, QueryShard):
            return queries
        d_all = None
        if isinstance(queries, (bytes, bytearray, memoryview)):
            data = bytes(queries)
            if self.world > 1:
                # this rank scans, uploads and maps only its byte range of the FASTA; the ranks'
                # record counts give its first query's index in the whole input
                b0, b1 = shard_bytes(data, self.rank, self.world)
                d_rng, fx = self._upload_while(data, b0, b1, lambda: FastaIndex(data, byte_range=(b0, b1)))
                sh = QueryShard.from_fasta(self.gpu, fx, 0, fx.n, self.cfg.map_batch_bases, q_base=0,
                                           d_all=d_rng, d_base=b0)
                sh.fasta, sh.fasta_r0 = fx, 0
                # every rank of a byte-sharded run takes this branch, whatever its range holds
                # (one rank may get the whole file, another nothing): the name-pool gather of
                # _global_names keys on this flag, never on the range, so all ranks join it
                sh.byte_sharded = True
                sh.q_base = None
                if not defer_base:
                    self.shard_base(sh)
                return sh
            if len(data):
                # one rank takes every record: the bytes go up while the record table is scanned
                d_all, queries = self._upload_while(data, 0, len(data), lambda: FastaIndex(data))
            else:
                queries = FastaIndex(data)
        if isinstance(queries, FastaIndex):
            r0, r1 = queries.shard(self.rank, self.world)
            sh = QueryShard.from_fasta(self.gpu, queries, r0, r1, self.cfg.map_batch_bases,
                                       d_all=d_all if (r0, r1) == (0, queries.n) else None)
            sh.fasta, sh.fasta_r0 = queries, r0
            return sh
        if isinstance(queries, SeqSet):
            if self.world > 1:
                raise ValueError("multi-rank runs take the FASTA bytes (every rank shards the same input)")
            return QueryShard.from_seqset(self.gpu, queries, 0, self.cfg.map_batch_bases)
        raise TypeError(f"unsupported query input {type(queries)!r}")

    prepare = ingest

    def shard_base(self, sh: QueryShard) -> int:
        """A byte-range shard's first query index in the whole input: the ranks' record counts
        all-gathered (a collective; every rank of a byte-sharded run calls it once)."""
        if sh.q_base is None:
            counts = self.comm.allgather_np(np.array([sh.n], np.int64), tag="shard_records")
            sh.q_base = int(sum(int(c[0]) for c in counts[:self.rank]))
        return sh.q_base

    def _upload_while(self, data: bytes, b0: int, b1: int, scan):
        """Bytes [b0, b1) of data uploaded to HBM on a second thread (the library's staged,
        threaded copy) while scan() runs on this one (the record scan: both read host memory,
        neither holds the GIL).  Returns (device bytes, scan())."""
        import threading
        torch = self.gpu.torch
        d = self.gpu.empty(max(b1 - b0, 1), torch.uint8)
        up_err = []

        def upload():
            try:
                if b1 > b0:
                    src = ctypes.cast(ctypes.c_char_p(data), ctypes.c_void_p).value + b0
                    check(self.gpu.lib.hymet_copy_to_device(self.gpu.ctx, ptr(d), ctypes.c_void_p(src), b1 - b0, 16),
                          "hymet_copy_to_device")
            except BaseException as e:  # noqa: BLE001 -- re-raised below
                up_err.append(e)
        up = threading.Thread(target=upload, name="hymet-upload")
        up.start()
        try:
            out = scan()
        finally:
            up.join()
        if up_err:
            raise up_err[0]
        return d, out

    def screen_select(self, pool):
        t0 = time.perf_counter()
        res = scr.screen(self.gpu, pool, self.dbs, self.tables, self.comm)
        self.last_screen = res
        ph = getattr(self, "phases", None)
        if ph is not None:                    # the screen's share of run()'s screen_select_s
            ph["screen_only_s"] = ph.get("screen_only_s", 0.0) + time.perf_counter() - t0
        rows, thr, selections = [], [], []
        for r in res:
            s = sel.sort_gr(sel.sort_unique_k5(r.lines(v_max=0.9)))
            t, top, names = sel.select_threshold(s, self.cfg.mash_thresh, self.cfg.n_input_files)
            rows.append(s)
            thr.append(t)
            selections.append(names)
        selected = sel.union_sorted(*selections)
        if not self.cfg.limit:            # main.pl:94-104: the sort -u union goes to downloadDB.py
            return selected, rows, thr
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
        ix = make_index_set(self.gpu, list(refs.names), refs.lengths, parts, first)
        self.index_cache = {key: ix}  # one cached candidate set, like the sha1 cache dir
        return ix

    def map_all(self, ix: IndexSet, sh: QueryShard) -> int:
        self.opt = ix.opt
        if self.map_gpus:
            self.gpu.sync()  # the shard's pools were written on this context's stream
            return map_shard_streams(self.map_gpus, self.map_accs, ix, sh, self.acc)
        return map_shard(self.gpu, ix, sh, self.acc)

    def classify_rows(self, ix: IndexSet, sh: QueryShard):
        """ref_counts (all-reduced) + device LCA over the accumulator -> row tensors."""
        gpu, torch = self.gpu, self.gpu.torch
        tabs = self.classifier.device_tables(ix.names)
        counts = gpu.zeros(max(len(ix.names), 1), torch.int32)
        gpu.call("hymet_acc_ref_counts", self.acc.h, ptr(counts))
        if self.world > 1:
            self.comm.allreduce_sum_(counts)
        n_q = max(sh.n, 1)
        rq, rp, rd, rt = (gpu.zeros(n_q, torch.int32) for _ in range(4))
        rn = gpu.zeros(n_q * 8, torch.int32)
        rc = gpu.zeros(n_q, torch.float64)
        nr = _c.c_int32()
        legacy = self.variant == cls.LEGACY
        gpu.call("hymet_acc_classify", self.acc.h, self.variant, sh.n, ptr(sh.qlen), ptr(counts), ptr(tabs["t_tax"]),
                 ptr(tabs["tax_names"]), ptr(tabs["in_hier"]), ptr(sh.qname) if legacy else None,
                 ptr(sh.qname_off) if legacy else None, ptr(ix.dev["tname"]) if legacy else None,
                 ptr(ix.dev["tname_off"]) if legacy else None, ptr(rq), ptr(rp), ptr(rd), ptr(rn), ptr(rc), ptr(rt),
                 _c.byref(nr))
        R = nr.value
        return {"q": rq[:R], "part": rp[:R], "depth": rd[:R], "names": rn[:R * 8], "conf": rc[:R], "tax": rt[:R]}, R

    def emit_tsv(self, rows, R, qname, qname_off) -> bytes:
        gpu = self.gpu
        tabs = self.classifier.device_tables(None)
        legacy = self.variant == cls.LEGACY
        nb = _c.c_int64()
        cap = max(256 * R, 1 << 16)
        while True:
            out = self._dev_buf("tsv", cap)
            rc = gpu.lib.hymet_emit_tsv(gpu.ctx, self.variant, R, ptr(rows["q"]), ptr(rows["depth"]), ptr(rows["names"]),
                                        ptr(rows["conf"]), ptr(rows["tax"]), ptr(qname), ptr(qname_off), ptr(tabs["label"]),
                                        ptr(tabs["label_off"]), ptr(tabs["taxlin"]) if legacy else None,
                                        ptr(tabs["taxlin_off"]) if legacy else None,
                                        ptr(tabs["taxlvl"]) if legacy else None,
                                        ptr(tabs["taxlvl_off"]) if legacy else None, ptr(out), cap, _c.byref(nb))
            if rc == -3:
                cap = nb.value
                continue
            check(rc, "hymet_emit_tsv")
            break
        return self._to_host("tsv_h", out, nb.value, prefix=TSV_HEADER)

    def emit_paf(self, ix: IndexSet, sh: QueryShard) -> HostText:
        """This rank's resultados.paf text (its queries' lines, part-major), written on the
        device and landed in pinned host memory by one DMA."""
        gpu, torch = self.gpu, self.gpu.torch
        if getattr(self, "_paf_copy", None) is not None:  # a run that raised after its copy was issued
            self._paf_copy.synchronize()
            self._paf_copy = None
        n = self.acc.n
        if n == 0:
            return HostText(b"", 0)
        nb = _c.c_int64()
        cap = 200 * n
        while True:
            out = self._dev_buf("paf", cap)
            rc = gpu.lib.hymet_emit_paf(gpu.ctx, self.acc.h, ptr(sh.qname), ptr(sh.qname_off), ptr(sh.qlen),
                                        ptr(ix.dev["tname"]), ptr(ix.dev["tname_off"]), ptr(ix.dev["tlen"]), ptr(out), cap,
                                        _c.byref(nb), None)
            if rc == -3:
                cap = nb.value
                continue
            check(rc, "hymet_emit_paf")
            break
        m = nb.value
        slot = self._paf_slot = (getattr(self, "_paf_slot", 1) + 1) % 2
        holder = self._paf_holders[slot]() if self._paf_holders[slot] is not None else None
        if holder is not None:
            holder.detach()                       # an earlier result still holds this buffer's text
        buf = self._paf_pin[slot]
        if buf is None or buf.numel() < m:
            # both slots at once (pinning ~1.5 GB costs ~0.4 s): the first run with the PAF
            # text pays for both, not the first two
            for s_ in (slot, 1 - slot):
                b_ = self._paf_pin[s_]
                if b_ is None or b_.numel() < m:
                    h_ = self._paf_holders[s_]() if self._paf_holders[s_] is not None else None
                    if h_ is not None:
                        h_.detach()
                    self._paf_pin[s_] = None      # release before allocating the larger one
                    self._paf_pin[s_] = torch.empty(int(m * 1.25) + 4096, dtype=torch.uint8, pin_memory=True)
            buf = self._paf_pin[slot]
        if self.map_gpus:
            # one D2H DMA into pinned memory on an idle mapping stream, after the text kernels
            # (an event on this stream), overlapping the classification; run() waits for it
            side = self.map_gpus[0].stream
            ev = torch.cuda.Event()
            ev.record(gpu.bound_stream)          # the stream hymet_emit_paf wrote the text on
            side.wait_event(ev)
            with torch.cuda.stream(side):
                buf[:m].copy_(out[:m], non_blocking=True)
            self._paf_copy = side
        else:
            gpu.sync()                            # the text was written on the library's stream
            buf[:m].copy_(out[:m])                # one D2H DMA into pinned memory (synchronous)
        t = HostText(buf.numpy(), m)
        import weakref
        self._paf_holders[slot] = weakref.ref(t)
        return t

    def _dev_buf(self, key, nbytes):
        return _dev_buf(self.gpu, self._bufs, key, nbytes)

    def _to_host(self, key, dev, n, prefix: bytes = b"") -> bytes:
        return _to_host(self.gpu, self._bufs, key, dev, n, prefix)

    # ------------------------------------------------------------------- run
    def run(self, queries, with_paf=False) -> RunResult:
        """queries: FASTA bytes, a FastaIndex, a SeqSet, or a QueryShard already resident.
        Rank 0's RunResult.tsv is the whole classified_sequences.tsv."""
        side = self.map_gpus[0] if self.map_gpus else None
        reader = self.cfg.reload_inputs and self._ran
        self._ran = True
        ph = self.phases = {}   # host wall seconds of the run's phases (bench.py --emulate-rank)
        tp = [time.perf_counter()]

        def lap(name):
            t = time.perf_counter()
            ph[name] = ph.get(name, 0.0) + t - tp[0]
            tp[0] = t

        def read():
            t0 = time.perf_counter()
            try:
                self._read_inputs(side)
            finally:
                self.timings["reader_s"] = time.perf_counter() - t0

        def ingest():
            sh_ = self.ingest(queries, defer_base=True)
            lap("ingest_s")
            return sh_
        # the input loads (.msh parse into pinned memory and, with a mapping context to spare,
        # the DB all-gathers and HBM tables on its stream; taxonomy tables) overlap the
        # contigs' ingest, which issues no collective meanwhile
        sh = run_beside(read if reader else None, ingest)
        lap("input_wait_s")                   # the loader thread's remainder after the ingest
        if getattr(sh, "byte_sharded", False):
            self.shard_base(sh)               # the record-count all-gather, now that the loader is done
        if reader and self.db_paths and side is None:
            self._build_tables()
        elif reader and side is not None and not self.tables and self._sliced():
            self._join_slices(side)           # HYMET_DB_GATHER=main
            lap("db_join_s")
        selected, rows, thr = self.screen_select(sh.mash)
        if not selected:
            raise RuntimeError("candidate list empty after applying limit")  # run_hymet_cami.sh:126
        lap("screen_select_s")
        ix = self.index_for(selected)
        n_lines = self.map_all(ix, sh)
        lap("map_s")
        paf_text = self.emit_paf(ix, sh) if with_paf else None
        lap("emit_paf_s")
        tsv, n_rows, n_cls = b"", 0, 0
        if self.classifier is not None:
            rws, R = self.classify_rows(ix, sh)
            lap("classify_s")
            if self.world > 1:
                rws, R = self.comm.gather_rows(rws, sh.q_base, self.gpu)
                qname, qname_off = self._global_names(sh)
            else:
                qname, qname_off = sh.qname, sh.qname_off
            lap("gather_rows_s")
            if self.rank == 0:
                tsv = self.emit_tsv(rws, R, qname, qname_off)
                n_rows = R
                n_cls = int((rws["depth"] != 0).sum().item()) if R else 0
            lap("emit_tsv_s")
        total_rows = self.comm.broadcast_obj(n_rows) if self.world > 1 else n_rows
        if total_rows < 1:  # fewer than 2 TSV lines: run_hymet_cami.sh:182-206
            tsv = self._fallback(ix, sh)
            n_rows = n_cls = 0
        if getattr(self, "_paf_copy", None) is not None:
            self._paf_copy.synchronize()          # the PAF text has landed in host memory
            self._paf_copy = None
        lap("finish_s")
        return RunResult(selected, rows, thr, tsv, n_rows, n_cls, n_lines, paf_text, self.last_screen)

    def _global_names(self, sh: QueryShard):
        """Rank 0's name pool of the whole input (rows from every rank index into it): the
        ranks' pools gathered (a byte-range shard indexes only its own records), or the
        whole-file record table's names.  A collective: every rank calls it."""
        fx = sh.fasta
        if getattr(sh, "byte_sharded", False):
            return self.comm.gather_name_pools(sh.qname, sh.qname_off, sh.n)
        if self._bufs.get("names_of") is not fx:
            torch = self.gpu.torch
            pool, off = fx.name_pool()
            self._bufs["names"] = (torch.from_numpy(pool.copy() if len(pool) else np.zeros(1, np.uint8)).to(self.gpu.dev),
                                   torch.from_numpy(off).to(self.gpu.dev))
            self._bufs["names_of"] = fx
        return self._bufs["names"]

    def _fallback(self, ix: IndexSet, sh: QueryShard) -> bytes:
        """build_id_map + mini_classify over the PAF lines (first mapped hit per query), then
        the awk rewrite; dies like the script when even that leaves no row."""
        from . import fallback
        q, part, t = self.acc.columns()
        if sh.names_host is not None:
            names = sh.names_host
        else:
            names = sh.fasta.names()[sh.fasta_r0:sh.fasta_r0 + sh.n]
        pairs = [(names[int(a)], ix.names[int(b)]) for a, b in zip(q, t)]
        if self.world > 1:
            # lines of a query sit together per part; queries sort by (part, input index)
            got = self.comm.gather_obj([(int(p_), sh.q_base + int(a), j, pa[0], pa[1])
                                        for j, (p_, a, pa) in enumerate(zip(part, q, pairs))])
            if self.rank != 0:
                return b""
            pairs = [(x[3], x[4]) for x in sorted(y for g in got for y in g)]
        tsv = fallback.fallback_tsv(pairs, self.taxonomy)
        if tsv.count(b"\n") < 2:
            raise RuntimeError("classification still empty after fallback")  # run_hymet_cami.sh:205
        return tsv

"""Process-group plumbing for the multi-GPU path.

One process per GPU, torch.distributed over RCCL ("nccl" backend = RCCL on ROCm, xGMI
inside a node) or gloo on CPU for the tests.  The path shards by contig / k-mer position
with three exchange steps: the screen hit counts (all-reduce, uint32 sum), the per-target
PAF-line counts (all-reduce, int32 sum) and the per-contig results (gather to rank 0).
"""
from __future__ import annotations

import contextlib
import os
import threading
from typing import List, Sequence

import numpy as np


class Comm:
    """Collectives of one rank.  Invariant: at any moment ONE host thread issues collectives.
    The per-run DB load (Pipeline's loader thread) takes the communicator with `owned()` for
    the whole of its all-gathers and the table build behind them, and the calling thread
    issues no collective until it has joined the loader; `_check_owner` turns any breach of
    that order into an error instead of an RCCL deadlock (NCCL/RCCL guarantee progress only
    when every rank issues its collectives in one order)."""

    def __init__(self, rank: int = 0, world: int = 1, replicated_pool: bool = False):
        """replicated_pool: every rank holds the same contig pool (the screen then splits
        k-mer positions); otherwise (default) each rank's pool is its own contig shard."""
        self.rank, self.world = rank, world
        self.replicated_pool = replicated_pool
        self.dist = None
        self.device = None
        self.db_group = None
        self._owner = None          # thread ident holding the communicator (owned()), else None

    @contextlib.contextmanager
    def owned(self):
        """This thread alone may issue collectives until the block ends (the loader thread's
        DB all-gathers: the block also covers the stream synchronisation behind them, so no
        collective of theirs is still running on the GPU when another thread's is issued)."""
        me = threading.get_ident()
        if self._owner is not None and self._owner != me:
            raise RuntimeError("Comm.owned: another thread holds the communicator")
        prev, self._owner = self._owner, me
        try:
            yield self
        finally:
            self._owner = prev

    def _check_owner(self):
        o = self._owner
        if o is not None and o != threading.get_ident():
            raise RuntimeError("collective issued while another thread holds the communicator "
                               "(two threads' collectives could interleave differently per rank)")

    @classmethod
    def from_env(cls) -> "Comm":
        return cls(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")))

    def init_backend(self, gpu=None, backend: str = None):
        if self.world <= 1:
            return self
        import torch
        import torch.distributed as dist
        if not dist.is_initialized():
            if backend is None:
                backend = "nccl" if gpu is not None else "gloo"
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            kw = {}
            if backend == "nccl" and gpu is not None:
                kw["device_id"] = gpu.dev
            dist.init_process_group(backend, rank=self.rank, world_size=self.world, **kw)
        # a second communicator over the same ranks for the per-run DB load (the loader
        # thread's all-gathers, while it holds the communicator: owned())
        self.db_group = dist.new_group(list(range(self.world)))
        self.dist = dist
        self.device = gpu.dev if gpu is not None else torch.device("cpu")
        self.torch = torch
        # both communicators created now, on this thread and in this order on every rank (RCCL
        # would otherwise create db_group's lazily, on the loader thread, at its first use)
        on_dev = dist.get_backend() == "nccl"
        for g in (None, self.db_group):
            t = torch.zeros(1, dtype=torch.int32, device=self.device if on_dev else "cpu")
            dist.all_reduce(t, group=g)
        if on_dev:
            torch.cuda.synchronize(self.device)
        return self

    # ------------------------------------------------------------- partitioning
    def shard_range(self, n: int):
        """Contiguous, balanced [begin, end) slice of n items for this rank."""
        b = n * self.rank // self.world
        e = n * (self.rank + 1) // self.world
        return b, e

    @staticmethod
    def partition_by_length(lengths: Sequence[int], world: int) -> List[np.ndarray]:
        """Greedy longest-first assignment of items to `world` bins by total length
        (SURVEY.md §8e step 1).  Returns the item indices of each bin, sorted."""
        lengths = np.asarray(lengths, dtype=np.int64)
        order = np.argsort(-lengths, kind="stable")
        load = np.zeros(world, dtype=np.int64)
        bins = [[] for _ in range(world)]
        for i in order:
            b = int(np.argmin(load))
            bins[b].append(int(i))
            load[b] += lengths[i]
        return [np.array(sorted(b), dtype=np.int64) for b in bins]

    # -------------------------------------------------------------- collectives
    def _staged(self, t):
        """gloo works on host tensors: device tensors travel through a host copy (the
        multi-process tests run several ranks on one GPU this way); RCCL takes them as is."""
        return self.dist.get_backend() == "gloo" and t.is_cuda

    def allreduce_sum_(self, t):
        if self.world > 1:
            self._check_owner()
            if self._staged(t):
                h = t.cpu()
                self.dist.all_reduce(h, op=self.dist.ReduceOp.SUM)
                t.copy_(h)
            else:
                self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return t

    def all_gather_padded(self, t, n: int):
        """All-gather the first n rows of t (n may differ per rank): rows padded to the
        largest n; returns the list of every rank's first-n slices."""
        torch = self.torch
        self._check_owner()
        ns = [int(x[0]) for x in self.allgather_np(np.array([n], np.int64))]
        m = max(ns) if ns else 0
        pad = torch.zeros((max(m, 1),) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        if n:
            pad[:n].copy_(t[:n])
        src = pad.cpu() if self._staged(pad) else pad
        out = [torch.empty_like(src) for _ in range(self.world)]
        self.dist.all_gather(out, src)
        if src is not pad:
            out = [o.to(t.device) for o in out]
        return [o[:k] for o, k in zip(out, ns)]

    def allgather_slices_(self, t, c: int, key=None):
        """t: a device tensor of world * c entries whose slice [rank * c, (rank + 1) * c) this
        rank filled (its slice of a sketch DB's hashes, read_msh(shard=...)); every other
        rank's slice is filled in place (RCCL all-gather over xGMI) on the DB-load communicator
        (db_group: called from the loader thread).  key names the DB for EmulatedComm."""
        if self.world <= 1:
            return t
        self._check_owner()
        mine = t[self.rank * c:(self.rank + 1) * c]
        if self._staged(t):
            parts = [self.torch.empty(c, dtype=t.dtype) for _ in range(self.world)]
            self.dist.all_gather(parts, mine.cpu(), group=self.db_group)
            t[:self.world * c].copy_(self.torch.cat(parts).to(t.device))
        else:
            self.dist.all_gather_into_tensor(t[:self.world * c], mine, group=self.db_group)
        return t

    def gather_rows(self, rows, q_base: int, gpu=None):
        """every rank's LCA rows (fixed-size records: query index in
        the whole input, index part of its first PAF line, depth, taxid, 8 name ids,
        confidence) are all-gathered over RCCL; rank 0 orders them like the reference's
        output -- minimap2 prints the pooled input part by part, queries in input order
        within a part, and classification_cami.py writes queries in first-appearance order
        (:333-339) -- i.e. by (first part, query index).  Other ranks get empty rows."""
        torch = self.torch
        R = int(rows["q"].shape[0])
        dev = rows["q"].device
        rec = torch.zeros((max(R, 1), 12), dtype=torch.int32, device=dev)
        if R:
            rec[:R, 0] = rows["q"] + int(q_base)
            rec[:R, 1] = rows["part"]
            rec[:R, 2] = rows["depth"]
            rec[:R, 3] = rows["tax"]
            rec[:R, 4:] = rows["names"].view(R, 8)
        recs = self.all_gather_padded(rec, R)
        confs = self.all_gather_padded(rows["conf"], R)
        if self.rank != 0:
            e = torch.zeros(0, dtype=torch.int32, device=dev)
            return {"q": e, "part": e, "depth": e, "tax": e, "names": e,
                    "conf": torch.zeros(0, dtype=torch.float64, device=dev)}, 0
        allr = torch.cat(recs)
        allc = torch.cat(confs)
        key = allr[:, 1].to(torch.int64) * (1 << 32) + allr[:, 0].to(torch.int64)
        order = torch.sort(key, stable=True).indices
        allr, allc = allr[order], allc[order]
        n = int(allr.shape[0])
        return {"q": allr[:, 0].contiguous(), "part": allr[:, 1].contiguous(), "depth": allr[:, 2].contiguous(),
                "tax": allr[:, 3].contiguous(), "names": allr[:, 4:].contiguous().view(-1), "conf": allc.contiguous()}, n

    def gather_name_pools(self, qname, qname_off, n: int):
        """Rank 0: the whole input's query-name pool (uint8) and offsets (int64, n_all + 1) on
        its device, the ranks' shard pools concatenated in rank order (each rank's shard is a
        contiguous record range, so rank order is input order); other ranks get (None, None).
        Two padded all-gathers: name bytes and name starts."""
        torch = self.torch
        nb = int(qname_off[n].item()) if n else 0
        pools = self.all_gather_padded(qname.view(-1), nb)
        starts = self.all_gather_padded(qname_off[:max(n, 1)], n)
        if self.rank != 0:
            return None, None
        base, offs = 0, []
        for p_, o_ in zip(pools, starts):
            offs.append(o_ + base)
            base += int(p_.shape[0])
        dev = qname.device
        pool = torch.cat(pools) if base else torch.zeros(1, dtype=torch.uint8, device=dev)
        off = torch.cat(offs + [torch.tensor([base], dtype=torch.int64, device=dev)])
        return pool.contiguous(), off.contiguous()

    def allgather_np(self, arr: np.ndarray, tag: str = None) -> List[np.ndarray]:
        """All-gather of a small host array (tag names the exchange for EmulatedComm)."""
        if self.world <= 1:
            return [arr]
        self._check_owner()
        objs = [None] * self.world
        self.dist.all_gather_object(objs, np.ascontiguousarray(arr))
        return objs

    def gather_obj(self, obj, dst: int = 0):
        if self.world <= 1:
            return [obj]
        self._check_owner()
        out = [None] * self.world if self.rank == dst else None
        self.dist.gather_object(obj, out, dst=dst)
        return out

    def broadcast_obj(self, obj, src: int = 0):
        if self.world <= 1:
            return obj
        self._check_owner()
        lst = [obj]
        self.dist.broadcast_object_list(lst, src=src)
        return lst[0]

    def barrier(self):
        if self.world > 1:
            self._check_owner()
            self.dist.barrier()

    def max_float(self, v: float) -> float:
        if self.world <= 1:
            return v
        self._check_owner()
        t = self.torch.tensor([v], dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.dist is not None and self.dist.is_initialized():
            self.dist.destroy_process_group()


class EmulatedComm(Comm):
    """Rank `rank` of a `world`-rank job, run alone in one process (bench.py --emulate-rank):
    every collective is replaced by a local stand-in that returns the job-wide result, taken
    from a one-rank run of the same input (`glob`), and the bytes each collective would move
    over xGMI are recorded for the transfer model.  No process group exists; the rank does
    exactly its own shard's work plus everything the real code replicates on every rank.

    glob: "screen_by_hash" -> [device tensor per DB, hash order], "bottom" -> np.uint64,
    "nk" -> int, "ref_counts" -> device int32 per target, "rows" -> the one-rank LCA rows
    (query index = global index), "n_rows" -> int."""

    def __init__(self, rank: int, world: int, glob: dict):
        super().__init__(rank, world)
        import torch
        self.torch = torch
        self.glob = glob
        self.log: List[tuple] = []     # (kind, bytes per rank) of every collective since reset_log
        self.db_log: List[tuple] = []  # the same for the DB-load communicator (loader thread)
        import threading
        self._lock = threading.Lock()

    def reset_log(self):
        self.log = []
        with self._lock:
            self.db_log = []

    def allreduce_sum_(self, t):
        for g in self.glob["screen_by_hash"] + [self.glob["ref_counts"]]:
            if g.numel() == t.numel() and g.dtype == t.dtype:
                t.copy_(g)
                self.log.append(("allreduce", t.numel() * t.element_size()))
                return t
        raise ValueError(f"EmulatedComm: no job-wide value for an all-reduce of {t.numel()} x {t.dtype}")

    def allgather_slices_(self, t, c: int, key=None):
        """The other ranks' slices of sketch DB `key`'s hashes, copied from the job-wide DB
        (glob["msh_hashes"][key])."""
        g = self.glob["msh_hashes"][key]
        n = g.numel()
        if -(-n // self.world) != c or t.numel() < n:
            raise ValueError(f"EmulatedComm: DB {key} has {n} hashes, not {self.world} slices of {c}")
        lo, hi = min(n, self.rank * c), min(n, (self.rank + 1) * c)
        t[:lo].copy_(g[:lo])
        t[hi:n].copy_(g[hi:])
        with self._lock:                       # the loader thread's entry
            self.db_log.append(("allgather", c * t.element_size()))
        return t

    def allgather_np(self, arr: np.ndarray, tag: str = None) -> List[np.ndarray]:
        arr = np.asarray(arr)
        self.log.append(("allgather", arr.nbytes))
        if tag == "shard_records":           # ingest: every rank's record count
            return [np.array([c], np.int64) for c in self.glob["shard_records"]]
        if tag == "bottom":                  # screen: the ranks' bottom-s candidates
            return [np.asarray(self.glob["bottom"], np.uint64)]
        if tag == "n_kmers":                 # screen: the ranks' k-mer totals
            return [np.array([self.glob["nk"]], np.int64)]
        raise ValueError(f"EmulatedComm: no job-wide value for the all-gather {tag!r}")

    def gather_name_pools(self, qname, qname_off, n: int):
        nb = int(qname_off[n].item()) if n else 0
        self.log.append(("allgather", nb + 8 * n))
        if self.rank != 0:
            return None, None
        return self.glob["names"]

    def gather_rows(self, rows, q_base: int, gpu=None):
        """Rank 0 merges its own rows with the other ranks' (from the one-rank run) and sorts
        them exactly as Comm.gather_rows does; other ranks return nothing."""
        torch = self.torch
        R = int(rows["q"].shape[0])
        dev = rows["q"].device
        g = self.glob["rows"]
        n_all = int(g["q"].shape[0])
        self.log.append(("allgather", max(R, 1) * (12 * 4 + 8)))
        if self.rank != 0:
            e = torch.zeros(0, dtype=torch.int32, device=dev)
            return {"q": e, "part": e, "depth": e, "tax": e, "names": e,
                    "conf": torch.zeros(0, dtype=torch.float64, device=dev)}, 0
        rec = torch.zeros((max(R, 1), 12), dtype=torch.int32, device=dev)
        if R:
            rec[:R, 0] = rows["q"] + int(q_base)
            rec[:R, 1] = rows["part"]
            rec[:R, 2] = rows["depth"]
            rec[:R, 3] = rows["tax"]
            rec[:R, 4:] = rows["names"].view(R, 8)
        grec = torch.zeros((max(n_all, 1), 12), dtype=torch.int32, device=dev)
        if n_all:
            grec[:n_all, 0] = g["q"]
            grec[:n_all, 1] = g["part"]
            grec[:n_all, 2] = g["depth"]
            grec[:n_all, 3] = g["tax"]
            grec[:n_all, 4:] = g["names"].view(n_all, 8)
        lo, hi = int(q_base), int(q_base) + int(self.glob.get("shard_n", 0))
        other = (grec[:n_all, 0] < lo) | (grec[:n_all, 0] >= hi)
        allr = torch.cat([rec[:R], grec[:n_all][other]])
        allc = torch.cat([rows["conf"][:R], g["conf"][:n_all][other]])
        key = allr[:, 1].to(torch.int64) * (1 << 32) + allr[:, 0].to(torch.int64)
        order = torch.sort(key, stable=True).indices
        allr, allc = allr[order], allc[order]
        n = int(allr.shape[0])
        return {"q": allr[:, 0].contiguous(), "part": allr[:, 1].contiguous(), "depth": allr[:, 2].contiguous(),
                "tax": allr[:, 3].contiguous(), "names": allr[:, 4:].contiguous().view(-1), "conf": allc.contiguous()}, n

    def broadcast_obj(self, obj, src: int = 0):
        return obj if self.rank == src else self.glob["n_rows"]

    def gather_obj(self, obj, dst: int = 0):
        raise NotImplementedError("EmulatedComm: the fallback path is not emulated")

    def barrier(self):
        pass

    def max_float(self, v: float) -> float:
        return v

    def close(self):
        pass

    @staticmethod
    def model_ms(log, world: int, gbps: float = 100.0, latency_us: float = 30.0) -> float:
        """xGMI transfer model of the recorded collectives (ring algorithms): an all-reduce of
        B bytes per rank moves 2 (N-1)/N B per rank, an all-gather of B bytes per rank
        (N-1) B, at `gbps` per rank (a conservative RCCL bus bandwidth over xGMI), plus a
        fixed latency per collective."""
        ms = 0.0
        for kind, b in log:
            moved = 2.0 * (world - 1) / world * b if kind == "allreduce" else (world - 1) * b
            ms += latency_us / 1e3 + moved / (gbps * 1e9) * 1e3
        return ms

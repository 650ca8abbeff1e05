"""Process-group plumbing for the multi-GPU path.

One process per GPU, torch.distributed over RCCL ("nccl" backend = RCCL on ROCm, xGMI
inside a node) or gloo on CPU for the tests.  The path shards by contig / k-mer position
with three exchange steps: the screen hit counts (all-reduce, uint32 sum), the per-target
PAF-line counts (all-reduce, int32 sum) and the per-contig results (gather to rank 0).
"""
from __future__ import annotations

import os
from typing import List, Sequence

import numpy as np


class Comm:
    def __init__(self, rank: int = 0, world: int = 1, replicated_pool: bool = False):
        """replicated_pool: every rank holds the same contig pool (the screen then splits
        k-mer positions); otherwise (default) each rank's pool is its own contig shard."""
        self.rank, self.world = rank, world
        self.replicated_pool = replicated_pool
        self.dist = None
        self.device = None

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
        self.dist = dist
        self.device = gpu.dev if gpu is not None else torch.device("cpu")
        self.torch = torch
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
    def allreduce_sum_(self, t):
        if self.world > 1:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return t

    def allgather_np(self, arr: np.ndarray) -> List[np.ndarray]:
        if self.world <= 1:
            return [arr]
        objs = [None] * self.world
        self.dist.all_gather_object(objs, np.ascontiguousarray(arr))
        return objs

    def gather_obj(self, obj, dst: int = 0):
        if self.world <= 1:
            return [obj]
        out = [None] * self.world if self.rank == dst else None
        self.dist.gather_object(obj, out, dst=dst)
        return out

    def broadcast_obj(self, obj, src: int = 0):
        if self.world <= 1:
            return obj
        lst = [obj]
        self.dist.broadcast_object_list(lst, src=src)
        return lst[0]

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max_float(self, v: float) -> float:
        if self.world <= 1:
            return v
        t = self.torch.tensor([v], dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.dist is not None and self.dist.is_initialized():
            self.dist.destroy_process_group()

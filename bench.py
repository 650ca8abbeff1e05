#!/usr/bin/env python3
"""Benchmark contract (see README/DESIGN.md §Measurement).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload screen|cami-medium]

One "step" = one pass of the hot path over one batch of synthetic input that is already
resident in HBM.  Rank 0 prints ONE JSON line.  Multi-GPU: launched by the driver through
torch.distributed.run, one rank per GPU; contigs/k-mer positions are sharded (weak scaling).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def make_screen_workload(rng, n_refs, s, n_contigs, total_bases):
    """C2-shaped screen workload: a pooled contig set and a sketch DB with n_refs x s hashes
    (the first 25 references are real sketches of genomes the contigs come from)."""
    from hymet_amd.msh import SketchDB
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    n_src = 25
    glen = 2_000_000
    genomes = [acgt[rng.integers(0, 4, glen, dtype=np.uint8)].tobytes() for _ in range(n_src)]
    lens = np.clip(rng.lognormal(np.log(14963), 1.0, n_contigs), 4404, 400_000).astype(np.int64)
    lens = (lens * (total_bases / lens.sum())).astype(np.int64).clip(1000, glen - 1)
    recs = []
    for i, L in enumerate(lens):
        g = genomes[i % n_src]
        st = int(rng.integers(0, glen - L))
        recs.append((f"ctg{i}", "", g[st:st + int(L)]))
    hashes = rng.integers(0, 2 ** 63, size=(n_refs, s), dtype=np.int64).astype(np.uint64) * np.uint64(2) + np.uint64(1)
    hashes.sort(axis=1)
    db = SketchDB(k=21, seed=42, sketch_size=s, names=[f"GCF_{i:09d}.1_ref_genomic.fna.gz" for i in range(n_refs)],
                  comments=["[1 seqs] synthetic"] * n_refs, lengths=np.full(n_refs, glen, np.int64),
                  offsets=np.arange(n_refs + 1, dtype=np.int64) * s, hashes=hashes.reshape(-1))
    return recs, db, genomes


def bench_screen(args, comm, gpu, torch):
    from hymet_amd import screen as scr
    from hymet_amd.seqio import DevicePool, from_records
    rng = np.random.default_rng(1)
    n_refs = args.screen_refs
    recs, db, genomes = make_screen_workload(rng, n_refs, 1000, 1043, 53_800_000)
    ss = from_records(recs)
    pool = DevicePool(gpu, ss, DevicePool.ALPHA_MASH)
    table = scr.ScreenTable(gpu, db)
    torch.cuda.synchronize()
    n_pos = max(0, pool.n_bases - 21 + 1)
    b, e = comm.shard_range(n_pos) if comm.world > 1 else (0, n_pos)

    def step():
        counts, bottom, nk = scr.count_pool(gpu, pool, [table], 21, 42, 1000, b, e)
        if comm.world > 1:
            comm.allreduce_sum_(counts[0])
        sh, md = scr.table_stats(gpu, table, counts[0])
        return nk

    for _ in range(args.warmup):
        step()
    comm.barrier()
    torch.cuda.synchronize()
    # kernel timing with HIP events on the stream the kernels are launched on
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    nk = 0
    for _ in range(args.steps):
        nk = step()
    ev1.record()
    torch.cuda.synchronize()
    comm.barrier()
    t1 = time.perf_counter()
    dt = comm.max_float(t1 - t0)
    # dominant kernel alone (hash/probe/count), timed separately with events
    counts = [gpu.zeros(table.n_slots + 1, torch.int32)]
    cand = gpu.empty(1 << 20, torch.int64)
    cn = gpu.zeros(1, torch.int64)
    nkt = gpu.zeros(1, torch.int64)
    import ctypes
    from hymet_amd._lib import ptr
    keys_arr = (ctypes.c_void_p * 4)(ptr(table.keys).value)
    slots_arr = (ctypes.c_int64 * 4)(table.n_slots)
    cnt_arr = (ctypes.c_void_p * 4)(ptr(counts[0]).value)
    thr = int(16 * 1000 / max(1, e - b) * 2 ** 64)
    kt = []
    for _ in range(5):
        cn.zero_()
        a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a0.record()
        gpu.call("hymet_screen_count", ptr(pool.w2b), ptr(pool.wmask), pool.n_bases, b, e, 21, 42, 1, keys_arr,
                 slots_arr, cnt_arr, thr, ptr(cand), 1 << 20, ptr(cn), ptr(nkt))
        a1.record()
        torch.cuda.synchronize()
        kt.append(a0.elapsed_time(a1) / 1e3)
    k_avg = float(np.mean(kt[1:]))
    bases = e - b
    alg_bytes = bases * 0.375 + nk * 8.0  # packed read + one 8-B key probe per k-mer
    achieved = alg_bytes / k_avg / 1e9
    n_contigs = len(recs)
    total_mbp = ss.total_bases / 1e6
    value = n_contigs * args.steps / dt
    res = {
        "metric": "contigs/s (screen stage, C2 Zymo-shaped pool vs sketch1-sized DB)",
        "value": value, "unit": "contigs/s", "n_gpus": comm.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u64", "data": "synthetic",
        "mbp_per_s": total_mbp * args.steps / dt,
        "config": {"workload": "C2 screen: 1043 contigs / 53.8 Mbp vs %d refs x 1000 hashes (k=21, seed 42)" % n_refs,
                   "parallelism": f"kmer-shard x{comm.world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel": "screen_count_kernel<21>", "kernel_ms": k_avg * 1e3,
                     "alg_bytes_per_launch": alg_bytes},
    }
    if comm.rank == 0 and not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline_screen(recs, db)
    return res


def cpu_baseline_screen(recs, db, budget_s=15.0):
    from oracle import oracle_lib
    sub, tot = [], 0
    for r in recs:
        sub.append(r[2])
        tot += len(r[2])
        if tot > 4_000_000:
            break
    t0 = time.perf_counter()
    oracle_lib.screen(sub, db.k, db.seed, db.sketch_size, [db.ref_hashes(i) for i in range(min(db.n_refs, 20000))])
    dt = time.perf_counter() - t0
    return {"value": len(sub) / dt, "unit": "contigs/s", "cores": 1, "kind": "port",
            "sample": f"{len(sub)} contigs / {tot/1e6:.1f} Mbp vs 20000 refs, oracle/mash_oracle.c single thread",
            "mbp_per_s": tot / 1e6 / dt}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="screen", choices=["screen"])
    ap.add_argument("--screen-refs", type=int, default=100_000)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    import torch
    from hymet_amd.dist import Comm
    comm = Comm.from_env()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    from hymet_amd._lib import Gpu
    gpu = Gpu(local)
    comm.init_backend(gpu)
    res = bench_screen(args, comm, gpu, torch)
    if comm.rank == 0:
        print(json.dumps(res), flush=True)
    comm.close()


if __name__ == "__main__":
    main()

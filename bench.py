#!/usr/bin/env python3
"""Benchmark contract.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cami-medium|screen]

One step = one pass of the HYMET hot path (screen -> select -> limit -> map -> LCA -> TSV)
over one batch of synthetic, HBM-resident input.  Default workload: CAMI-medium (C4,
BASELINE.json configs[3]; it fits one MI355X): 12 taxa, ~1 Gbp of contigs per rank, 744
candidate genomes (~3 Gbp, two -I2g index parts), a sketch1-sized DB (1e5 refs x 1000).
The candidate-keyed index is built in the untimed cold run (run_hymet_cami.sh caches it the
same way) and its time is reported separately.  Rank 0 prints ONE JSON line.

Multi-GPU (torch.distributed.run, one rank per GPU): every rank holds its own ~1 Gbp contig
sample of the same community (weak scaling); screen counts and per-target PAF line counts
are all-reduced over RCCL; rank 0 writes the TSV.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
METRIC = "contigs/s + Mbp/s classified, CAMI-medium, 1/2/4/8 MI355X; % HBM roofline"


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench {time.strftime('%H:%M:%S')}]", *a, file=sys.stderr, flush=True)


# profiling scope (hymet_amd/csrc ProfScope tag) -> kernel symbol in rocprofv3 output
SCOPE_KERNEL = {"mm_chain": "chain_groups_kernel<0>", "mm_chain_long": "chain_groups_kernel<1>",
                "screen_count": "screen_count_kernel<21>", "mm_anchors": "write_anchor_keys_kernel",
                "mm_backtrack": "backtrack_groups_kernel"}
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")  # tools/pmc_summary.py output


def pmc_traffic(scope):
    """HBM bytes per launch of the scope's kernel from the committed PMC passes (FETCH_SIZE /
    WRITE_SIZE, gfx950-corrected: tools/pmc_summary.py), or None."""
    try:
        with open(PMC_FILE) as fh:
            tab = json.load(fh)
    except (OSError, ValueError):
        return None
    r = tab.get(SCOPE_KERNEL.get(scope, ""), {})
    return r.get("traffic_bytes")


def roofline_from_prof(prof, prefer=None):
    """Dominant kernel = the largest summed device time (every hot kernel has a byte model).
    The sub-scope `mm_backtrack.long` is part of `mm_backtrack` and never a candidate."""
    cand = {k: v for k, v in prof.items() if "." not in k}
    if not cand:
        return None
    name = prefer if prefer in cand else max(cand, key=lambda k: cand[k][0])
    ms, n, b = cand[name]
    achieved = b / (ms / 1e3) / 1e9 if ms > 0 else 0.0
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
            "traffic": pmc_traffic(name), "kernel": name, "kernel_symbol": SCOPE_KERNEL.get(name),
            "kernel_avg_ms": ms / max(n, 1), "launches": n, "alg_bytes_per_launch": b / max(n, 1)}


# ------------------------------------------------------------------ CAMI-medium
def build_cami(args, comm, gpu):
    from hymet_amd import pipeline, screen as scr, synth
    from hymet_amd.msh import SketchDB
    from hymet_amd.seqio import DevicePool, from_records
    t0 = time.time()
    w = synth.make_cami(np.random.default_rng(1234), n_taxa=args.taxa, per_taxon=args.per_taxon,
                        contig_gbp=args.contig_gbp, contig_rng=np.random.default_rng(5000 + comm.rank))
    log(f"synth: {len(w.refs)} refs {w.ref_bases/1e9:.2f} Gbp, {len(w.contigs)} contigs {w.contig_bases/1e6:.0f} Mbp "
        f"({time.time()-t0:.1f}s)")
    t0 = time.time()
    db_names = [n + ".fna.gz" for n in w.ref_names]
    refs_ss = from_records([(n, "", s) for n, s in zip(w.ref_names, w.refs)])
    sk = scr.sketch_sequences(gpu, DevicePool(gpu, refs_ss, DevicePool.ALPHA_MASH), 21, 42, 1000)
    n_dec = max(0, args.screen_refs - len(sk))
    dec = synth.decoy_sketches(np.random.default_rng(99), n_dec, 1000)
    lens = [len(h) for h in sk] + [1000] * n_dec
    off = np.zeros(len(lens) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    hashes = np.concatenate(sk + [dec.reshape(-1)])
    names = db_names + [f"GCF_{900000000 + i:09d}.1_decoy_genomic.fna.gz" for i in range(n_dec)]
    db = SketchDB(names=names, comments=[f"[1 seqs] {n}" for n in names], lengths=np.full(len(names), 4_000_000, np.int64),
                  offsets=off, hashes=hashes)
    log(f"sketch DB: {db.n_refs} refs, {len(db.hashes)/1e6:.0f}M hashes ({time.time()-t0:.1f}s)")
    td = tempfile.mkdtemp(prefix="hymet_bench_")
    tax = os.path.join(td, "detailed_taxonomy.tsv")
    hier = os.path.join(td, "taxonomy_hierarchy.tsv")
    open(tax, "w").write(w.taxonomy_tsv())
    open(hier, "w").write(w.hierarchy_tsv())
    by_name = {n + ".fna.gz": i for i, n in enumerate(w.ref_names)}

    def ref_lookup(sel):
        return refs_ss.subset([by_name[n] for n in sel])

    cfg = pipeline.Config(map_batch_bases=int(args.batch_mbp * 1e6))
    pipe = pipeline.Pipeline(gpu, [db], ref_lookup, tax, hier, cfg, comm)
    queries = from_records([(n, "", s) for n, s in zip(w.contig_names, w.contigs)])
    t0 = time.time()
    pq = pipe.prepare(queries)
    gpu.sync()
    log(f"queries resident: {len(pq.batches)} map batches ({time.time()-t0:.1f}s)")
    return w, db, pipe, pq, refs_ss, tax, hier, by_name


def bench_cami(args, comm, gpu, torch):
    w, db, pipe, pq, refs_ss, tax, hier, by_name = build_cami(args, comm, gpu)
    comm.barrier()
    t0 = time.time()
    res = pipe.run(pq)                      # cold: builds the candidate index (cached afterwards)
    gpu.sync()
    cold = time.time() - t0
    ix = pipe.index_for(res.selected)
    log(f"cold run {cold:.1f}s: {len(res.selected)} candidates, {len(ix.parts)} index parts, "
        f"{res.n_classified}/{res.n_queries} classified, {res.n_paf_lines} PAF lines")
    for _ in range(max(0, args.warmup - 1)):
        pipe.run(pq)
    gpu.sync()
    comm.barrier()
    gpu.prof_reset()
    gpu.prof(True)
    torch.cuda.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    prof_host = os.environ.get("HYMET_BENCH_PYPROF") and comm.rank == 0
    if prof_host:
        import cProfile
        cp = cProfile.Profile()
        cp.enable()
    for _ in range(args.steps):
        res = pipe.run(pq)
    torch.cuda.synchronize()
    if prof_host:
        import io
        import pstats
        cp.disable()
        sio = io.StringIO()
        pstats.Stats(cp, stream=sio).sort_stats("cumulative").print_stats(30)
        print(sio.getvalue(), file=sys.stderr)
    comm.barrier()
    dt = comm.max_float(time.perf_counter() - t0)
    gpu.prof(False)
    prof = gpu.prof_table()
    # Host-buffer boundary (the drop-in scripts read FASTA into host memory): re-time the
    # ingest (host alphabet encode + PCIe upload of every pool) once, outside the timed
    # region.  Reported beside `value` as the PCIe-inclusive rate; never `value` itself.
    comm.barrier()
    t_in = time.perf_counter()
    pq_in = pipe.prepare(pq.queries)
    torch.cuda.synchronize()
    ingest_s = comm.max_float(time.perf_counter() - t_in)
    del pq_in
    n_contigs = comm.world * len(w.contigs)        # weak scaling: every rank its own sample
    mbp = sum(comm.allgather_np(np.array([pq.queries.total_bases], np.int64)))[0] / 1e6
    step = dt / args.steps
    log("kernel time per step (ms): " + ", ".join(f"{k}={v[0]/args.steps:.1f}" for k, v in sorted(prof.items(), key=lambda kv: -kv[1][0])))
    out = {
        "metric": METRIC, "value": n_contigs / step, "unit": "contigs/s", "n_gpus": comm.world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": step * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u64", "data": "synthetic",
        "mbp_per_s": mbp / step,
        "config": {"workload": f"CAMI-medium (C4): {args.taxa} taxa, {len(w.contigs)} contigs / {pq.queries.total_bases/1e6:.0f} Mbp "
                               f"per rank; {len(res.selected)} candidates / {refs_ss.total_bases/1e9:.2f} Gbp in {len(ix.parts)} "
                               f"-I2g parts; sketch DB {db.n_refs} refs x 1000",
                   "global_contigs": n_contigs, "parallelism": f"contig-shard x{comm.world}"},
        "cold_run_s": cold,
        "ingest_ms": ingest_s * 1e3,
        "pcie_inclusive_contigs_per_s": n_contigs / (step + ingest_s),
        "stage_ms_per_step": {k: v[0] / args.steps for k, v in prof.items()},
        "roofline": roofline_from_prof(prof),
    }
    if comm.rank == 0 and not args.no_cpu:
        try:
            out["cpu_baseline"] = cpu_baseline_cami(args, gpu, pipe, pq, db, res, w, tax, hier)
        except Exception as e:  # the baseline is informative; never lose the GPU line
            out["cpu_baseline"] = {"error": repr(e)}
    return out


def cpu_baseline_cami(args, gpu, pipe, pq, db, res, w, tax, hier, budget_s=20.0):
    """The CPU oracle restatement on a bounded sample of the same workload, on the host's
    cores: worker threads take 8-contig batches of a random rank-0 sample and run minimap2
    asm10 against the same candidate index parts (exported from the device index,
    content-identical to the oracle's own per tests/test_mm_index_gpu.py; the C mapper
    releases the GIL) and the classification_cami restatement; then the contigs done are
    screened in one run (Mash screens the pooled input once: its per-run O(H) statistics
    pass over the 1e8-hash DB would dominate if paid per batch).  One-time table/index builds
    are excluded, like the warm GPU step."""
    import threading
    from concurrent.futures import ThreadPoolExecutor
    from oracle import classify_oracle, oracle_lib
    t0 = time.time()
    so = oracle_lib.ScreenOracle(db)
    ix = pipe.index_for(res.selected)
    parts = []
    for pi, part in enumerate(ix.parts):
        hs, pos = part.export()
        first = ix.part_first[pi]
        n = len(part.names)
        parts.append(oracle_lib.mm_index_from_arrays(hs, pos, ix.lens[first:first + n], ix.names[first:first + n]))
    opt = oracle_lib.asm10_opt()
    opt.mid_occ = pipe.opt.mid_occ
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    log(f"cpu baseline setup {time.time()-t0:.1f}s, {threads} threads")
    qs = pq.queries
    order = [int(q) for q in np.random.default_rng(7).permutation(qs.n)]
    lock = threading.Lock()
    state = {"next": 0, "contigs": 0, "bases": 0, "done": []}
    t_start = time.perf_counter()

    def worker(_):
        while time.perf_counter() - t_start < budget_s:
            with lock:
                b0 = state["next"]
                state["next"] += 8
            batch = order[b0:b0 + 8]
            if not batch:
                return
            seqs = [(qs.names[i], qs.seq(i)) for i in batch]
            paf = []
            for p in parts:                                               # map, part-major
                for name, s in seqs:
                    regs, rl = oracle_lib.mm_map(p, opt, s, name)
                    paf.extend(oracle_lib.format_paf(name, len(s), regs, rl, p.names, p.lens))
            fd, path = tempfile.mkstemp(suffix=".paf")
            os.write(fd, "".join(l + "\n" for l in paf).encode())
            os.close(fd)
            classify_oracle.classify_cami(path, tax, hier)                 # classify
            os.unlink(path)
            with lock:
                state["contigs"] += len(batch)
                state["bases"] += sum(len(s) for _, s in seqs)
                state["done"].extend(batch)

    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(worker, range(threads)))
    so.run([qs.seq(i) for i in state["done"]])                              # screen, one pooled run
    dt = time.perf_counter() - t_start
    return {"value": state["contigs"] / dt, "unit": "contigs/s", "cores": threads, "kind": "port",
            "mbp_per_s": state["bases"] / 1e6 / dt,
            "sample": f"{state['contigs']} random contigs / {state['bases']/1e6:.2f} Mbp of the rank-0 pool on {threads} "
                      f"threads: oracle minimap2 asm10 vs the same {len(ix.parts)} index parts + classification_cami "
                      f"restatement, then one oracle screen run over those contigs (prebuilt table, {db.n_refs} refs), "
                      f"{dt:.1f}s"}


# ------------------------------------------------------------------- screen only
def bench_screen(args, comm, gpu, torch):
    from hymet_amd import screen as scr, synth
    from hymet_amd.msh import SketchDB
    from hymet_amd.seqio import DevicePool, from_records
    rng = np.random.default_rng(1)
    w = synth.make_cami(rng, n_taxa=10, per_taxon=3, genome_mbp=(2.0, 4.0), contig_gbp=0.0538,
                        contig_rng=np.random.default_rng(11 + comm.rank))
    refs_ss = from_records([(n, "", s) for n, s in zip(w.ref_names, w.refs)])
    sk = scr.sketch_sequences(gpu, DevicePool(gpu, refs_ss, DevicePool.ALPHA_MASH), 21, 42, 1000)
    dec = synth.decoy_sketches(rng, max(0, args.screen_refs - len(sk)), 1000)
    hl = sk + list(dec)
    off = np.zeros(len(hl) + 1, np.int64)
    off[1:] = np.cumsum([len(h) for h in hl])
    db = SketchDB(names=[f"r{i}" for i in range(len(hl))], comments=[""] * len(hl), lengths=np.ones(len(hl), np.int64),
                  offsets=off, hashes=np.concatenate(hl))
    ss = from_records([(n, "", s) for n, s in zip(w.contig_names, w.contigs)])
    pool = DevicePool(gpu, ss, DevicePool.ALPHA_MASH)
    table = scr.ScreenTable(gpu, db)
    for _ in range(args.warmup):
        scr.screen(gpu, pool, [db], [table], comm)
    gpu.prof_reset()
    gpu.prof(True)
    torch.cuda.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        scr.screen(gpu, pool, [db], [table], comm)
    torch.cuda.synchronize()
    comm.barrier()
    dt = comm.max_float(time.perf_counter() - t0)
    gpu.prof(False)
    prof = gpu.prof_table()
    step = dt / args.steps
    return {"metric": "contigs/s screened (C2 Zymo-shaped pool vs sketch1-sized DB)", "value": comm.world * ss.n / step,
            "unit": "contigs/s", "n_gpus": comm.world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": step * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "mbp_per_s": comm.world * ss.total_bases / 1e6 / step,
            "config": {"workload": f"C2 screen: {ss.n} contigs / {ss.total_bases/1e6:.1f} Mbp vs {db.n_refs} refs x 1000"},
            "roofline": roofline_from_prof(prof, "screen_count")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="cami-medium", choices=["cami-medium", "screen"])
    ap.add_argument("--contig-gbp", type=float, default=1.0)
    ap.add_argument("--taxa", type=int, default=12)
    ap.add_argument("--per-taxon", type=int, default=62)
    ap.add_argument("--batch-mbp", type=float, default=40.0)
    ap.add_argument("--screen-refs", type=int, default=100_000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16, help="CPU baseline threads (the GPU box's CPU share is 16)")
    args = ap.parse_args()
    import torch
    from hymet_amd._lib import Gpu
    from hymet_amd.dist import Comm
    comm = Comm.from_env()
    gpu = Gpu(int(os.environ.get("LOCAL_RANK", "0")))
    comm.init_backend(gpu)
    res = bench_cami(args, comm, gpu, torch) if args.workload == "cami-medium" else bench_screen(args, comm, gpu, torch)
    if comm.rank == 0:
        print(json.dumps(res), flush=True)
    comm.close()


if __name__ == "__main__":
    main()

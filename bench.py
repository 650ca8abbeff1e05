#!/usr/bin/env python3
"""Benchmark contract (DESIGN.md §5 Measurement).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cami-medium|screen]

One step = one pass of the HYMET hot path over one input, in the SURVEY.md §8(d) window:
sketch DB files (.msh) parsed and their HBM tables built, detailed_taxonomy.tsv +
taxonomy_hierarchy.tsv loaded, FASTA text in host memory -> record table -> host-to-device
copy -> screen -> select -> limit -> map (both -I2g parts) -> LCA ->
classified_sequences.tsv written (and the resultados.paf text emitted to host memory).  Default workload: CAMI-medium (C4,
BASELINE.json configs[3]): 12 taxa, ~1 Gbp / ~151k contigs, 744 candidate genomes (~3 Gbp,
two index parts), a sketch1-sized DB (1e5 refs x 1000 hashes).  The candidate-keyed index
is built in the untimed cold run (run_hymet_cami.sh caches it the same way) and reported
separately.  Rank 0 prints ONE JSON line.

Multi-GPU (torch.distributed.run, one rank per GPU): STRONG scaling -- every rank holds the
same FASTA bytes and maps the contiguous record range FastaIndex.shard(rank, N); screen
counts and per-target PAF line counts are all-reduced over RCCL, LCA row records are
all-gathered and rank 0 writes the TSV.  value = all contigs / max-over-ranks step time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

# HIP multiplexes a process's streams over GPU_MAX_HW_QUEUES hardware queues (4 by default),
# assigned as streams are created; two mapping streams that land on one queue run one after
# the other (profiles/r05_streams/: +90 ms per C4 step).  A rank of a multi-GPU job also
# holds the RCCL communicators' streams, so give the process enough queues for every stream
# it creates (before the HIP runtime starts; at N = 1 it measured the same as 4).
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
METRIC = "contigs/s + Mbp/s classified, CAMI-medium, 1/2/4/8 MI355X; % HBM roofline"


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench {time.strftime('%H:%M:%S')}]", *a, file=sys.stderr, flush=True)


# profiling scope (hymet_amd/csrc ProfScope tag) -> kernel symbol in rocprofv3 output
SCOPE_KERNEL = {"mm_chain": "chain_groups_kernel<0>", "mm_chain_long": "chain_groups_kernel<1>",
                "mm_chain_small": "chain_small_kernel", "mm_chain_long_small": "chain_small_kernel",
                "screen_count": "screen_count_kernel<21>", "mm_anchors": "write_anchor_keys_kernel",
                "mm_backtrack": "backtrack_groups_kernel"}
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")  # tools/pmc_summary.py output
ISSUE_FILE = os.path.join(ROOT, "profiles", "pmc_issue.json")   # tools/sq_summary.py output (SQ counters)


def pmc_issue(scope, workload=None, batch_mbp=None):
    """Instruction-issue roofline of the scope's kernel from the committed SQ counter passes
    (tools/chain_pmc2.sh, tools/sq_summary.py): the kernel is latency/issue-bound, so beside
    its HBM fraction the line reports how busy the CU's scalar unit (1 SALU/cycle) and SIMDs
    (a wave64 VALU op per 2 cycles) are, measured on this workload's real anchors, or None."""
    try:
        with open(ISSUE_FILE) as fh:
            tab = json.load(fh)
    except (OSError, ValueError):
        return None
    w = tab.get(workload or "", {})
    if batch_mbp is not None and w.get("batch_mbp") != batch_mbp:
        return None
    k = w.get("kernels", {}).get(SCOPE_KERNEL.get(scope, ""))
    if not k:
        return None
    return {"bound": "issue", "salu_issue_frac": k["salu_issue_frac"], "valu_issue_frac": k["valu_issue_frac"],
            "per_64_anchors": {"salu": k["per_64_anchors"]["SQ_INSTS_SALU"], "valu": k["per_64_anchors"]["SQ_INSTS_VALU"]},
            "model": k["model"], "source": k["source"]}


def pmc_traffic(scope, workload=None, batch_mbp=None):
    """HBM bytes per launch of the scope's kernel from the committed PMC passes (FETCH_SIZE /
    WRITE_SIZE, gfx950-corrected: tools/pmc_summary.py), measured on THIS workload at THIS
    mapping batch size (per-launch bytes scale with the batch), or None."""
    try:
        with open(PMC_FILE) as fh:
            tab = json.load(fh)
    except (OSError, ValueError):
        return None
    w = tab.get(workload or "", {})
    if batch_mbp is not None and w.get("batch_mbp") != batch_mbp:
        return None
    return w.get("kernels", {}).get(SCOPE_KERNEL.get(scope, ""), {}).get("traffic_bytes")


def roofline_from_prof(prof, prefer=None, workload=None, batch_mbp=None):
    """Dominant kernel = the largest summed device time among the scopes that time one main
    kernel (SCOPE_KERNEL: mm_chain times chain_groups_kernel<0> alone -- plus its µs-sized
    work-list split -- and counts 28 B for each anchor of the groups that kernel took, from the
    device; the small-group lane kernel has its own scope).
    Multi-kernel sections with host syncs inside (mm_anchor_gsort, mm_z_order) are not
    candidates, nor is the sub-scope `mm_backtrack.long` (part of `mm_backtrack`)."""
    cand = {k: v for k, v in prof.items() if k in SCOPE_KERNEL} or {k: v for k, v in prof.items() if "." not in k}
    if not cand:
        return None
    name = prefer if prefer in cand else max(cand, key=lambda k: cand[k][0])
    ms, n, b = cand[name]
    achieved = b / (ms / 1e3) / 1e9 if ms > 0 else 0.0
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
            "traffic": pmc_traffic(name, workload, batch_mbp), "issue": pmc_issue(name, workload, batch_mbp),
            "kernel": name, "kernel_symbol": SCOPE_KERNEL.get(name),
            "kernel_avg_ms": ms / max(n, 1), "launches": n, "alg_bytes_per_launch": b / max(n, 1)}


def path_roofline(prof, steps, step_s, L, K, P, n_parts, world, w=10):
    """Whole-path roofline with SURVEY.md §8(d)'s algorithmic bytes per step:
    screen 0.25 L + 8 K (packed read, one key probe per k-mer); map per index part
    0.25 L + 8 M_q + 40 A (M_q = 2L/(w+1) minimizer lookups, A anchors: position fetch,
    anchor write + read); classify 16 P.  A is counted by the anchor kernel's scope (20 B
    per anchor, write_anchor_keys).  K_hit count updates and the once-per-run table build
    are left out (not in a warm step)."""
    A = prof.get("mm_anchors", (0.0, 0, 0.0))[2] / 20.0 / steps
    Mq = 2.0 * L / (w + 1)
    by = 0.25 * L + 8.0 * K + n_parts * (0.25 * L + 8.0 * Mq) + 40.0 * A + 16.0 * P
    ach = by / step_s / 1e9
    return {"bound": "hbm", "alg_bytes_per_step": by, "anchors_per_step": A, "achieved": ach,
            "peak": HBM_PEAK_GBS * world, "unit": "GB/s", "frac": ach / (HBM_PEAK_GBS * world)}


def gpu_scratch_gb(gpu):
    """Bytes held by the library's scratch cache (all contexts), GB."""
    import ctypes
    tot = 0
    for g in [gpu] + list(gpu.children):
        v = ctypes.c_int64()
        if g.lib.hymet_scratch_cached(g.ctx, ctypes.byref(v)) == 0:
            tot = max(tot, v.value)   # the cache is process-wide: every context reports the same
    return tot / 1e9


def scratch_stats(gpu):
    """The scratch allocator's (hipMalloc calls, OOM cache drops, frees past the cap) so far."""
    import numpy as _np
    v = _np.zeros(3, _np.int64)
    gpu.lib.hymet_scratch_stats(gpu.ctx, v.ctypes.data)
    return [int(x) for x in v]


def cpu_info():
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model, os.cpu_count() or 0


# ------------------------------------------------------------------ CAMI-medium
def cami_inputs(args, sketch):
    """The CAMI-shaped workload of `args` (bench.py's own; tests/golden/make_cami_golden.py
    builds the same one on the CPU): (workload, FASTA bytes, sketch DBs).  sketch(w) returns
    the Mash sketch (k=21, s=1000, seed 42) of every candidate genome, by the GPU here and
    by the oracle in the fixture generator, so both sides screen the same DB bytes."""
    from hymet_amd import ingest, synth
    from hymet_amd.msh import SketchDB
    t0 = time.time()
    # the same community and the same contig pool on every rank (strong scaling)
    w = make_workload(args)
    # MEGAHIT-style headers, as CAMI's assemblies carry them
    heads = [f"{n} flag=1 multi={2 + i % 7}.0000 len={len(s)}" for i, (n, s) in enumerate(zip(w.contig_names, w.contigs))]
    fasta = ingest.to_fasta(heads, w.contigs, width=args.fasta_width)
    log(f"synth: {len(w.refs)} refs {w.ref_bases/1e9:.2f} Gbp, {len(w.contigs)} contigs {w.contig_bases/1e6:.0f} Mbp, "
        f"FASTA {len(fasta)/1e6:.0f} MB ({time.time()-t0:.1f}s)")
    t0 = time.time()
    db_names = [n + ".fna.gz" for n in w.ref_names]
    sk = sketch(w)
    # sketch DBs of H hashes each (sketch1, and for CAMI-high GTDB/custom-sized sketch2/3):
    # the candidates' own sketches split over the DBs by share, decoy references fill up
    sizes = [int(float(x)) for x in args.db_hashes.split(",")]
    shares = np.array(sizes, np.float64) / sum(sizes)
    cut = np.r_[0, np.round(np.cumsum(shares) * len(sk)).astype(int)]
    dbs = []
    for d, H in enumerate(sizes):
        mine = list(range(cut[d], cut[d + 1]))
        n_dec = max(0, H // 1000 - len(mine))
        dec = synth.decoy_sketches(np.random.default_rng(99 + d), n_dec, 1000)
        lens = [len(sk[i]) for i in mine] + [1000] * n_dec
        off = np.zeros(len(lens) + 1, np.int64)
        off[1:] = np.cumsum(lens)
        hashes = np.concatenate([sk[i] for i in mine] + [dec.reshape(-1)])
        names = [db_names[i] for i in mine] + [f"GCF_{900000000 + d * 10**7 + i:09d}.1_decoy_genomic.fna.gz"
                                               for i in range(n_dec)]
        dbs.append(SketchDB(names=names, comments=[f"[1 seqs] {n}" for n in names],
                            lengths=np.full(len(names), 4_000_000, np.int64), offsets=off, hashes=hashes))
    log(f"sketch DBs: " + ", ".join(f"{x.n_refs} refs / {len(x.hashes)/1e6:.0f}M hashes" for x in dbs) +
        f" ({time.time()-t0:.1f}s)")
    return w, fasta, dbs


def zymo_genomes():
    """One real genome per shipped Zymo species (tests/golden/zymo: the reference's
    case/truth/zymo_refs genomes, committed as data): the first file of each species, its
    largest record; the yeast's 16 nuclear chromosomes joined."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _zymo
    out, seen = [], set()
    for sp, _f, recs in _zymo.genome_files():
        if sp in seen:
            continue
        seen.add(sp)
        if sp == "saccharomyces_cerevisiae":
            out.append((sp, b"".join(s for n, s in recs if n != "NC_001224.1")))  # without the mitochondrion
        else:
            out.append((sp, max((s for _, s in recs), key=len)))
    return out


def make_workload(args):
    from hymet_amd import synth
    rng = np.random.default_rng(1234)
    kw = {}
    if args.workload == "cami-medium-zymo":
        kw = {"backbones": synth.zymo_backbones(rng, zymo_genomes(), args.taxa), "div": (0.005, 0.02)}
    return synth.make_cami(rng, n_taxa=args.taxa, per_taxon=args.per_taxon, contig_gbp=args.contig_gbp,
                           contig_rng=np.random.default_rng(5000), **kw)


def build_cami(args, comm, gpu):
    from hymet_amd import pipeline, screen as scr
    from hymet_amd.msh import write_msh
    from hymet_amd.seqio import DevicePool, from_records
    held = {}

    def gpu_sketch(w):
        held["refs"] = from_records([(n, "", s) for n, s in zip(w.ref_names, w.refs)])
        return scr.sketch_sequences(gpu, DevicePool(gpu, held["refs"], DevicePool.ALPHA_MASH), 21, 42, 1000)

    w, fasta, dbs = cami_inputs(args, gpu_sketch)
    refs_ss = held["refs"]
    db = dbs[0]
    td = tempfile.mkdtemp(prefix="hymet_bench_")
    # the DBs as Mash .msh files (data/sketch{1,2,3}.msh): every step reads them, as every
    # `mash screen` does (scripts/mash.sh:14), so S1 is inside the timed window
    t0 = time.time()
    db_paths = []
    for d, x in enumerate(dbs):
        db_paths.append(os.path.join(td, f"sketch{d + 1}.msh"))
        write_msh(x, db_paths[-1])
    log(f"wrote {len(db_paths)} .msh files ({sum(os.path.getsize(q) for q in db_paths)/1e9:.2f} GB, {time.time()-t0:.1f}s)")
    tax = os.path.join(td, "detailed_taxonomy.tsv")
    hier = os.path.join(td, "taxonomy_hierarchy.tsv")
    open(tax, "w").write(w.taxonomy_tsv())
    open(hier, "w").write(w.hierarchy_tsv())
    by_name = {n + ".fna.gz": i for i, n in enumerate(w.ref_names)}

    def ref_lookup(sel):
        return refs_ss.subset([by_name[n] for n in sel])

    cfg = pipeline.Config(map_batch_bases=int(args.batch_mbp * 1e6), map_streams=args.map_streams,
                          cand_max=args.cand_max)
    pipe = pipeline.Pipeline(gpu, db_paths, ref_lookup, tax, hier, cfg, comm)
    return w, db, pipe, fasta, refs_ss, tax, hier, td


def bench_cami(args, comm, gpu, torch):
    from hymet_amd.ingest import FastaIndex
    w, db, pipe, fasta, refs_ss, tax, hier, td = build_cami(args, comm, gpu)
    tsv_path = os.path.join(td, "classified_sequences.tsv")
    comm.barrier()
    t0 = time.time()
    # cold: builds the candidate index (cached afterwards) and the pinned PAF text buffers
    res = pipe.run(fasta, with_paf=True)
    gpu.sync()
    cold = time.time() - t0
    ix = pipe.index_for(res.selected)
    log(f"cold run {cold:.1f}s: {len(res.selected)} candidates, {len(ix.parts)} index parts, "
        f"{res.n_classified}/{res.n_queries} classified, {res.n_paf_lines} PAF lines on rank 0")
    for _ in range(max(0, args.warmup - 1)):
        pipe.run(fasta, with_paf=True)
    gpu.sync()
    comm.barrier()
    gpu.prof_reset()
    gpu.prof(True)
    torch.cuda.synchronize()
    comm.barrier()
    ss0 = scratch_stats(gpu)
    t0 = time.perf_counter()
    prof_host = os.environ.get("HYMET_BENCH_PYPROF") and comm.rank == 0
    if prof_host:
        import cProfile
        cp = cProfile.Profile()
        cp.enable()
    loads = {}
    for _ in range(args.steps):
        res = pipe.run(fasta, with_paf=True)        # .msh + taxonomy files, FASTA bytes in host memory -> TSV + PAF text
        for k, v in pipe.timings.items():
            loads[k] = loads.get(k, 0.0) + v
        if comm.rank == 0:
            with open(tsv_path, "wb") as f:             # classified_sequences.tsv written
                f.write(res.tsv)
    if comm.rank == 0 and args.tsv_out:
        with open(args.tsv_out, "wb") as f:
            f.write(res.tsv)
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
    n_contigs = len(w.contigs)
    total_bases = w.contig_bases
    step = dt / args.steps
    kern_ms = sum(v[0] for k, v in prof.items() if "." not in k) / args.steps
    log("kernel time per step (ms): " + ", ".join(f"{k}={v[0]/args.steps:.1f}" for k, v in sorted(prof.items(), key=lambda kv: -kv[1][0])))
    n_lines = sum(int(x[0]) for x in comm.allgather_np(np.array([res.n_paf_lines], np.int64)))
    out = {
        "metric": METRIC, "value": n_contigs / step, "unit": "contigs/s", "n_gpus": comm.world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": step * 1e3, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u64", "data": "synthetic",
        "mbp_per_s": total_bases / 1e6 / step,
        "config": {"workload": f"{args.workload_name}: {args.taxa} taxa, {n_contigs} contigs / {total_bases/1e6:.0f} Mbp FASTA "
                               f"({len(fasta)/1e6:.0f} MB) sharded over {comm.world} GPU(s); {len(res.selected)} candidates / "
                               f"{refs_ss.total_bases/1e9:.2f} Gbp in {len(ix.parts)} -I2g parts; sketch DBs "
                               + " + ".join(f"{d.n_refs} refs" for d in pipe.dbs) + " x 1000",
                   "global_contigs": n_contigs, "parallelism": f"contig-shard x{comm.world}",
                   "backend": (("nccl (RCCL over xGMI)" if comm.dist.get_backend() == "nccl" else comm.dist.get_backend())
                               if comm.dist is not None else "none (1 rank)"),
                   "window": " + ".join(os.path.basename(q) for q in (pipe.db_paths or [])) +
                             " + detailed_taxonomy.tsv + taxonomy_hierarchy.tsv read, FASTA bytes in host "
                             "memory -> classified_sequences.tsv written + resultados.paf text in host memory (DB parse + "
                             "table build, taxonomy load, ingest, H2D, screen, select, limit, map, LCA, text emit inside "
                             "every step)"},
        "cold_run_s": cold,
        "scratch_cached_gb": gpu_scratch_gb(gpu),
        # allocator events inside the timed steps (hipMalloc, OOM drops, over-cap frees): each
        # can synchronise the device; a steady state has none
        "scratch_events_timed": [b - a for a, b in zip(ss0, scratch_stats(gpu))],
        "hbm_free_gb": torch.cuda.mem_get_info(gpu.dev)[0] / 1e9,
        "torch_reserved_gb": torch.cuda.memory_reserved(gpu.dev) / 1e9,
        "paf_lines": n_lines,
        "kernel_ms_per_step_rank0": kern_ms,
        "stage_ms_per_step": {k: v[0] / args.steps for k, v in prof.items()},
        # algorithmic GB/s of each stage (its ProfScope byte model / its kernel time)
        "stage_alg_gbps": {k: v[2] / v[0] / 1e6 for k, v in prof.items() if v[0] > 0 and v[2] > 0},
        # host wall time of the per-step input loads (inside ms_per_step): S1 .msh parse and
        # HBM table build, C1-C2 taxonomy + hierarchy load
        "input_load_ms_per_step": {k.replace("_s", "_ms"): v * 1e3 / args.steps for k, v in loads.items()},
        "roofline": roofline_from_prof(prof, workload=args.workload, batch_mbp=args.batch_mbp),
        "path_roofline": path_roofline(prof, args.steps, step, total_bases, total_bases, n_lines, len(ix.parts), comm.world),
    }
    if comm.world == 1:
        try:
            out["config"]["predicted_imbalance"] = shard_balance(gpu, pipe, fasta)
        except Exception as e:  # informative only
            out["config"]["predicted_imbalance"] = {"error": repr(e)}
    if comm.rank == 0 and comm.world == 1 and not args.no_cpu:   # the CPU leg runs at N=1 only
        try:
            out["cpu_baseline"] = cpu_baseline_cami(args, pipe, res, fasta, db, tax, hier)
        except Exception as e:  # the baseline is informative; never lose the GPU line
            import traceback
            traceback.print_exc()
            out["cpu_baseline"] = {"error": repr(e)}
    return out


def host_cpus():
    """(CPUs this process may run on, the cgroup CPU quota in CPUs or None): the box's
    nproc counts the whole machine, the scheduler affinity and the cgroup quota what a job
    actually gets."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    return aff, quota


def cpu_threads_default():
    """The job's CPU share: the affinity set, capped by the cgroup quota and by the thread
    count the box assigns a job (OMP_NUM_THREADS; the GPU pool sets 16 per GPU job)."""
    aff, quota = host_cpus()
    n = min(aff, int(quota) if quota else aff)
    try:
        n = min(n, int(os.environ.get("OMP_NUM_THREADS", "0")) or n)
    except ValueError:
        pass
    return max(1, n)


def shard_balance(gpu, pipe, fasta, worlds=(2, 4, 8)):
    """Per-rank mapping work of the N-rank runs predicted from this one-rank run (SURVEY.md
    §8(e) step 1): each rank maps the contiguous record range FastaIndex.shard(rank, N),
    balanced by bases; a contig's mapping cost is taken as its bases plus its chained
    anchors (the cm of its PAF lines, summed: chaining and backtrack work grow with the
    anchors, not the bases).  Returns max/mean over ranks of both, per N."""
    import ctypes
    from hymet_amd.ingest import FastaIndex
    acc = pipe.acc
    q, _part, _t = acc.columns()
    cm = np.zeros(max(len(q), 1), np.int32)
    gpu.call("hymet_paf_acc_field", acc.h, 9, cm.ctypes.data_as(ctypes.c_void_p))
    fx = FastaIndex(fasta)
    anchors = np.bincount(q, weights=cm[:len(q)].astype(np.float64), minlength=fx.n)
    bases = np.asarray(fx.nbases, np.float64)
    out = {"model": "contiguous byte-range shards (ingest.shard_bytes); cost = chained anchors (sum of cm) per contig"}
    for n in worlds:
        cuts = fx.byte_shards(n)
        a = np.array([anchors[r0:r1].sum() for r0, r1 in cuts])
        b = np.array([bases[r0:r1].sum() for r0, r1 in cuts])
        out[str(n)] = {"anchors_max_over_mean": float(a.max() / a.mean()), "bases_max_over_mean": float(b.max() / b.mean())}
    return out


def cpu_baseline_cami(args, pipe, res, fasta, db, tax, hier, budget_s=None, must=None, n_random=None):
    """The CPU oracle restatement on a bounded sample of the same workload, on the host's
    cores, CHECKED against the GPU run: worker threads take 8-contig batches of a random
    sample and run the minimap2 asm10 restatement against the same candidate index parts
    (exported from the device index, content-identical to the oracle's own build per
    tests/test_mm_index_gpu.py; the C mapper releases the GIL), then the sampled contigs are
    screened in one oracle run (Mash screens the pooled input once) and classified by the
    classification_cami restatement with the run's global ref_abundance (the per-target
    line counts of the whole PAF, classification_cami.py:181-208).  The sample's PAF lines
    and TSV rows must equal the GPU's for the same contigs (single GPU).
    must: contig indices mapped before the random ones and regardless of the budget (the
    stratified C5 check: every long contig); n_random: exactly this many random contigs
    after them, with no time budget."""
    import threading
    from concurrent.futures import ThreadPoolExecutor
    from hymet_amd.ingest import FastaIndex
    from oracle import classify_oracle, oracle_lib
    budget_s = args.cpu_budget if budget_s is None else budget_s
    t0 = time.time()
    fx = FastaIndex(fasta)
    names = fx.names()
    so = oracle_lib.ScreenOracle(db)
    ix = pipe.index_for(res.selected)
    parts = []
    for pi, part in enumerate(ix.parts):
        hs, pos = part.export()
        first = ix.part_first[pi]
        n = len(part.names)
        parts.append(oracle_lib.mm_index_from_arrays(hs, pos, ix.lens[first:first + n], ix.names[first:first + n]))
    opt = oracle_lib.asm10_opt()
    opt.mid_occ = ix.opt.mid_occ
    aff, quota = host_cpus()
    threads = max(1, min(args.cpu_threads or cpu_threads_default(), aff))
    log(f"cpu baseline setup {time.time()-t0:.1f}s, {threads} threads")
    d = fasta

    def seq(i):
        return d[fx.seq_off[i]:fx.seq_end[i]].replace(b"\n", b"").replace(b"\r", b"")

    forced = [int(q) for q in (must if must is not None else [])]
    fset = set(forced)
    order = forced + [int(q) for q in np.random.default_rng(7).permutation(fx.n) if int(q) not in fset]
    if n_random is not None:
        order = order[:len(forced) + n_random]
        budget_s = float("inf")
    lock = threading.Lock()
    state = {"next": 0, "contigs": 0, "bases": 0, "done": [], "paf": {}}
    t_start = time.perf_counter()

    def worker(_):
        while True:
            with lock:
                b0 = state["next"]
                if b0 >= len(forced) and time.perf_counter() - t_start >= budget_s:
                    return
                # the forced (long) contigs one at a time, the random ones 8 per batch
                state["next"] += 1 if b0 < len(forced) else 8
                batch = order[b0:state["next"]]
            if not batch:
                return
            seqs = [(names[i], seq(i)) for i in batch]
            got = {}
            for p in parts:                                               # map, part-major
                for name, s in seqs:
                    regs, rl = oracle_lib.mm_map(p, opt, s, name)
                    got.setdefault(name, []).extend(oracle_lib.format_paf(name, len(s), regs, rl, p.names, p.lens))
            with lock:
                state["contigs"] += len(batch)
                state["bases"] += sum(len(s) for _, s in seqs)
                state["done"].extend(batch)
                state["paf"].update(got)

    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(worker, range(threads)))
    done = state["done"]
    so.run([seq(i) for i in done])                                           # screen, one pooled run
    # classify the sample's lines with the run's global per-target line counts
    q, part, t = pipe.acc.columns()
    ref_counts = dict(zip(ix.names, np.bincount(t, minlength=len(ix.names)).tolist()))
    fd, path = tempfile.mkstemp(suffix=".paf")
    sample_names = [names[i] for i in done]
    paf_lines = [l for nm in sample_names for l in state["paf"].get(nm, [])]
    os.write(fd, "".join(l + "\n" for l in paf_lines).encode())
    os.close(fd)
    o_tsv = classify_oracle.classify_cami(path, tax, hier, ref_counts=ref_counts)
    os.unlink(path)
    dt = time.perf_counter() - t_start
    # check against the GPU run of the same contigs
    want = set(sample_names)
    g_paf = {}
    for line in res.paf_bytes.decode().split("\n"):
        nm = line.split("\t", 1)[0]
        if nm in want:
            g_paf.setdefault(nm, []).append(line)
    paf_ok = sum(1 for nm in sample_names if g_paf.get(nm, []) == state["paf"].get(nm, []))
    g_rows = {}
    for row in res.tsv.decode().split("\r\n")[1:]:
        nm = row.split("\t", 1)[0]
        if nm in want:
            g_rows[nm] = row
    o_rows = {r.split("\t", 1)[0]: r for r in o_tsv.decode().split("\r\n")[1:] if r}
    tsv_ok = sum(1 for nm in sample_names if g_rows.get(nm) == o_rows.get(nm))
    model, ncpu = cpu_info()
    import shutil
    # BASELINE.md rule 1: the real tools as the pipeline invokes them when they are installed
    # (scripts/mash.sh:14, scripts/minimap2.sh:23); the image has neither, so the oracle port
    # is timed -- recorded as observed on this host, not assumed
    tools = {t: shutil.which(t) for t in ("mash", "minimap2")}
    out = {"value": state["contigs"] / dt, "unit": "contigs/s", "cores": threads, "kind": "port",
           "reference_tools_on_path": tools,
           "mbp_per_s": state["bases"] / 1e6 / dt, "cpu_model": model, "nproc": ncpu,
           "sched_affinity_cpus": aff, "cgroup_cpu_quota": quota,
           "checked": {"contigs": len(done), "paf_identical": paf_ok, "tsv_rows_identical": tsv_ok,
                       "paf_lines": len(paf_lines)},
           "sample": (f"{len(forced)} listed + " if forced else "") +
                     f"{state['contigs'] - len(forced)} random contigs / {state['bases']/1e6:.2f} Mbp on {threads} threads: oracle "
                     f"minimap2 asm10 vs the same {len(ix.parts)} index parts, one oracle screen run over those contigs "
                     f"(prebuilt table, {db.n_refs} refs), classification_cami restatement with the run's global "
                     f"ref_abundance, {dt:.1f}s"}
    if paf_ok != len(done) or tsv_ok != len(done):
        out["error"] = "GPU output differs from the oracle on the sampled contigs"
    return out


# ------------------------------------------------------------- one rank of N, emulated
def bench_emulate(args, gpu, torch):
    """`--emulate-rank R[,R2...]/N`: bound the N-GPU step from one GPU.  A one-rank run of the
    workload (untimed cold run, then `--steps` timed steps for the one-rank reference) records
    the job-wide results of every exchange step -- screen hit counts in the DB's hash order,
    the pool's bottom-s sketch and k-mer total, per-target PAF line counts, the LCA rows.
    Then each listed rank runs alone, `--steps` timed steps of exactly what it does in an
    N-rank job (its contiguous record shard, plus everything the code replicates on every
    rank), with every collective replaced by a local stand-in that returns the job-wide value
    (hymet_amd.dist.EmulatedComm).  The bytes each collective would move are modelled over
    xGMI (EmulatedComm.model_ms) and added: predicted step = max over the emulated ranks of
    (measured rank step + modelled transfers).  A prediction, not a measured scaling curve."""
    from hymet_amd import pipeline, screen as scr
    from hymet_amd.dist import Comm, EmulatedComm
    from hymet_amd.ingest import FastaIndex
    ranks_s, world_s = args.emulate_rank.split("/")
    N = int(world_s)
    ranks = [int(r) for r in ranks_s.split(",")]
    if N < 2 or any(r < 0 or r >= N for r in ranks):
        raise SystemExit(f"--emulate-rank {args.emulate_rank}: want R[,R...]/N with 0 <= R < N, N >= 2")
    w, db, pipe1, fasta, refs_ss, tax, hier, td = build_cami(args, Comm(), gpu)
    glob = {}
    orig_reduce = scr.reduce_partials
    orig_rows = pipe1.classify_rows

    def capture_screen(comm, counts, bottom, nk, s, tables=None):
        glob["screen_by_hash"] = [c.clone() for c in counts]     # by canonical index: the same on every rank
        glob["bottom"] = np.asarray(bottom, np.uint64).copy()
        glob["nk"] = int(nk)
        return orig_reduce(comm, counts, bottom, nk, s, tables)

    def capture_rows(ix, sh):
        import ctypes
        rws, n = orig_rows(ix, sh)
        glob["rows"] = {k: v.clone() for k, v in rws.items()}
        glob["n_rows"] = n
        counts = gpu.zeros(max(len(ix.names), 1), torch.int32)
        gpu.call("hymet_acc_ref_counts", pipe1.acc.h, ctypes.c_void_p(counts.data_ptr()))
        glob["ref_counts"] = counts
        return rws, n

    scr.reduce_partials, pipe1.classify_rows = capture_screen, capture_rows
    t0 = time.time()
    try:
        res1 = pipe1.run(fasta, with_paf=True)
    finally:
        scr.reduce_partials, pipe1.classify_rows = orig_reduce, orig_rows
    gpu.sync()
    log(f"one-rank cold run {time.time()-t0:.1f}s: {len(res1.selected)} candidates, {res1.n_queries} rows")
    # keep the TSV only: a RunResult still holding its PAF text makes the pipeline copy that
    # text out of the pinned buffer (copy-on-reuse) inside a later timed run
    tsv1 = res1.tsv
    del res1

    def timed(pipe, steps, warmup):
        for _ in range(warmup):
            pipe.run(fasta, with_paf=True)
        gpu.sync()
        gpu.prof_reset()
        gpu.prof(True)
        phases = {}
        if isinstance(pipe.comm, EmulatedComm):
            pipe.comm.reset_log()
        t0 = time.perf_counter()
        for _ in range(steps):
            r = pipe.run(fasta, with_paf=True)
            for k, v in pipe.phases.items():
                phases[k] = phases.get(k, 0.0) + v
            # the loader thread's wall time (input loads; with slices: + the DB all-gathers
            # and the table build), beside the main thread's ingest_s
            phases["reader_s"] = phases.get("reader_s", 0.0) + pipe.timings.get("reader_s", 0.0)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        gpu.prof(False)
        prof = gpu.prof_table()
        return r, dt, {k: v * 1e3 / steps for k, v in phases.items()}, {k: v[0] / steps for k, v in prof.items()}

    _, t1, ph1, st1 = timed(pipe1, args.steps, max(0, args.warmup - 1))
    log(f"one rank: {t1*1e3:.1f} ms/step")
    # the one-rank pipeline's mapping contexts keep their scratch blocks cached; the emulated
    # rank's contexts are new streams and would otherwise push the cache past its cap
    gpu.sync()
    gpu.lib.hymet_scratch_trim(gpu.ctx, None)
    # each rank of an N-rank job loads one slice of every DB's hashes and all-gathers the rest
    # (Pipeline._join_slices): the stand-in copies them from the whole DB
    from hymet_amd.msh import read_msh
    glob["msh_hashes"] = [torch.from_numpy(np.ascontiguousarray(read_msh(p).hashes).view(np.int64)).to(gpu.dev)
                          for p in pipe1.db_paths]
    fx = FastaIndex(fasta)
    shards = fx.byte_shards(N)          # the records each rank's byte range holds (ingest.shard_bytes)
    glob["shard_records"] = [r1 - r0 for r0, r1 in shards]
    pool, off = fx.name_pool()
    glob["names"] = (torch.from_numpy(pool.copy() if len(pool) else np.zeros(1, np.uint8)).to(gpu.dev),
                     torch.from_numpy(off).to(gpu.dev))
    out_ranks = {}
    for R in ranks:
        r0, r1 = shards[R]
        glob["shard_n"] = r1 - r0
        comm = EmulatedComm(R, N, glob)
        pipe_e = pipeline.Pipeline(gpu, pipe1.db_paths, pipe1.ref_lookup, tax, hier, pipe1.cfg, comm)
        pipe_e.index_cache = pipe1.index_cache
        pipe_e.run(fasta, with_paf=True)               # cold: pinned buffers, contexts
        res_e, te, phe, ste = timed(pipe_e, args.steps, max(0, args.warmup - 1))
        per_step = [(k, b) for k, b in comm.log[:len(comm.log) // max(args.steps, 1)]]
        db_step = [(k, b) for k, b in comm.db_log[:len(comm.db_log) // max(args.steps, 1)]]
        # the main thread's collectives are in series with its work; the DB all-gathers run on
        # the loader thread beside the ingest, and lengthen the step only by what they add to
        # the loader's finish past the ingest's end, beyond the wait measured (stand-in copies)
        x_main = EmulatedComm.model_ms(per_step, N)
        x_db = EmulatedComm.model_ms(db_step, N)
        ing, wait, rd = phe.get("ingest_s", 0.0), phe.get("input_wait_s", 0.0), phe.get("reader_s", 0.0)
        x_db_exposed = max(0.0, rd + x_db - ing) - wait
        if os.environ.get("HYMET_DB_GATHER", "loader") == "main":
            x_db_exposed = x_db                # on the calling thread: in series with the step
        model = x_main + max(0.0, x_db_exposed)
        out_ranks[str(R)] = {
            "shard_records": [int(r0), int(r1)], "shard_mbp": float(fx.nbases[r0:r1].sum()) / 1e6,
            "ms_per_step": te * 1e3, "phases_ms": phe, "stage_ms_per_step": ste,
            "input_load_ms_last_step": {k.replace("_s", "_ms"): v * 1e3 for k, v in pipe_e.timings.items()},
            "collectives_per_step": [{"kind": k, "bytes_per_rank": int(b)} for k, b in per_step],
            "db_load_collectives_per_step": [{"kind": k, "bytes_per_rank": int(b)} for k, b in db_step],
            "xgmi_model_ms": model, "xgmi_main_ms": x_main, "xgmi_db_load_ms": x_db,
            "xgmi_db_load_exposed_ms": max(0.0, x_db_exposed), "predicted_ms_per_step": te * 1e3 + model,
            "tsv_rows": res_e.n_queries, "paf_lines": res_e.n_paf_lines}
        if R == 0:
            out_ranks[str(R)]["tsv_identical_to_one_rank"] = res_e.tsv == tsv1
        log(f"rank {R}/{N}: {te*1e3:.1f} ms/step + {model:.1f} ms modelled xGMI")
        pipe_e.acc.close()
        for a in pipe_e.map_accs:
            a.close()
        del pipe_e, comm
        import gc
        gc.collect()
        gpu.lib.hymet_scratch_trim(gpu.ctx, None)
    pred = max(v["predicted_ms_per_step"] for v in out_ranks.values())
    meas = max(v["ms_per_step"] for v in out_ranks.values())
    # T_N = A + B / N and T_1 = A + B: the part of the step that does not shrink with N
    fixed = (N * meas - t1 * 1e3) / (N - 1)
    return {"metric": METRIC + " (emulated)", "emulated_world": N, "emulated_ranks": ranks, "steps": args.steps,
            "warmup": args.warmup, "one_rank_ms_per_step": t1 * 1e3, "one_rank_phases_ms": ph1,
            "one_rank_stage_ms_per_step": st1, "ranks": out_ranks, "predicted_ms_per_step": pred,
            "predicted_speedup_vs_one_rank": t1 * 1e3 / pred, "predicted_contigs_per_s": len(w.contigs) / (pred / 1e3),
            "non_shardable_ms_per_step": fixed,
            "model": "predicted = max over the emulated ranks of (its measured step with local stand-ins for the "
                     "collectives + ring transfers of the recorded bytes at 100 GB/s per rank + 30 us per collective; "
                     "the DB-load all-gathers, on the loader thread beside the ingest, count only for what they add "
                     "to the loader's finish past the ingest's end: max(0, reader + x_db - ingest) - measured wait); "
                     "non_shardable = (N * max rank step - one-rank step) / (N - 1), from T = A + B / N",
            "config": {"workload": args.workload_name, "contigs": len(w.contigs), "contig_mbp": w.contig_bases / 1e6}}


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
            "roofline": roofline_from_prof(prof, "screen_count", workload="screen")}


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` started without a launcher (no WORLD_SIZE in the environment):
    start N rank processes of this same command line, one per GPU, with the environment
    torch.distributed.run would give them (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR /
    MASTER_PORT on 127.0.0.1), and return the first non-zero exit status.  This runs before
    anything touches the GPU (the parent never initialises HIP) and starts children rather
    than exec'ing into them."""
    import signal
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    try:
        for p in procs:
            r = p.wait()
            if r != 0 and rc == 0:
                rc = r
                for q in procs:          # one rank failed: the others would wait in a collective
                    if q.poll() is None:
                        q.send_signal(signal.SIGTERM)
    finally:
        for q in procs:
            if q.poll() is None:
                q.kill()
    return rc


def bench_dry(args, comm):
    """CPU rehearsal of the multi-rank launch (no GPU, gloo): every rank builds the same
    synthetic FASTA, indexes only its byte range exactly as Pipeline.ingest does
    (ingest.shard_bytes, the ranks' record counts all-gathered for the query base), and the
    ranks all-reduce their contig and base counts; rank 0 reports the world and checks the
    shards cover the input once."""
    import torch
    from hymet_amd import ingest, synth
    from hymet_amd.ingest import FastaIndex
    w = synth.make_cami(np.random.default_rng(1234), n_taxa=2, per_taxon=2, genome_mbp=(0.2, 0.3),
                        contig_gbp=0.002, contig_rng=np.random.default_rng(5000), max_contigs=400)
    data = ingest.to_fasta(list(w.contig_names), w.contigs)
    fx = FastaIndex(data, byte_range=ingest.shard_bytes(data, comm.rank, comm.world))
    counts = comm.allgather_np(np.array([fx.n], np.int64), tag="shard_records")
    r0 = int(sum(int(c[0]) for c in counts[:comm.rank]))
    r1 = r0 + fx.n
    assert fx.names() == list(w.contig_names[r0:r1])
    t = torch.tensor([r1 - r0, int(fx.nbases.sum())], dtype=torch.int64)
    comm.allreduce_sum_(t)
    spans = comm.allgather_np(np.array([r0, r1], np.int64))
    ok = int(t[0]) == len(w.contigs) and int(t[1]) == w.contig_bases and all(int(a[1]) == int(b[0]) for a, b in zip(spans, spans[1:]))
    return {"metric": METRIC, "value": None, "unit": "contigs/s", "n_gpus": comm.world, "dry_run": True,
            "backend": comm.dist.get_backend() if comm.dist is not None else None, "shards": [[int(a[0]), int(a[1])] for a in spans],
            "contigs": int(t[0]), "bases": int(t[1]), "covers_input_once": bool(ok)}


def parse_args(argv=None):
    """The command line, with the workload's defaults resolved (tests build the same
    workloads through this)."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="cami-medium", choices=["cami-medium", "cami-medium-zymo", "cami-high", "screen"])
    ap.add_argument("--contig-gbp", type=float, default=None, help="Gbp of contigs (default: 1.0; cami-high 2.0)")
    ap.add_argument("--taxa", type=int, default=12)
    ap.add_argument("--per-taxon", type=int, default=62)
    ap.add_argument("--batch-mbp", type=float, default=None,
                    help="query Mbp per mapping batch (default: 60 for cami-medium, 40 for cami-high)")
    ap.add_argument("--map-streams", type=int, default=2, help="concurrent mapping batches (library contexts)")
    ap.add_argument("--fasta-width", type=int, default=0, help="FASTA line width (0: one line per contig, as MEGAHIT)")
    ap.add_argument("--screen-refs", type=int, default=100_000, help="screen-only workload: references in the DB")
    ap.add_argument("--db-hashes", default=None, help="hashes per sketch DB, comma-separated (C4: 1e8; C5: 1e8,5e7,1e7)")
    ap.add_argument("--cand-max", type=int, default=5000, help="CAND_MAX (run_hymet_cami.sh:26)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="CPU baseline threads (default: every CPU the scheduler affinity and cgroup quota give this job)")
    ap.add_argument("--cpu-budget", type=float, default=20.0, help="seconds of CPU mapping in the checked CPU leg")
    ap.add_argument("--backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="process-group backend for N > 1 (auto: nccl = RCCL over xGMI)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rank r uses GPU r %% device_count (rehearse N ranks on fewer GPUs; use with --backend gloo)")
    ap.add_argument("--dry-run", action="store_true", help="CPU rehearsal of the N-rank launch and sharding (gloo, no GPU)")
    ap.add_argument("--tsv-out", default=None, help="rank 0 writes the last step's classified_sequences.tsv here")
    ap.add_argument("--emulate-rank", default=None, metavar="R[,R...]/N",
                    help="run rank R of an N-rank job alone on this GPU, collectives replaced by stand-ins "
                         "(bench_emulate: a predicted N-GPU step, not a measurement)")
    args = ap.parse_args(argv)
    # CAMI-high (C5, BASELINE.json configs[4]): 14 taxa (tools/generate_cami_subsets.py:343),
    # the full CAND_MAX of 5000 candidates (~20 Gbp, ten -I2g parts), ~2 Gbp of contigs,
    # three sketch DBs of 1e8 / 5e7 / 1e7 hashes
    if args.workload == "cami-high":
        args.taxa = 14
        args.per_taxon = [358] * 2 + [357] * 12
        args.contig_gbp = args.contig_gbp or 2.0
        args.db_hashes = args.db_hashes or "1e8,5e7,1e7"
        args.workload_name = "CAMI-high (C5)"
        # 5000 candidates: ~6x C4's anchors per query base, so smaller mapping batches
        args.batch_mbp = args.batch_mbp or 40.0
    else:
        args.contig_gbp = args.contig_gbp or 1.0
        args.db_hashes = args.db_hashes or "1e8"
        # C4: 60 Mbp batches measured 2327 ms/step vs 2460 (30) and ~2390 (40); scratch 148 GB
        args.batch_mbp = args.batch_mbp or 60.0
        args.workload_name = "CAMI-medium (C4)"
        if args.workload == "cami-medium-zymo":
            args.workload_name = "CAMI-medium on Zymo backbones (C4 shape, real sequence composition)"
    return args


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    from hymet_amd.dist import Comm
    comm = Comm.from_env()
    if comm.world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but the launcher started {comm.world} rank(s)")
    if args.dry_run:
        comm.init_backend(None, "gloo")
        res = bench_dry(args, comm)
        if comm.rank == 0:
            print(json.dumps(res), flush=True)
        comm.close()
        return
    import torch
    from hymet_amd._lib import Gpu
    if args.emulate_rank:
        if comm.world != 1:
            raise SystemExit("--emulate-rank runs in one process")
        gpu = Gpu(0)
        print(json.dumps(bench_emulate(args, gpu, torch)), flush=True)
        return
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.share_gpu:
        local %= max(1, torch.cuda.device_count())
    gpu = Gpu(local)
    comm.init_backend(gpu, None if args.backend == "auto" else args.backend)
    res = bench_screen(args, comm, gpu, torch) if args.workload == "screen" else bench_cami(args, comm, gpu, torch)
    if comm.rank == 0:
        print(json.dumps(res), flush=True)
    comm.close()


if __name__ == "__main__":
    main()

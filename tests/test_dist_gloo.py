"""Multi-rank host logic of the sharded path on CPU: world_size 2, gloo.

  * hymet_amd.screen.reduce_partials  -- screen hit counts summed, pool bottom-s merged,
    k-mer totals added (the exchange after each rank screens its own contig shard)
  * hymet_amd.dist.Comm.gather_rows   -- rank 0 assembles the fixed-size LCA row records of
    every contiguous query shard in the reference's first-PAF-appearance order
  * hymet_amd.dist.Comm collectives used by bench.py (barrier, max over ranks, gathers)
"""
import multiprocessing as mp
import os
import socket
import traceback

import numpy as np
import pytest


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn_name, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        from hymet_amd.dist import Comm
        comm = Comm(rank, world).init_backend(None, "gloo")
        try:
            out = globals()[fn_name](comm)
        finally:
            comm.close()
        q.put((rank, "ok", out))
    except Exception:
        q.put((rank, "err", traceback.format_exc()))


def _run_ranks(fn_name, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, fn_name, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        rank, status, out = q.get(timeout=240)
        assert status == "ok", out
        res[rank] = out
    for p in ps:
        p.join(timeout=60)
    return res


# ------------------------------------------------------------------ screen exchange
def _screen_data():
    rng = np.random.default_rng(3)
    counts = [rng.integers(0, 5, size=(2, 1001)).astype(np.int32) for _ in range(2)]   # [rank][db]
    cands = [np.unique(rng.integers(1, 2 ** 62, size=n, dtype=np.int64).astype(np.uint64)) for n in (700, 900)]
    nks = [12345, 67890]
    return counts, cands, nks


def _screen_fn(comm):
    import torch
    from hymet_amd.screen import _bottom_s, reduce_partials
    counts, cands, nks = _screen_data()
    mine = [torch.from_numpy(counts[comm.rank][d].copy()) for d in range(2)]
    c, b, nk = reduce_partials(comm, mine, _bottom_s(cands[comm.rank], 1000), nks[comm.rank], 1000)
    return [x.numpy() for x in c], b, nk


def test_screen_partials_reduce_like_one_pool():
    from hymet_amd.screen import _bottom_s
    res = _run_ranks("_screen_fn")
    counts, cands, nks = _screen_data()
    exp_b = _bottom_s(np.concatenate(cands), 1000)
    for r in (0, 1):
        c, b, nk = res[r]
        for d in range(2):
            np.testing.assert_array_equal(c[d], counts[0][d] + counts[1][d])
        np.testing.assert_array_equal(b, exp_b)
        assert nk == sum(nks)


def _screen_perm_fn(comm):
    """Each rank's table puts the same hashes in different slots (its own insertion order, as
    parallel insertion does); hits are counted per canonical index -- the smallest DB index
    holding the key, kept per slot (csrc/screen.hip table_insert_kernel) -- so the ranks'
    count arrays line up by hash and add up as they are."""
    import torch
    from hymet_amd.screen import reduce_partials
    rng = np.random.default_rng(21)
    H, S = 300, 1024
    keys = rng.integers(0, 200, size=H)            # duplicates: one key in several references
    hits = [rng.integers(0, 200, size=500) for _ in range(2)]   # [rank] the k-mer keys it sees
    # this rank's table: insertion in a rank-specific order, linear probing, canon = min index
    order = np.random.default_rng(100 + comm.rank).permutation(H)
    slot_key, slot_canon = {}, {}
    home = (np.random.default_rng(7).permutation(S))          # a fixed home slot per key value
    slot_of = np.zeros(H, np.int64)
    for j in order:
        s = int(home[keys[j] % S])
        while s in slot_key and slot_key[s] != keys[j]:
            s = (s + 1) % S
        slot_key[s] = keys[j]
        slot_canon[s] = min(slot_canon.get(s, H), int(j))
        slot_of[j] = s
    canon_of = np.array([slot_canon[int(slot_of[j])] for j in range(H)])
    by_key = {v: s for s, v in slot_key.items()}
    c = torch.zeros(H + 1, dtype=torch.int32)
    for k in hits[comm.rank]:
        if k in by_key:
            c[slot_canon[by_key[k]]] += 1
    out, _, _ = reduce_partials(comm, [c], np.zeros(0, np.uint64), 0, 10, None)
    got = out[0][torch.from_numpy(canon_of)].numpy()          # per DB hash, as screen_stats reads
    exp = np.array([sum(int((h == keys[j]).sum()) for h in hits) for j in range(H)], np.int32)
    return got, exp


def test_screen_counts_reduce_by_hash_not_slot():
    res = _run_ranks("_screen_perm_fn")
    for r in (0, 1):
        got, exp = res[r]
        np.testing.assert_array_equal(got, exp)


# ---------------------------------------------------------------- TSV row gather
def _global_rows():
    """120 queries of a pooled input; queries with hits get the index part of their first
    PAF line; the reference TSV order is (first part, input position)."""
    rng = np.random.default_rng(9)
    n = 120
    has = rng.random(n) < 0.8
    first_part = rng.integers(0, 3, size=n)
    lengths = rng.integers(1000, 100000, size=n)
    depth = rng.integers(0, 9, size=n)
    names = rng.integers(-1, 50, size=(n, 8))
    conf = rng.random(n)
    expect = sorted(np.flatnonzero(has).tolist(), key=lambda q: (first_part[q], q))
    return has, first_part, lengths, depth, names, conf, expect


def _gather_fn(comm):
    import torch
    has, first_part, lengths, depth, names, conf, _ = _global_rows()
    cuts = [0, 50, 120]                                   # contiguous shards (FastaIndex.shard)
    b, e = cuts[comm.rank], cuts[comm.rank + 1]
    local = [q for q in range(b, e) if has[q]]
    local.sort(key=lambda q: (first_part[q], q))          # rank-local row order (device LCA)
    rows = {"q": torch.tensor([q - b for q in local], dtype=torch.int32),
            "part": torch.tensor([first_part[q] for q in local], dtype=torch.int32),
            "depth": torch.tensor([depth[q] for q in local], dtype=torch.int32),
            "tax": torch.tensor([q * 3 for q in local], dtype=torch.int32),
            "names": torch.tensor(names[local].reshape(-1) if local else [], dtype=torch.int32),
            "conf": torch.tensor([conf[q] for q in local], dtype=torch.float64)}
    out, n = comm.gather_rows(rows, b)
    return n, {k: v.numpy() for k, v in out.items()}


def test_gather_rows_matches_pooled_order():
    res = _run_ranks("_gather_fn")
    has, first_part, lengths, depth, names, conf, expect = _global_rows()
    n, r = res[0]
    assert n == len(expect)
    assert r["q"].tolist() == expect
    assert r["part"].tolist() == [first_part[q] for q in expect]
    assert r["depth"].tolist() == [depth[q] for q in expect]
    assert r["tax"].tolist() == [q * 3 for q in expect]
    np.testing.assert_array_equal(r["names"].reshape(-1, 8), names[expect])
    assert r["conf"].tolist() == [conf[q] for q in expect]        # doubles travel bit-exact
    assert res[1][0] == 0


# ------------------------------------------------------------------ collectives
def _comm_fn(comm):
    mx = comm.max_float(1.5 + comm.rank)
    ag = comm.allgather_np(np.arange(3) + 10 * comm.rank)
    bc = comm.broadcast_obj({"sel": ["a", "b"]} if comm.rank == 0 else None)
    g = comm.gather_obj(comm.rank * 2)
    comm.barrier()
    return mx, [a.tolist() for a in ag], bc, g


def test_comm_collectives():
    res = _run_ranks("_comm_fn")
    for r in (0, 1):
        mx, ag, bc, g = res[r]
        assert mx == 2.5
        assert ag == [[0, 1, 2], [10, 11, 12]]
        assert bc == {"sel": ["a", "b"]}
    assert res[0][3] == [0, 2] and res[1][3] is None


def test_partition_and_shard_range():
    from hymet_amd.dist import Comm
    lengths = [5, 100, 7, 60, 60, 1, 1, 33]
    bins = Comm.partition_by_length(lengths, 3)
    assert sorted(np.concatenate(bins).tolist()) == list(range(len(lengths)))
    loads = [sum(lengths[i] for i in b) for b in bins]
    assert max(loads) - min(loads) <= max(lengths)
    spans = [Comm(r, 3).shard_range(10) for r in range(3)]
    assert spans == [(0, 3), (3, 6), (6, 10)]


# ------------------------------------------------- loader-thread placement of the DB load
def _loader_placement_fn(comm):
    """Pipeline.run's placement, with CPU tensors: the loader thread (pipeline.run_beside)
    holds the communicator (Comm.owned) and all-gathers two DBs' hash slices in place --
    Comm.allgather_slices_'s un-staged branch, all_gather_into_tensor on db_group, the RCCL
    path's call -- while the calling thread ingests; a collective the calling thread tries
    meanwhile is refused before it reaches the backend; after the join the calling thread runs
    the deferred record-count all-gather (Pipeline.shard_base's tag) on the default group."""
    import threading
    import time
    import torch
    from hymet_amd.pipeline import run_beside
    sizes = (1001, 64)                       # hashes per DB: ragged last slice, and c * world == H
    held, tried = threading.Event(), threading.Event()
    refused = []

    def loader():
        with comm.owned():
            held.set()
            tried.wait(60)
            out = []
            for d, h in enumerate(sizes):
                c = -(-h // comm.world)
                t = torch.full((comm.world * c,), -1, dtype=torch.int64)
                lo, hi = comm.rank * c, min(h, (comm.rank + 1) * c)
                t[lo:hi] = torch.arange(lo, hi, dtype=torch.int64) * 7 + d
                comm.allgather_slices_(t, c, key=d)
                out.append(t[:h].clone())
            time.sleep(0.2)                  # stands in for the table build behind the gathers
        return out

    got = []

    def ingest():
        held.wait(60)
        try:
            comm.allgather_np(np.array([1], np.int64), tag="shard_records")
        except RuntimeError as e:
            refused.append(str(e))
        tried.set()
        return 100 + comm.rank               # this rank's record count

    n = run_beside(lambda: got.extend(loader()), ingest)
    counts = comm.allgather_np(np.array([n], np.int64), tag="shard_records")
    q_base = int(sum(int(c[0]) for c in counts[:comm.rank]))
    return [g.numpy() for g in got], refused, q_base


def test_loader_thread_allgather_slices_and_deferred_record_counts():
    res = _run_ranks("_loader_placement_fn")
    for r in (0, 1):
        got, refused, q_base = res[r]
        for d, h in enumerate((1001, 64)):
            np.testing.assert_array_equal(got[d], np.arange(h, dtype=np.int64) * 7 + d)
        assert len(refused) == 1 and "holds the communicator" in refused[0]
        assert q_base == (0 if r == 0 else 100)


def test_comm_owner_guard_single_process():
    """The guard refuses another thread's collective while one thread holds the communicator,
    and lets the holder's own (and everyone's after release) through -- checked before any
    backend call, with a stand-in backend."""
    import threading
    from hymet_amd.dist import Comm

    class FakeDist:
        calls = 0

        def barrier(self):
            FakeDist.calls += 1
    c = Comm(0, 2)
    c.dist = FakeDist()
    errs = []

    def other():
        try:
            c.barrier()
        except RuntimeError as e:
            errs.append(e)
    with c.owned():
        c.barrier()                          # the holder's own
        th = threading.Thread(target=other)
        th.start()
        th.join()
        with c.owned():                      # re-entrant on the holding thread
            c.barrier()
    c.barrier()
    th = threading.Thread(target=other)
    th.start()
    th.join()
    assert len(errs) == 1 and FakeDist.calls == 4

"""FASTA record table (hymet_fasta_index, host C++) vs seqio.parse_fasta_bytes -- the
semantics the oracle and every earlier stage use (kseq-style records, first whitespace
token as the name, line breaks dropped) -- on edge cases and on a multi-MiB input that
takes the threaded path.  No GPU: the device half is tested in test_ingest_gpu.py."""
import numpy as np
import pytest

from hymet_amd.ingest import FastaIndex, to_fasta
from hymet_amd.seqio import parse_fasta_bytes

CASES = [
    b"",
    b">",
    b">a",
    b">a\n",
    b">a\nACGT",
    b">a\nACGT\n>b\n\n>c\nAC\nGT\n",
    b">a desc words\r\nAC\r\nGT\r\n>b\tx\r\nNNNN\r\n",
    b"junk line\n>first\nAAA\n>second\nCCC\n",
    b"no records at all\nACGT\n",
    b">  lead_ws name\nACGT\n",
    b">a>b\nAC>GT\n>c\n>d\nT",
    b">x\n\n\nA\n\nC\n",
    b"\n>y\nGG",
    b">\nAC\n",
]


def _check(data, threads=1):
    fx = FastaIndex(data, threads=threads)
    ref = parse_fasta_bytes(data)
    assert fx.n == len(ref)
    assert fx.names() == [r[0] for r in ref]
    for i, (_, _, seq) in enumerate(ref):
        raw = data[fx.seq_off[i]:fx.seq_end[i]].replace(b"\n", b"").replace(b"\r", b"")
        assert raw == seq
        assert fx.nbases[i] == len(seq)


@pytest.mark.parametrize("data", CASES)
def test_fasta_index_edge_cases(data):
    _check(data)


def test_fasta_index_threaded_large():
    rng = np.random.default_rng(3)
    names, seqs = [], []
    for i in range(3000):
        names.append(f"k141_{i} flag=1 multi={rng.random():.3f}")
        seqs.append(b"ACGTN"[0:4][0:4] * int(rng.integers(1, 800)))
    data = to_fasta(names, seqs, width=60)
    assert len(data) > (1 << 22)
    _check(data, threads=8)
    fx = FastaIndex(data, threads=8)
    r = [fx.shard(k, 3) for k in range(3)]
    assert r[0][0] == 0 and r[-1][1] == fx.n and all(r[i][1] == r[i + 1][0] for i in range(2))
    per = [int(fx.nbases[a:b].sum()) for a, b in r]
    assert max(per) - min(per) <= 2 * int(fx.nbases.max())
    pool, off = fx.name_pool(5, 9)
    assert pool.tobytes() == b"".join(n.split()[0].encode() for n in names[5:9]) and off[-1] == len(pool)


@pytest.mark.parametrize("world", [1, 2, 3, 5, 8, 64])
@pytest.mark.parametrize("data", CASES + [to_fasta([f"c{i} len={i}" for i in range(40)],
                                                  [b"ACGT" * (1 + 37 * i % 50) for i in range(40)], width=13)])
def test_byte_shards_partition_the_records(data, world):
    """ingest.shard_bytes + FastaIndex(byte_range=...): what each rank indexes of its own byte
    range, concatenated over the ranks, is the whole-file record table (names, sequences,
    base counts, absolute offsets) -- including junk before the first record, CRLF, '>' inside
    lines, empty records and more ranks than records -- and byte_shards predicts the split."""
    from hymet_amd.ingest import shard_bytes
    whole = FastaIndex(data)
    got = []
    prev_end = 0
    for r in range(world):
        b0, b1 = shard_bytes(data, r, world)
        assert b0 == prev_end and b0 <= b1
        prev_end = b1
        fx = FastaIndex(data, byte_range=(b0, b1))
        got.append(fx)
    assert prev_end == len(data)
    names = [n for fx in got for n in fx.names()]
    assert names == whole.names()
    for a in ("name_off", "name_len", "nbases"):
        np.testing.assert_array_equal(np.concatenate([getattr(fx, a) for fx in got]), getattr(whole, a))
    # sequences: a rank's last record ends at the range end, so its byte range may keep the
    # line break before the next '>' (a header-only record may then start one byte later);
    # the bases are the same
    seqs = [data[fx.seq_off[i]:fx.seq_end[i]].replace(b"\n", b"").replace(b"\r", b"") for fx in got for i in range(fx.n)]
    assert seqs == [data[a:b].replace(b"\n", b"").replace(b"\r", b"") for a, b in zip(whole.seq_off, whole.seq_end)]
    counts = [fx.n for fx in got]
    assert [b - a for a, b in whole.byte_shards(world)] == counts


def _greedy_batches(lengths, max_bases):
    """The batching rule spelled out record by record: a batch closes before the record
    that would take it past max_bases (a record longer than that sits alone)."""
    out, b0, acc = [], 0, 0
    for i, L in enumerate(lengths):
        if acc and acc + int(L) > max_bases:
            out.append((b0, i))
            b0, acc = i, 0
        acc += int(L)
    if b0 < len(lengths) or not out:
        out.append((b0, len(lengths)))
    return out


def test_mapping_batches_match_the_greedy_rule():
    from hymet_amd.ingest import _batches
    rng = np.random.default_rng(5)
    for _ in range(500):
        n = int(rng.integers(0, 80))
        lengths = rng.integers(1, 120, size=n)
        if n and rng.random() < 0.3:  # records longer than a batch
            lengths[rng.integers(0, n, size=min(n, 3))] = rng.integers(150, 600, size=min(n, 3))
        max_bases = int(rng.integers(1, 400))
        assert _batches(lengths, max_bases) == _greedy_batches(lengths, max_bases)

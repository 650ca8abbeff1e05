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

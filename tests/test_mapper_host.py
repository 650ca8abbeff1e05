"""Host-side logic of the align stage (no GPU)."""
import numpy as np


def test_split_parts_follows_minimap2_reader():
    from hymet_amd.mapper import parse_num, split_parts
    assert parse_num("2g") == 2_000_000_000 and parse_num("500k") == 500_000 and parse_num("4G") == 4_000_000_000
    lens = np.array([30_000_000] * 10)
    parts = split_parts(lens, batch_size=100e6, mini_batch=50e6)
    # mini-batches of 2 sequences (60 Mbp >= 50 Mbp); a part stops once it exceeds 100 Mbp
    assert [list(p) for p in parts] == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9]]

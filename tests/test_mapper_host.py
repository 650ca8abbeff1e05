"""Host-side logic of the align stage (no GPU)."""
import numpy as np


def test_split_parts_follows_minimap2_reader():
    from hymet_amd.mapper import parse_num, split_parts
    assert parse_num("2g") == 2_000_000_000 and parse_num("500k") == 500_000 and parse_num("4G") == 4_000_000_000
    lens = np.array([30_000_000] * 10)
    parts = split_parts(lens, batch_size=100e6, mini_batch=50e6)
    # mini-batches of 2 sequences (60 Mbp >= 50 Mbp); a part stops once it exceeds 100 Mbp
    assert [list(p) for p in parts] == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9]]


def test_index_manifest_mismatch_is_reported(tmp_path):
    """The manifest's reference/split fields are checked and reported (the index is still
    reused, as minimap2.sh:10's `[ -s ]` test does)."""
    import os
    from hymet_amd import mapper as mp
    ref = tmp_path / "combined_genomes.fasta"
    ref.write_text(">a\nACGT\n")
    st = os.stat(ref)
    man = {"reference": os.path.abspath(ref), "reference_size": st.st_size, "reference_mtime": st.st_mtime,
           "split_idx": "2g"}
    assert mp.index_mismatch(man, str(ref), "2g") == []
    assert mp.index_mismatch(man, None, None) == []
    assert any("-I 2g -> 1g" in m for m in mp.index_mismatch(man, str(ref), "1g"))
    ref.write_text(">a\nACGTACGT\n")
    assert any("size/mtime" in m for m in mp.index_mismatch(man, str(ref), "2g"))

"""CPU: the full-size row checker (tests/fullcheck.py) itself — its oracle rows are the scalar
restatement's, its digests are chunk.rs:40-46's, and a single flipped byte anywhere is named."""
import numpy as np
import pytest

import oracle as o
from fullcheck import compare_device_rows, oracle_rows, shard_oracle_digests

torch = pytest.importorskip("torch")

SEED, CSEED = 0xDEC05099, 0xC0EF0099


def test_oracle_rows_are_the_scalar_restatement_with_a_partial_last_chunkset():
    blob_len = 2 * o.CS + 12345          # chunksets 0, 1 full, chunkset 2 holds 12,345 data bytes
    rows = oracle_rows(SEED, CSEED, blob_len, 1, 3)
    assert rows.shape == (2 * o.N, o.F)
    for c in (1, 2):
        data = np.zeros(o.CS, np.uint8)
        have = min(o.CS, blob_len - c * o.CS)
        data[:have] = o.fill_random(SEED, blob_len)[c * o.CS:c * o.CS + have]
        cv = o.fill_random(CSEED, 3 * o.N * o.K)[c * o.N * o.K:(c + 1) * o.N * o.K]
        assert np.array_equal(rows[(c - 1) * o.N:c * o.N], o.chunkset_encode(data, cv, nthreads=4)), c


def test_digests_are_chunk_digests_with_global_ids():
    lo, hi = 2, 4
    blob_len = 4 * o.CS
    dig = shard_oracle_digests(lo, hi, SEED, CSEED, blob_len, batch=1, threads=2)
    rows = oracle_rows(SEED, CSEED, blob_len, lo, hi)
    for r in (0, 5, 16, 31):
        g = lo * o.N + r
        assert dig[r].tobytes() == o.chunk_digest(g // o.N, g, rows[r]), r


def test_compare_names_the_chunkset_of_a_flipped_byte():
    lo, hi = 5, 8
    blob_len = 8 * o.CS - 777
    ref = np.concatenate([oracle_rows(SEED, CSEED, blob_len, c, c + 1) for c in range(lo, hi)])
    dev = torch.from_numpy(ref.copy())
    assert compare_device_rows(dev, lo, hi, SEED, CSEED, blob_len, batch=2, threads=2) == (hi - lo) * o.N
    dev[(7 - lo) * o.N + 3, o.F - 1] ^= 0x40   # the last payload byte of chunkset 7's row 3
    with pytest.raises(AssertionError, match=r"chunkset 7: coded rows \[3\]"):
        compare_device_rows(dev, lo, hi, SEED, CSEED, blob_len, batch=2, threads=2)
    # a strided (payload-aligned pitch) view compares the same way
    pitch = 1048704
    buf = torch.zeros((hi - lo) * o.N * pitch, dtype=torch.uint8)
    view = buf.as_strided(((hi - lo) * o.N, o.F), (pitch, 1))
    view.copy_(torch.from_numpy(ref))
    assert compare_device_rows(view, lo, hi, SEED, CSEED, blob_len, batch=3, threads=2) == (hi - lo) * o.N

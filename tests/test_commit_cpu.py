"""Commitment layer on the CPU: the BLAKE3 restatement (oracle/blake3_oracle.c)
pinned by BLAKE3's published known answers, the product's host BLAKE3 / Merkle helpers against it,
and decds' Merkle semantics (merkle_tree.rs:23-146: zero-hash padding that climbs with the level,
proofs, verification)."""
import ctypes

import numpy as np
import pytest

from decds_amd import _capi
import oracle as o

# Published BLAKE3 known answers: the empty message, "abc", "hello world", and entries of the
# official test_vectors.json (input byte i = i mod 251, default 32-byte hash).
KAT = {
    b"": "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262",
    b"abc": "6437b3ac38465133ffb63b75273a8db548c558465d79db03fd359c6cd5bd9d85",
    b"hello world": "d74981efa70a0c880b8d8c1985d075dbcbf679b99a5f9914e5aaf96b831a9e24",
}
KAT_MOD251 = {
    1023: "10108970eeda3eb932baac1428c7a2163b0e924c9a9e25b35bba72b28f70bd11",
    1024: "42214739f095a406f3fc83deb889744ac00df831c10daa55189b5d121c855af7",
    1025: "d00278ae47eb27b34faecf67b4fe263f82d5412916c1ffd97c8cb7fb814b8444",
    2048: "e776b6028c7cd22a4d0ba182a8bf62205d2ef576467e838ed6f2529b85fba24a",
}


def host_blake3(data):
    buf = np.frombuffer(bytes(data), np.uint8).copy() if len(data) else np.zeros(1, np.uint8)
    out = np.empty(32, np.uint8)
    _capi.lib().decds_blake3(buf.ctypes.data, len(data), out.ctypes.data)
    return out.tobytes()


def mod251(n):
    return bytes(i % 251 for i in range(n))


def test_oracle_blake3_known_answers():
    for msg, h in KAT.items():
        assert o.blake3(msg).hex() == h
    for n, h in KAT_MOD251.items():
        assert o.blake3(mod251(n)).hex() == h


@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 1023, 1024, 1025, 2048, 2049, 3073, 8192, 8193, 16384, 16385, 49157,
                               65537, 1048603, 3 * 2**20 + 11])
def test_host_blake3_matches_oracle(n):
    msg = o.fill_random(n + 5, n).tobytes()
    assert host_blake3(msg) == o.blake3(msg)


def test_host_blake3_known_answers():
    for msg, h in KAT.items():
        assert host_blake3(msg).hex() == h
    for n, h in KAT_MOD251.items():
        assert host_blake3(mod251(n)).hex() == h


def test_chunk_digest_layout():
    # chunk.rs:40-46: BLAKE3(chunkset_id u64 LE || chunk_id u64 LE || data)
    data = o.fill_random(3, 1000)
    d = o.chunk_digest(7, 7 * 16 + 3, data)
    assert d == o.blake3((7).to_bytes(8, "little") + (115).to_bytes(8, "little") + data.tobytes())


def test_host_chunk_digest_matches_oracle():
    # the host Chunk::digest the chunkset mirror's add_chunk validates with, on a full coded piece
    from decds_amd.chunkset import Chunk
    data = o.fill_random(11, 1048587)
    for cs_id, chunk_id in [(0, 0), (7, 7 * 16 + 3), (2**40 + 1, (2**40 + 1) * 16 + 15)]:
        out = ctypes.create_string_buffer(32)
        _capi.lib().decds_chunk_digest(cs_id, chunk_id, data.tobytes(), data.size, out)
        assert out.raw == o.chunk_digest(cs_id, chunk_id, data)
        assert Chunk(cs_id, chunk_id, data.tobytes()).digest() == out.raw


def test_host_chunk_validation_semantics():
    # chunk.rs:88-110 over a 3-chunkset blob built from synthetic digests: chunkset-level proofs are
    # the first 4 hashes, the blob-level path follows (chunkset.rs:98-102)
    from decds_amd.chunkset import Chunk
    rows = {(c, c * 16 + j): o.fill_random(100 * c + j, 257).tobytes() for c in range(3) for j in range(16)}
    leaves = {k: o.chunk_digest(k[0], k[1], np.frombuffer(v, np.uint8)) for k, v in rows.items()}
    cs_roots, cs_proofs = [], []
    for c in range(3):
        r, p = o.merkle([leaves[(c, c * 16 + j)] for j in range(16)])
        cs_roots.append(r)
        cs_proofs.append(p)
    blob_root, blob_proofs = o.merkle(cs_roots)
    for (c, gid), data in rows.items():
        ch = Chunk(c, gid, data, cs_proofs[c][gid % 16] + blob_proofs[c])
        assert ch.validate_inclusion_in_chunkset(cs_roots[c])
        assert ch.validate_inclusion_in_blob(blob_root)
        assert not ch.validate_inclusion_in_chunkset(cs_roots[(c + 1) % 3])
        short = Chunk(c, gid, data, cs_proofs[c][gid % 16][:3])
        assert not short.validate_inclusion_in_chunkset(cs_roots[c])
        wrong_id = Chunk(c, gid ^ 1, data, cs_proofs[c][gid % 16] + blob_proofs[c])
        assert not wrong_id.validate_inclusion_in_blob(blob_root)


def host_merkle(leaves):
    n = len(leaves)
    depth = max(0, (n - 1).bit_length())
    lv = np.frombuffer(b"".join(leaves), np.uint8).copy()
    root = np.empty(32, np.uint8)
    proofs = np.empty(max(1, n * depth * 32), np.uint8)
    assert _capi.lib().decds_merkle_tree(lv.ctypes.data, n, root.ctypes.data, proofs.ctypes.data) == depth
    return root.tobytes(), [[proofs[(i * depth + k) * 32:(i * depth + k + 1) * 32].tobytes() for k in range(depth)]
                            for i in range(n)]


@pytest.mark.parametrize("n", [1, 2, 3, 5, 16, 17, 103])
def test_merkle_host_matches_oracle_and_verifies(n):
    leaves = [o.blake3(i.to_bytes(4, "little")) for i in range(n)]
    root, proofs = o.merkle(leaves)
    hroot, hproofs = host_merkle(leaves)
    assert hroot == root and hproofs == proofs
    lib = _capi.lib()
    for i in range(n):
        assert o.merkle_verify(i, leaves[i], proofs[i], root)
        pf = np.frombuffer(b"".join(proofs[i]) or b"\0", np.uint8).copy()
        assert lib.decds_merkle_verify(i, leaves[i], pf.ctypes.data, len(proofs[i]), root) == 1
    if n > 1:  # a flipped bit in a proof fails (merkle_tree.rs:185-231)
        bad = [bytearray(p) for p in proofs[0]]
        bad[0][3] ^= 0x10
        assert not o.merkle_verify(0, leaves[0], [bytes(b) for b in bad], root)


def test_merkle_three_leaves_by_hand():
    # merkle_tree.rs:31-45: odd levels pair with a zero hash, which is re-hashed per level
    a, b, c = (o.blake3(bytes([i])) for i in range(3))
    z = bytes(32)
    ab, cz = o.blake3(a + b), o.blake3(c + z)
    assert o.merkle([a, b, c])[0] == o.blake3(ab + cz)
    root5 = o.merkle([a, b, c, a, b])[0]
    z1 = o.blake3(z + z)
    l1 = [ab, o.blake3(c + a), o.blake3(b + z)]
    l2 = [o.blake3(l1[0] + l1[1]), o.blake3(l1[2] + z1)]
    assert root5 == o.blake3(l2[0] + l2[1])


def _stream_blake3(data, cuts, threads=4):
    L = _capi.lib()
    s = L.decds_blake3_stream_new()
    try:
        lo = 0
        for hi in list(cuts) + [data.size]:
            L.decds_blake3_stream_update(s, data[lo:hi].ctypes.data if hi > lo else None, hi - lo, threads)
            lo = hi
        out = np.empty(32, np.uint8)
        L.decds_blake3_stream_finalize(s, out.ctypes.data)
        return out.tobytes()
    finally:
        L.decds_blake3_stream_free(s)


def test_blake3_stream_matches_one_shot_for_any_split():
    # blake3::Hasher semantics (lazy CV-stack merges, aligned power-of-two subtrees, one chunk held
    # back): every split of the message gives the one-shot hash; KAT lengths pinned as well
    for n, h in KAT_MOD251.items():
        d = np.frombuffer(mod251(n), np.uint8).copy()
        assert _stream_blake3(d, []).hex() == h
        assert _stream_blake3(d, [1, 1024 % max(1, n)] if n > 1024 else [n // 2]).hex() == h
    rng = np.random.default_rng(0xB3)
    for n in (0, 1, 64, 1024, 1025, 2048, 2049, 3 * 1024 + 5, 8192, (1 << 20) + 17, 5 * (1 << 20) + 3,
              10 * (1 << 20) * 3 - 99):
        d = rng.integers(0, 256, n, dtype=np.uint8)
        want = host_blake3(d.tobytes()) if n < (1 << 20) else None
        if want is None:
            out = np.empty(32, np.uint8)
            _capi.lib().decds_blake3_parallel(d.ctypes.data, n, out.ctypes.data, 4)
            want = out.tobytes()
        assert _stream_blake3(d, []) == want, n
        for _ in range(4):
            k = int(rng.integers(1, 6))
            cuts = sorted(int(c) for c in rng.integers(0, n + 1, k)) if n else []
            assert _stream_blake3(d, cuts) == want, (n, cuts)
        if n >= 3 * 1024:  # pieces ending exactly on chunk / power-of-two boundaries
            cuts = [c for c in (1024, 2048, 4096, 10 << 20, 20 << 20) if c < n]
            assert _stream_blake3(d, cuts) == want, (n, cuts)
    assert _stream_blake3(np.zeros(0, np.uint8), [0, 0]) == bytes.fromhex(KAT[b""])

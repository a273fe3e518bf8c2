"""Wire / on-disk format: bincode 2 standard() encodings of ProofCarryingChunk and
BlobHeader (chunk.rs:152-170, blob.rs:168-197) — byte layout against an independent restatement of
the bincode rules, the reference's own round-trip / truncation tests (chunk.rs:205-233), and the
parallel host BLAKE3 used for the blob digest. Parity of the layout itself is unpinned: the
reference ships no serialized fixture."""
import ctypes
import struct

import numpy as np
import pytest

from decds_amd import wire
from decds_amd._capi import CHUNKSET_BYTES as CS, DecdsError, lib
from decds_amd.chunkset import Chunk
import oracle as o


def varint(v):
    # bincode 2 varint (config::standard()): < 251 one byte, else tag 251/252/253 + u16/u32/u64 LE
    if v < 251:
        return bytes([v])
    if v <= 0xFFFF:
        return b"\xfb" + struct.pack("<H", v)
    if v <= 0xFFFFFFFF:
        return b"\xfc" + struct.pack("<I", v)
    return b"\xfd" + struct.pack("<Q", v)


def expected_pcc(cs, ch, data, proof):
    return varint(cs) + varint(ch) + varint(len(data)) + data + varint(len(proof)) + b"".join(proof)


@pytest.mark.parametrize("cs,ch", [(0, 0), (5, 300), (250, 251), (65535, 65536), (2**32 - 1, 2**32), (2**40, 2**63)])
def test_pcc_layout_and_round_trip(cs, ch):
    data = o.fill_random(cs % 97 + ch % 89, 777).tobytes()
    proof = [o.fill_random(1000 + i, 32).tobytes() for i in range(6)]
    c = Chunk(cs, ch, data, proof)
    b = wire.pcc_to_bytes(c)
    assert b == expected_pcc(cs, ch, data, proof)
    c2, n = wire.pcc_from_bytes(b)
    assert n == len(b)
    assert (c2.chunkset_id, c2.chunk_id, c2.erasure_coded_data, c2.proof) == (cs, ch, data, proof)


def test_pcc_full_size_chunk_length_prefix():
    # a real coded chunk: 1,048,587 data bytes -> length tag 0xFC + u32 LE; 4 + 11 proof hashes
    data = o.fill_random(9, 1048587).tobytes()
    proof = [bytes([i]) * 32 for i in range(15)]
    b = wire.pcc_to_bytes(Chunk(1638, 1638 * 16 + 15, data, proof))
    assert b[:3] == b"\xfb" + struct.pack("<H", 1638)
    assert b[3:6] == b"\xfb" + struct.pack("<H", 1638 * 16 + 15)
    assert b[6:11] == b"\xfc" + struct.pack("<I", 1048587)
    assert len(b) == 11 + 1048587 + 1 + 15 * 32


def test_pcc_truncated_and_trailing_bytes():
    # chunk.rs:231: decoding half of the bytes fails; every strict prefix fails
    data = o.fill_random(3, 300).tobytes()
    b = wire.pcc_to_bytes(Chunk(2, 35, data, [bytes(32)] * 4))
    for cut in [0, 1, 2, 3, 4, 5, len(b) // 2, len(b) - 33, len(b) - 1]:
        with pytest.raises(DecdsError) as e:
            wire.pcc_from_bytes(b[:cut])
        assert e.value.kind == "ProofCarryingChunkDeserializationFailed"
    # trailing bytes are not consumed (decds-bin rejects files with trailing bytes, utils.rs:60-70)
    c, n = wire.pcc_from_bytes(b + b"\x00\x01")
    assert n == len(b)
    # invalid varint tags
    for bad in [b"\xfe" + bytes(16), b"\xff" + bytes(8)]:
        with pytest.raises(DecdsError):
            wire.pcc_from_bytes(bad)


def test_blob_header_layout_round_trip_and_mismatch():
    roots = [o.fill_random(50 + i, 32).tobytes() for i in range(103)]
    digest, root = o.blake3(b"blob"), o.blake3(b"root")
    h = wire.BlobHeader(1 << 30, 103, digest, root, roots)
    b = h.to_bytes()
    assert b == varint(1 << 30) + varint(103) + digest + root + varint(103) + b"".join(roots)
    h2, n = wire.BlobHeader.from_bytes(b)
    assert n == len(b) and h2 == h
    # blob.rs:187-191: num_chunksets must equal the number of roots
    bad = wire.BlobHeader(1 << 30, 104, digest, root, roots).to_bytes()
    with pytest.raises(DecdsError) as e:
        wire.BlobHeader.from_bytes(bad)
    assert e.value.kind == "BlobHeaderDeserializationFailed"
    with pytest.raises(DecdsError) as e:
        wire.BlobHeader.from_bytes(b[:-1])
    assert e.value.kind == "BlobHeaderDeserializationFailed"


def test_serialize_into_too_small_buffer_fails():
    out = ctypes.create_string_buffer(10)
    w = ctypes.c_size_t()
    st = lib().decds_pcc_to_bytes(0, 0, b"x" * 20, 20, None, 0, out, 10, ctypes.byref(w))
    assert st == 14  # DECDS_ERR_PCC_SERIALIZATION_FAILED


@pytest.mark.parametrize("n,threads", [(0, 4), (1025, 8), (3 << 20, 8), ((5 << 20) + 123, 16), (1 << 22, 3)])
def test_parallel_blake3_matches_oracle(n, threads):
    msg = o.fill_random(n + 17, n).tobytes()
    out = ctypes.create_string_buffer(32)
    lib().decds_blake3_parallel(msg, n, out, threads)
    assert out.raw == o.blake3(msg)


def _header_2_5():
    # a 2.5-chunkset blob's header (blob.rs:507-631 build theirs with Blob::new; the queries read
    # only the sizes and roots)
    from decds_amd.wire import BlobHeader
    n = 3
    roots = [bytes([i]) * 32 for i in range(n)]
    return BlobHeader(2 * CS + CS // 2, n, b"\1" * 32, b"\2" * 32, roots)


def _err(kind, fn, *a, **kw):
    with pytest.raises(DecdsError) as e:
        fn(*a, **kw)
    assert e.value.kind == kind, e.value
    return e.value


def test_blob_header_chunkset_queries_like_reference():
    h = _header_2_5()
    assert h.get_num_chunks() == 48
    # blob.rs:507-526 get_chunkset_commitment
    assert h.get_chunkset_commitment(0) == b"\0" * 32 and h.get_chunkset_commitment(1) == b"\1" * 32
    _err("InvalidChunksetId", h.get_chunkset_commitment, 3)
    # blob.rs:529-551 get_chunkset_size
    assert [h.get_chunkset_size(c) for c in range(3)] == [CS, CS, CS // 2]
    _err("InvalidChunksetId", h.get_chunkset_size, 3)
    # blob.rs:554-580 get_byte_range_for_chunkset
    assert h.get_byte_range_for_chunkset(0) == (0, CS)
    assert h.get_byte_range_for_chunkset(1) == (CS, 2 * CS)
    assert h.get_byte_range_for_chunkset(2) == (2 * CS, 2 * CS + CS // 2)
    _err("InvalidChunksetId", h.get_byte_range_for_chunkset, 3)


def test_blob_header_chunkset_ids_for_byte_range_like_reference():
    # blob.rs:583-631
    h = _header_2_5()
    blen = h.get_blob_size()
    q = h.get_chunkset_ids_for_byte_range
    assert q(0, 10) == [0] and q(range(0, 10)) == [0]
    assert q(CS + 10, CS + 20) == [1]
    assert q(10, CS + 10) == [0, 1]
    assert q(10, blen) == [0, 1, 2]
    assert q(0, CS) == [0]
    assert q(0, CS - 1, end_inclusive=True) == [0]
    _err("InvalidEndBound", q, 0, 0)
    assert q(0, 0, end_inclusive=True) == [0]
    beyond = blen + CS
    e = _err("InvalidChunksetId", q, 0, beyond)
    assert str((beyond - 1) // CS) in str(e)
    _err("InvalidEndBound", q, None, None)
    _err("InvalidEndBound", q, 0, None)

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
from decds_amd._capi import DecdsError, lib
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

"""decds' wire / on-disk format over the C-ABI (decds_amd/csrc/wire.cpp): bincode 2 `standard()`
(consts.rs:2) encodings of ProofCarryingChunk (chunk.rs:152-170) and BlobHeader (blob.rs:15-21,
168-197), with the reference's method names."""
import ctypes

from ._capi import CHUNKSET_BYTES, N, STATUS, DecdsError, check, lib
from .chunkset import Chunk


def pcc_to_bytes(chunk):
    """ProofCarryingChunk::to_bytes"""
    data = bytes(chunk.get_erasure_coded_data())
    proof = b"".join(chunk.get_proof())
    n = len(chunk.get_proof())
    cap = lib().decds_pcc_encoded_len(chunk.get_chunkset_id(), chunk.get_global_chunk_id(), len(data), n)
    out = ctypes.create_string_buffer(cap)
    w = ctypes.c_size_t()
    check(lib().decds_pcc_to_bytes(chunk.get_chunkset_id(), chunk.get_global_chunk_id(), data, len(data), proof, n,
                                   out, cap, ctypes.byref(w)))
    return out.raw[:w.value]


def pcc_from_bytes(buf):
    """ProofCarryingChunk::from_bytes -> (Chunk with proof, bytes read)"""
    b = bytes(buf)
    cs, ch = ctypes.c_uint64(), ctypes.c_uint64()
    d, p = ctypes.c_void_p(), ctypes.c_void_p()
    dl, pl, used = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
    src = ctypes.create_string_buffer(b, len(b))
    check(lib().decds_pcc_from_bytes(src, len(b), ctypes.byref(cs), ctypes.byref(ch), ctypes.byref(d),
                                     ctypes.byref(dl), ctypes.byref(p), ctypes.byref(pl), ctypes.byref(used)))
    base = ctypes.addressof(src)
    doff = (d.value or base) - base
    poff = (p.value or base) - base
    data = b[doff:doff + dl.value]
    proof = [b[poff + 32 * k:poff + 32 * (k + 1)] for k in range(pl.value)]
    return Chunk(cs.value, ch.value, data, proof), used.value


class BlobHeader:
    """BlobHeader (blob.rs:15-21)."""

    def __init__(self, byte_length, num_chunksets, digest, root_commitment, chunkset_root_commitments):
        self.byte_length = byte_length
        self.num_chunksets = num_chunksets
        self.digest = bytes(digest)
        self.root_commitment = bytes(root_commitment)
        self.chunkset_root_commitments = [bytes(r) for r in chunkset_root_commitments]

    def get_blob_size(self):
        return self.byte_length

    def get_num_chunksets(self):
        return self.num_chunksets

    def get_blob_digest(self):
        return self.digest

    def get_root_commitment(self):
        return self.root_commitment

    def get_num_chunks(self):
        """blob.rs:38-40"""
        return self.num_chunksets * N

    def _check_id(self, chunkset_id):
        if not 0 <= chunkset_id < self.num_chunksets:
            raise DecdsError(STATUS["InvalidChunksetId"],
                             "invalid chunkset id: %d (num_chunksets: %d)" % (chunkset_id, self.num_chunksets))

    def get_chunkset_commitment(self, chunkset_id):
        """blob.rs:65-71"""
        self._check_id(chunkset_id)
        return self.chunkset_root_commitments[chunkset_id]

    def get_chunkset_size(self, chunkset_id):
        """blob.rs:84-94: the chunkset's real byte count (the last one may be partial)"""
        lo, hi = self.get_byte_range_for_chunkset(chunkset_id)
        return hi - lo

    def get_byte_range_for_chunkset(self, chunkset_id):
        """blob.rs:108-117: [start, end) of the chunkset within the blob"""
        self._check_id(chunkset_id)
        lo = chunkset_id * CHUNKSET_BYTES
        return lo, min(lo + CHUNKSET_BYTES, self.byte_length)

    def get_chunkset_ids_for_byte_range(self, start=None, end=None, end_inclusive=False):
        """blob.rs:132-160 with Rust's RangeBounds spelled out: start None = unbounded (0), else included;
        end None = unbounded (InvalidEndBound(usize::MAX)), else excluded, or included if end_inclusive
        (`a..b` -> (a, b); `a..=b` -> (a, b, True); `..` -> (None, None)). A Python range works too."""
        if isinstance(start, range):
            if start.step != 1:
                raise ValueError("byte ranges have step 1")
            start, end, end_inclusive = start.start, start.stop, False
        if start is not None and start < 0:
            raise DecdsError(STATUS["InvalidStartBound"], "invalid start bound")
        first = 0 if start is None else start
        if end is None:
            raise DecdsError(STATUS["InvalidEndBound"], "invalid end bound: %d" % (2**64 - 1))
        if end_inclusive:
            last = end
        else:
            if end == 0:
                raise DecdsError(STATUS["InvalidEndBound"], "invalid end bound: 0")
            last = end - 1
        a, b = first // CHUNKSET_BYTES, last // CHUNKSET_BYTES
        if b >= self.num_chunksets:
            raise DecdsError(STATUS["InvalidChunksetId"],
                             "invalid chunkset id: %d (num_chunksets: %d)" % (b, self.num_chunksets))
        return list(range(a, b + 1))

    def validate_chunk(self, chunk):
        """blob.rs:211-215: the chunk's blob-level path against the root, its chunkset id in range and its
        chunkset-level path against that chunkset's root (host BLAKE3, chunk.rs:88-110)"""
        cs = chunk.get_chunkset_id()
        return (chunk.validate_inclusion_in_blob(self.root_commitment) and cs < self.num_chunksets
                and chunk.validate_inclusion_in_chunkset(self.chunkset_root_commitments[cs]))

    def to_bytes(self):
        """BlobHeader::to_bytes (blob.rs:168-170)"""
        roots = b"".join(self.chunkset_root_commitments)
        n = len(self.chunkset_root_commitments)
        cap = lib().decds_blob_header_encoded_len(self.byte_length, self.num_chunksets, n)
        out = ctypes.create_string_buffer(cap)
        w = ctypes.c_size_t()
        check(lib().decds_blob_header_to_bytes(self.byte_length, self.num_chunksets, self.digest, self.root_commitment,
                                               roots, n, out, cap, ctypes.byref(w)))
        return out.raw[:w.value]

    @classmethod
    def from_bytes(cls, buf):
        """BlobHeader::from_bytes (blob.rs:183-197) -> (header, bytes read)"""
        b = bytes(buf)
        src = ctypes.create_string_buffer(b, len(b))
        bl, nc = ctypes.c_uint64(), ctypes.c_uint64()
        dg, rt = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
        rp, nr, used = ctypes.c_void_p(), ctypes.c_size_t(), ctypes.c_size_t()
        check(lib().decds_blob_header_from_bytes(src, len(b), ctypes.byref(bl), ctypes.byref(nc), dg, rt,
                                                 ctypes.byref(rp), ctypes.byref(nr), ctypes.byref(used)))
        off = (rp.value or ctypes.addressof(src)) - ctypes.addressof(src)
        roots = [b[off + 32 * k:off + 32 * (k + 1)] for k in range(nr.value)]
        return cls(bl.value, nc.value, dg.raw, rt.raw, roots), used.value

    def __eq__(self, other):
        return isinstance(other, BlobHeader) and vars(self) == vars(other)

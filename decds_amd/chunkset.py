"""Python mirror of decds-lib's chunkset API over the C-ABI (decds-lib/src/chunkset.rs).

Names, argument meaning and errors follow the reference so the parity tests read like the
reference's own tests (chunkset.rs:211-481). The BLAKE3/Merkle commitment (chunkset.rs:54-63) and
proof validation (`add_chunk`, chunkset.rs:151-157) belong to the out-of-scope integrity layer;
`add_chunk_unvalidated` is the hot-path entry.
"""
import ctypes

from . import _capi
from ._capi import CHUNKSET_BYTES, CODED_PIECE_BYTES, DecdsError, K, N, check, lib


class Context:
    """One gfx950 device (decds_ctx). Defaults: GF(2^8) poly 0x11D, marker 0x81 (rlnc 0.4.0)."""

    def __init__(self, device=0):
        h = ctypes.c_void_p()
        check(lib().decds_ctx_create(int(device), ctypes.byref(h)))
        self._h = h
        self.device = device

    @property
    def handle(self):
        return self._h

    def set_field(self, poly, marker):
        check(lib().decds_ctx_set_field(self._h, poly, marker))

    def field(self):
        p, m = ctypes.c_uint32(), ctypes.c_uint8()
        check(lib().decds_ctx_get_field(self._h, ctypes.byref(p), ctypes.byref(m)))
        return p.value, m.value

    def close(self):
        if self._h:
            lib().decds_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Chunk:
    """decds-lib Chunk (chunk.rs:7-11) without its digest: ids + erasure-coded data."""

    __slots__ = ("chunkset_id", "chunk_id", "erasure_coded_data")

    def __init__(self, chunkset_id, chunk_id, erasure_coded_data):
        self.chunkset_id = chunkset_id
        self.chunk_id = chunk_id
        self.erasure_coded_data = erasure_coded_data

    def get_chunkset_id(self):
        return self.chunkset_id

    def get_erasure_coded_data(self):
        return self.erasure_coded_data


class ChunkSet:
    """ChunkSet (chunkset.rs:12-103): 10 MiB -> 16 RLNC-coded chunks."""

    NUM_ORIGINAL_CHUNKS = K
    BYTE_LENGTH = CHUNKSET_BYTES
    NUM_ERASURE_CODED_CHUNKS = N

    def __init__(self, ctx, chunkset_id, data, coeffs=None):
        """ChunkSet::new (chunkset.rs:37-69). `coeffs` (16x10 bytes) pins the coding vectors the
        reference draws from rand::rng(); None draws them from the library's RNG."""
        buf = bytes(data)
        cv = None if coeffs is None else bytes(coeffs)
        if cv is not None and len(cv) != N * K:
            raise ValueError("coeffs must be 16*10 bytes")
        h = ctypes.c_void_p()
        check(lib().decds_chunkset_new(ctx.handle, chunkset_id, buf, len(buf), cv, ctypes.byref(h)))
        self._h = h
        self.chunkset_id = chunkset_id

    @classmethod
    def new(cls, ctx, chunkset_id, data, coeffs=None):
        return cls(ctx, chunkset_id, data, coeffs)

    def get_chunk(self, chunk_id):
        """ChunkSet::get_chunk (chunkset.rs:87-89)."""
        out = ctypes.create_string_buffer(CODED_PIECE_BYTES)
        gid = ctypes.c_size_t()
        check(lib().decds_chunkset_get_chunk(self._h, chunk_id, out, CODED_PIECE_BYTES, ctypes.byref(gid)))
        return Chunk(self.chunkset_id, gid.value, out.raw)

    def __del__(self):
        try:
            if self._h:
                lib().decds_chunkset_free(self._h)
                self._h = None
        except Exception:
            pass


class RepairingChunkSet:
    """RepairingChunkSet (chunkset.rs:107-208)."""

    def __init__(self, ctx, chunkset_id):
        h = ctypes.c_void_p()
        check(lib().decds_repairing_chunkset_new(ctx.handle, chunkset_id, ctypes.byref(h)))
        self._h = h
        self.chunkset_id = chunkset_id

    def add_chunk_unvalidated(self, chunk):
        """chunkset.rs:173-184; raises DecdsError(InvalidChunkMetadata | ChunksetReadyToRepair |
        ChunkDecodingFailed)."""
        data = bytes(chunk.get_erasure_coded_data())
        check(lib().decds_repairing_chunkset_add_chunk_unvalidated(self._h, chunk.get_chunkset_id(), data, len(data)))

    def is_ready_to_repair(self):
        return bool(lib().decds_repairing_chunkset_is_ready_to_repair(self._h))

    def repair(self):
        """chunkset.rs:200-208; raises DecdsError(ChunksetNotYetReadyToRepair | ChunksetRepairingFailed)."""
        out = ctypes.create_string_buffer(CHUNKSET_BYTES)
        check(lib().decds_repairing_chunkset_repair(self._h, out, CHUNKSET_BYTES))
        return out.raw

    def __del__(self):
        try:
            if self._h:
                lib().decds_repairing_chunkset_free(self._h)
                self._h = None
        except Exception:
            pass


__all__ = ["Context", "Chunk", "ChunkSet", "RepairingChunkSet", "DecdsError"]

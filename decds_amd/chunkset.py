"""Python mirror of decds-lib's chunkset API over the C-ABI (decds-lib/src/chunkset.rs).

Names, argument meaning and errors follow the reference so the parity tests read like the
reference's own tests (chunkset.rs:211-481), including ChunkSet::new's commitment (chunkset.rs:54-63,
computed on the device) and RepairingChunkSet::add_chunk's proof check (chunkset.rs:151-157).
"""
import ctypes

from . import _capi
from ._capi import CHUNKSET_BYTES, CODED_PIECE_BYTES, DecdsError, K, N, check, lib


class Context:
    """One gfx950 device (decds_ctx). Defaults: GF(2^8) poly 0x11D, marker 0x81 (rlnc 0.4.0)."""

    def __init__(self, device=0):
        import weakref
        h = ctypes.c_void_p()
        check(lib().decds_ctx_create(int(device), ctypes.byref(h)))
        self._h = h
        self.device = device
        self._dependents = weakref.WeakSet()  # Blob / RepairingBlob objects built on this context

    def _adopt(self, obj):
        """obj (with a free() method) is released before this context is destroyed"""
        self._dependents.add(obj)

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
        """destroys the context; objects built on it (Blob, RepairingBlob) are released first, so
        none of them outlives the device state it uses"""
        if self._h:
            for d in list(getattr(self, "_dependents", ())):
                d.free()
            lib().decds_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Chunk:
    """decds-lib ProofCarryingChunk (chunk.rs:7-11, 58-150): ids, erasure-coded data, proof."""

    __slots__ = ("chunkset_id", "chunk_id", "erasure_coded_data", "proof")

    def __init__(self, chunkset_id, chunk_id, erasure_coded_data, proof=()):
        self.chunkset_id = chunkset_id
        self.chunk_id = chunk_id
        self.erasure_coded_data = erasure_coded_data
        self.proof = list(proof)  # 32-byte hashes

    def get_chunkset_id(self):
        return self.chunkset_id

    def get_global_chunk_id(self):
        return self.chunk_id

    def get_local_chunk_id(self):
        return self.chunk_id % N

    def get_erasure_coded_data(self):
        return self.erasure_coded_data

    def get_proof(self):
        return list(self.proof)

    def digest(self):
        """Chunk::digest (chunk.rs:40-46), host BLAKE3."""
        data = bytes(self.erasure_coded_data)
        out = ctypes.create_string_buffer(32)
        lib().decds_chunk_digest(self.chunkset_id, self.chunk_id, data, len(data), out)
        return out.raw

    def validate_inclusion_in_chunkset(self, chunkset_commitment):
        """chunk.rs:103-110; a proof shorter than PROOF_SIZE is invalid (the reference panics)."""
        if len(self.proof) < PROOF_SIZE:
            return False
        p = b"".join(self.proof[:PROOF_SIZE])
        return bool(lib().decds_merkle_verify(self.get_local_chunk_id(), self.digest(), p, PROOF_SIZE,
                                              bytes(chunkset_commitment)))

    def validate_inclusion_in_blob(self, blob_commitment):
        """chunk.rs:88-90."""
        p = b"".join(self.proof)
        return bool(lib().decds_merkle_verify(self.chunk_id, self.digest(), p, len(self.proof), bytes(blob_commitment)))


PROOF_SIZE = 4  # ChunkSet::PROOF_SIZE (chunkset.rs:22)


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
        """ChunkSet::get_chunk (chunkset.rs:87-89): the proof-carrying chunk."""
        out = ctypes.create_string_buffer(CODED_PIECE_BYTES)
        gid = ctypes.c_size_t()
        check(lib().decds_chunkset_get_chunk(self._h, chunk_id, out, CODED_PIECE_BYTES, ctypes.byref(gid)))
        plen = ctypes.c_size_t()
        check(lib().decds_chunkset_get_chunk_proof(self._h, chunk_id, None, 0, ctypes.byref(plen)))
        pbuf = ctypes.create_string_buffer(32 * plen.value)
        check(lib().decds_chunkset_get_chunk_proof(self._h, chunk_id, pbuf, len(pbuf), ctypes.byref(plen)))
        proof = [pbuf.raw[32 * k:32 * (k + 1)] for k in range(plen.value)]
        return Chunk(self.chunkset_id, gid.value, out.raw, proof)

    def get_root_commitment(self):
        """ChunkSet::get_root_commitment (chunkset.rs:72-74)."""
        out = ctypes.create_string_buffer(32)
        check(lib().decds_chunkset_get_root_commitment(self._h, out))
        return out.raw

    def append_blob_inclusion_proof(self, blob_proof):
        """ChunkSet::append_blob_inclusion_proof (chunkset.rs:98-102)."""
        b = b"".join(bytes(h) for h in blob_proof)
        check(lib().decds_chunkset_append_blob_inclusion_proof(self._h, b, len(blob_proof)))

    def __del__(self):
        try:
            if self._h:
                lib().decds_chunkset_free(self._h)
                self._h = None
        except Exception:
            pass


class RepairingChunkSet:
    """RepairingChunkSet (chunkset.rs:107-208)."""

    def __init__(self, ctx, chunkset_id, commitment=None):
        """RepairingChunkSet::new(chunkset_id, commitment) (chunkset.rs:129-135)."""
        h = ctypes.c_void_p()
        cm = None if commitment is None else bytes(commitment)
        check(lib().decds_repairing_chunkset_new(ctx.handle, chunkset_id, cm, ctypes.byref(h)))
        self._h = h
        self._ctx = ctx  # repair() runs on the context's device: keep it alive
        if hasattr(ctx, "_adopt"):
            ctx._adopt(self)  # ... and an explicit ctx.close() releases this object first
        self.chunkset_id = chunkset_id

    def add_chunk(self, chunk):
        """chunkset.rs:151-157; raises DecdsError(InvalidProofInChunk) before the unvalidated path's
        errors."""
        data = bytes(chunk.get_erasure_coded_data())
        proof = b"".join(chunk.get_proof())
        check(lib().decds_repairing_chunkset_add_chunk(self._h, chunk.get_chunkset_id(), chunk.get_global_chunk_id(),
                                                       data, len(data), proof, len(chunk.get_proof())))

    def add_chunk_unvalidated(self, chunk):
        """chunkset.rs:173-184; raises DecdsError(InvalidChunkMetadata | ChunksetReadyToRepair |
        ChunkDecodingFailed)."""
        data = bytes(chunk.get_erasure_coded_data())
        check(lib().decds_repairing_chunkset_add_chunk_unvalidated(self._h, chunk.get_chunkset_id(), data, len(data)))

    def is_ready_to_repair(self):
        return bool(lib().decds_repairing_chunkset_is_ready_to_repair(self._h))

    def repair(self):
        """chunkset.rs:200-208; raises DecdsError(ChunksetNotYetReadyToRepair | ChunksetRepairingFailed).
        Returns get_decoded_data's vector: the decoded pieces cut at the last boundary marker — the 10 MiB
        chunkset for validated chunks, shorter or up to 9 bytes longer for corrupted unvalidated ones."""
        cap = CHUNKSET_BYTES + K - 1  # DECDS_DECODED_MAX_BYTES
        out = ctypes.create_string_buffer(cap)
        n = ctypes.c_size_t()
        check(lib().decds_repairing_chunkset_repair(self._h, out, cap, ctypes.byref(n)))
        return out.raw[:n.value]

    def free(self):
        if self._h:
            lib().decds_repairing_chunkset_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


__all__ = ["Context", "Chunk", "ChunkSet", "RepairingChunkSet", "DecdsError"]

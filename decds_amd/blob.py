"""Python mirror of decds-lib's blob API over the C-ABI (decds-lib/src/blob.rs): Blob (new, header,
get_share) and RepairingBlob (new, add_chunk, is_chunkset_ready_to_repair,
is_chunkset_already_repaired, get_repaired_chunkset), with the reference's names and errors, plus
HostBuffer — page-locked host memory the library DMAs directly (decds_host_alloc)."""
import ctypes

import numpy as np

from ._capi import CHUNKSET_BYTES, CODED_PIECE_BYTES, N, check, lib
from .chunkset import Chunk
from .wire import BlobHeader


def _ctx_array(ctxs):
    ctxs = list(ctxs) if isinstance(ctxs, (list, tuple)) else [ctxs]
    arr = (ctypes.c_void_p * len(ctxs))(*[c.handle.value for c in ctxs])
    return arr, len(ctxs)


def _adopt_by(ctxs, obj):
    for c in (ctxs if isinstance(ctxs, (list, tuple)) else [ctxs]):
        if hasattr(c, "_adopt"):
            c._adopt(obj)


class _PinnedBlock:
    """owns one decds_host_alloc block; frees it when the last reference (a HostBuffer or any numpy
    view of its array) is gone, or on release()"""

    def __init__(self, p):
        self.p = p

    def release(self):
        if self.p:
            lib().decds_host_free(self.p)
            self.p = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


class HostBuffer:
    """Page-locked host bytes from decds_host_alloc, viewed as a numpy uint8 array (`.array`).

    Every numpy view of `.array` keeps the block alive (view -> array -> ctypes block -> owner), so the
    memory is released only when neither the HostBuffer nor any view remains. free() releases it early
    and returns True only when no view is alive; with views alive it refuses (returns False) and the
    block goes when the last view does."""

    def __init__(self, nbytes):
        p = ctypes.c_void_p()
        check(lib().decds_host_alloc(max(1, int(nbytes)), ctypes.byref(p)))
        self._block = _PinnedBlock(p)
        self.nbytes = int(nbytes)
        blk = (ctypes.c_uint8 * max(1, self.nbytes)).from_address(p.value)
        blk._owner = self._block
        self.array = np.frombuffer(blk, np.uint8, count=self.nbytes)

    def free(self):
        import sys
        if self.array is None:
            return True
        # references to the array: the attribute, getrefcount's argument; anything more is a view
        if sys.getrefcount(self.array) > 2:
            return False
        self.array = None
        self._block.release()
        return True


class Blob:
    """Blob (blob.rs:227-318): a blob erasure-coded into chunksets of 16 proof-carrying chunks."""

    def __init__(self, ctxs, data, coeffs=None):
        """Blob::new (blob.rs:244-285) on the device(s) of `ctxs` (one Context or a list: chunksets are
        sharded by contiguous index range). `coeffs` (n x 16 x 10 bytes) pins the coding vectors the
        reference draws from rand::rng()."""
        buf = np.ascontiguousarray(np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray)) else data,
                                   dtype=np.uint8).reshape(-1)
        arr, n_ctx = _ctx_array(ctxs)
        cv = None
        if coeffs is not None:
            cv = np.ascontiguousarray(coeffs, dtype=np.uint8).reshape(-1)
            if cv.size != -(-buf.size // CHUNKSET_BYTES) * N * 10:
                raise ValueError("coeffs must hold n*16*10 bytes")
        h = ctypes.c_void_p()
        check(lib().decds_blob_new(arr, n_ctx, ctypes.c_void_p(buf.ctypes.data if buf.size else 0), buf.size,
                                   None if cv is None else ctypes.c_void_p(cv.ctypes.data), ctypes.byref(h)))
        self._h = h
        self._ctxs = ctxs  # the contexts stay alive while this object uses them (close() still frees it first)
        _adopt_by(ctxs, self)

    def get_blob_header(self):
        """Blob::get_blob_header (blob.rs:288-290)"""
        bl, nc = ctypes.c_uint64(), ctypes.c_uint64()
        dg, rt = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
        rp = ctypes.c_void_p()
        check(lib().decds_blob_get_header(self._h, ctypes.byref(bl), ctypes.byref(nc), dg, rt, ctypes.byref(rp)))
        roots = ctypes.string_at(rp.value, 32 * nc.value)
        return BlobHeader(bl.value, nc.value, dg.raw, rt.raw, [roots[32 * k:32 * (k + 1)] for k in range(nc.value)])

    def proof_len(self):
        return lib().decds_blob_proof_len(self._h)

    def get_chunk(self, chunkset_id, share_id):
        """the proof-carrying chunk of (chunkset, share)"""
        d = ctypes.c_void_p()
        plen = self.proof_len()
        proof = ctypes.create_string_buffer(32 * plen)
        check(lib().decds_blob_get_chunk(self._h, chunkset_id, share_id, ctypes.byref(d), proof, len(proof)))
        return Chunk(chunkset_id, chunkset_id * N + share_id, ctypes.string_at(d.value, CODED_PIECE_BYTES),
                     [proof.raw[32 * k:32 * (k + 1)] for k in range(plen)])

    def get_share(self, share_id):
        """Blob::get_share (blob.rs:306-317): one chunk per chunkset"""
        n = self.get_blob_header().get_num_chunksets()
        plen = self.proof_len()
        data = np.empty((n, CODED_PIECE_BYTES), np.uint8)
        proofs = np.empty((n, plen * 32), np.uint8)
        check(lib().decds_blob_get_share(self._h, share_id, ctypes.c_void_p(data.ctypes.data), data.nbytes,
                                         ctypes.c_void_p(proofs.ctypes.data), proofs.nbytes))
        return [Chunk(c, c * N + share_id, data[c].tobytes(),
                      [proofs[c, 32 * k:32 * (k + 1)].tobytes() for k in range(plen)]) for c in range(n)]

    def free(self):
        """releases the Blob (its coded store goes to the library's page-locked block cache)"""
        if self._h:
            lib().decds_blob_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class RepairingBlob:
    """RepairingBlob (blob.rs:321-473)."""

    def __init__(self, ctxs, header, device_budget=None):
        """RepairingBlob::new(header) (blob.rs:341-353) on one Context or a list of them (chunksets
        sharded by contiguous index range, as Blob). device_budget: bytes of device memory per context
        for accepted rows and decoding; rows past it spill to page-locked host memory."""
        roots = b"".join(header.chunkset_root_commitments)
        arr, n_ctx = _ctx_array(ctxs)
        h = ctypes.c_void_p()
        check(lib().decds_repairing_blob_new_multi(arr, n_ctx, header.get_blob_size(), header.get_num_chunksets(),
                                                   header.get_root_commitment(), roots, ctypes.byref(h)))
        self._h = h
        self.header = header
        self._ctxs = ctxs  # the contexts stay alive while this object uses them (close() still frees it first)
        _adopt_by(ctxs, self)
        if device_budget is not None:
            check(lib().decds_repairing_blob_set_device_budget(h, int(device_budget)))

    def memory(self):
        """device bytes, chunksets with rows on the device / spilled to host, spill bytes, decode
        areas, contexts (decds_repairing_blob_memory)"""
        st = (ctypes.c_uint64 * 6)()
        check(lib().decds_repairing_blob_memory(self._h, st, 6))
        keys = ("device_bytes", "device_chunksets", "spilled_chunksets", "spill_bytes", "decode_areas", "contexts")
        return dict(zip(keys, [int(v) for v in st]))

    def add_chunk(self, chunk):
        """RepairingBlob::add_chunk (blob.rs:373-394): raises DecdsError(InvalidChunksetId |
        ChunksetAlreadyRepaired | InvalidProofInChunk | ChunksetReadyToRepair | ChunkDecodingFailed)"""
        data = bytes(chunk.get_erasure_coded_data())
        proof = b"".join(chunk.get_proof())
        check(lib().decds_repairing_blob_add_chunk(self._h, chunk.get_chunkset_id(), chunk.get_global_chunk_id(), data,
                                                   len(data), proof, len(chunk.get_proof())))

    def add_chunks(self, chunks):
        """add_chunk for every chunk in order, validated as one device batch; returns the per-chunk
        status codes (0 = accepted) that sequential add_chunk calls would have produced. All chunks
        carry full-length data and proofs of one length."""
        m = len(chunks)
        if m == 0:
            return np.zeros(0, np.int32)
        plen = len(chunks[0].get_proof())
        rows = np.empty((m, CODED_PIECE_BYTES), np.uint8)
        ids = np.empty((m, 2), np.uint64)
        proofs = np.empty((m, plen * 32), np.uint8)
        for i, c in enumerate(chunks):
            d = c.get_erasure_coded_data()
            if len(d) != CODED_PIECE_BYTES or len(c.get_proof()) != plen:
                raise ValueError("add_chunks needs full-length chunks with proofs of one length")
            rows[i] = np.frombuffer(d, np.uint8)
            ids[i] = (c.get_chunkset_id(), c.get_global_chunk_id())
            proofs[i] = np.frombuffer(b"".join(c.get_proof()), np.uint8)
        return self.add_rows(rows, ids, proofs, plen)

    def add_rows(self, rows, ids, proofs, proof_len):
        """decds_repairing_blob_add_chunks on arrays: rows (m, F) uint8, ids (m, 2) uint64, proofs (m, proof_len*32)"""
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        rows = np.ascontiguousarray(rows, dtype=np.uint8)
        proofs = np.ascontiguousarray(proofs, dtype=np.uint8)
        m = ids.shape[0] if ids.ndim == 2 else -1
        if ids.shape != (m, 2) or rows.shape != (m, CODED_PIECE_BYTES) or proofs.shape != (m, proof_len * 32):
            raise ValueError("add_rows needs rows (m, %d), ids (m, 2), proofs (m, %d); got %s, %s, %s"
                             % (CODED_PIECE_BYTES, proof_len * 32, rows.shape, ids.shape, proofs.shape))
        status = np.empty(m, np.int32)
        vp = ctypes.c_void_p
        check(lib().decds_repairing_blob_add_chunks(self._h, m, vp(ids.ctypes.data), vp(rows.ctypes.data),
                                                    vp(proofs.ctypes.data), proof_len, vp(status.ctypes.data)))
        return status

    def is_chunkset_ready_to_repair(self, chunkset_id):
        o = ctypes.c_int()
        check(lib().decds_repairing_blob_is_chunkset_ready_to_repair(self._h, chunkset_id, ctypes.byref(o)))
        return bool(o.value)

    def is_chunkset_already_repaired(self, chunkset_id):
        o = ctypes.c_int()
        check(lib().decds_repairing_blob_is_chunkset_already_repaired(self._h, chunkset_id, ctypes.byref(o)))
        return bool(o.value)

    def get_repaired_chunkset(self, chunkset_id, out=None):
        """RepairingBlob::get_repaired_chunkset (blob.rs:451-473): the chunkset's bytes, truncated to its
        real size; `out` may be a writable uint8 array of >= 10 MiB (e.g. a HostBuffer's array)."""
        buf = out if out is not None else np.empty(CHUNKSET_BYTES, np.uint8)
        got = ctypes.c_size_t()
        check(lib().decds_repairing_blob_get_repaired_chunkset(self._h, chunkset_id, ctypes.c_void_p(buf.ctypes.data),
                                                               buf.nbytes, ctypes.byref(got)))
        return buf[:got.value].tobytes() if out is None else buf[:got.value]

    def free(self):
        """releases the RepairingBlob (device slots, spill memory, streams)"""
        if self._h:
            lib().decds_repairing_blob_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


__all__ = ["Blob", "RepairingBlob", "HostBuffer", "BlobHeader"]

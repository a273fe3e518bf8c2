"""Batch codec over device-resident chunksets (torch CUDA tensors as HBM plumbing).

encode_batch / repair_plan_batch / decode_batch are thin wrappers of the C-ABI *_batch entry
points: they pass raw device pointers and the caller's HIP stream, so the kernels run on the
stream the caller times with events. blob_encode_host / blob_repair_host mirror Blob::new's
chunkset loop (blob.rs:244-264) and RepairingBlob's repair driver (blob.rs:373-473) over host
buffers with overlapped pinned copies.
"""
import ctypes

import numpy as np

from ._capi import (CHUNKSET_BYTES, CODED_PIECE_BYTES, CODED_PITCH_ALIGNED, CODED_ROW_OFFSET_ALIGNED, K, N,
                    NO_CANDIDATE, REPAIR_PLAN_BYTES, check, lib)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def _stream(stream):
    if stream is None:
        import torch
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)


def _need(t, nbytes, what):
    if not t.is_cuda:
        raise TypeError("%s must be a CUDA tensor (device-resident batch API)" % what)
    if not t.is_contiguous():
        raise ValueError("%s must be contiguous" % what)
    if t.numel() * t.element_size() < nbytes:
        raise ValueError("%s too small: %d < %d bytes" % (what, t.numel() * t.element_size(), nbytes))


def coded_buffer(n, aligned=True, device="cuda"):
    """device buffer for n chunksets' coded rows -> (rows view, pitch). aligned: the recommended layout
    (pitch 1,048,704, payloads 128-byte aligned: line-aligned encoder stores); else rows packed at F."""
    import torch
    if not aligned:
        return torch.empty(n * N * CODED_PIECE_BYTES, dtype=torch.uint8, device=device), CODED_PIECE_BYTES
    buf = torch.empty(n * N * CODED_PITCH_ALIGNED + 256, dtype=torch.uint8, device=device)
    off = (CODED_ROW_OFFSET_ALIGNED - buf.data_ptr()) % 128
    return buf[off:off + (n * N - 1) * CODED_PITCH_ALIGNED + CODED_PIECE_BYTES], CODED_PITCH_ALIGNED


def encode_batch(ctx, src, n, coeffs, dst, pitch=CODED_PIECE_BYTES, stream=None):
    """chunkset.rs:43-52 for n chunksets: src n*CS bytes, coeffs n*16*10, dst n*16 rows of `pitch`."""
    _need(src, n * CHUNKSET_BYTES, "src")
    _need(coeffs, n * N * K, "coeffs")
    _need(dst, (n * N - 1) * pitch + CODED_PIECE_BYTES, "dst")
    check(lib().decds_encode_batch(ctx.handle, _ptr(src), n, _ptr(coeffs), _ptr(dst), pitch, _stream(stream)))


def repair_plan_batch(ctx, coded, n, cand, plan, verdicts, status, pitch=CODED_PIECE_BYTES, stream=None):
    _need(coded, (n * N - 1) * pitch + CODED_PIECE_BYTES, "coded")
    _need(cand, n * N, "cand")
    _need(plan, n * REPAIR_PLAN_BYTES, "plan")
    _need(verdicts, n * N, "verdicts")
    _need(status, n * 4, "status")
    check(lib().decds_repair_plan_batch(ctx.handle, _ptr(coded), pitch, n, _ptr(cand), _ptr(plan),
                                        _ptr(verdicts), _ptr(status), _stream(stream)))


REPAIR_INFO_BYTES = 16  # decds_repair_info: u32 decoded_len, 10 tail bytes, 2 reserved


def decode_batch(ctx, coded, n, plan, dst, status, pitch=CODED_PIECE_BYTES, stream=None, info=None):
    """chunkset.rs:200-208 for n chunksets. info (optional, n*16 bytes, 4-byte aligned device tensor):
    per chunkset rlnc get_decoded_data's length (cut at the last boundary marker) and the 10 decoded
    tail bytes past the chunkset; read it with repair_info()."""
    _need(coded, (n * N - 1) * pitch + CODED_PIECE_BYTES, "coded")
    _need(plan, n * REPAIR_PLAN_BYTES, "plan")
    _need(dst, n * CHUNKSET_BYTES, "dst")
    _need(status, n * 4, "status")
    if info is not None:
        _need(info, n * REPAIR_INFO_BYTES, "info")
    check(lib().decds_decode_batch(ctx.handle, _ptr(coded), pitch, n, _ptr(plan), _ptr(dst), _ptr(status),
                                   None if info is None else _ptr(info), _stream(stream)))


def repair_batch(ctx, coded, n, cand, plan, verdicts, dst, status, pitch=CODED_PIECE_BYTES, stream=None, info=None):
    """decds_repair_batch: repair_plan_batch + decode_batch in one call — up to DECDS_PLAN_DECODE_MAX_N
    chunksets (default 2) one kernel launch (rlnc_plan_decode_kernel), the same outputs either way"""
    _need(coded, (n * N - 1) * pitch + CODED_PIECE_BYTES, "coded")
    _need(cand, n * N, "cand")
    _need(plan, n * REPAIR_PLAN_BYTES, "plan")
    _need(verdicts, n * N, "verdicts")
    _need(dst, n * CHUNKSET_BYTES, "dst")
    _need(status, n * 4, "status")
    if info is not None:
        _need(info, n * REPAIR_INFO_BYTES, "info")
    check(lib().decds_repair_batch(ctx.handle, _ptr(coded), pitch, n, _ptr(cand), _ptr(plan),
                                   _ptr(verdicts), _ptr(dst), _ptr(status), None if info is None else _ptr(info),
                                   _stream(stream)))


def repair_info(info, n):
    """(decoded_len int64[n], tail uint8[n, 10]) from an info tensor/array filled by decode_batch"""
    a = np.ascontiguousarray(info.cpu().numpy() if hasattr(info, "cpu") else info).view(np.uint8)[:n * REPAIR_INFO_BYTES]
    a = a.reshape(n, REPAIR_INFO_BYTES)
    return a[:, :4].copy().view("<u4").reshape(n).astype(np.int64), a[:, 4:14].copy()


def decoded_bytes(dst_chunkset, decoded_len, tail):
    """get_decoded_data's vector of one chunkset from its CS bytes in dst and its repair info"""
    from ._capi import CHUNKSET_BYTES as CS
    d = dst_chunkset.cpu().numpy() if hasattr(dst_chunkset, "cpu") else np.asarray(dst_chunkset)
    if decoded_len <= CS:
        return d[:decoded_len].tobytes()
    return d[:CS].tobytes() + bytes(tail[:decoded_len - CS])


def commit_batch(ctx, coded, n, digests, roots, proofs, first_chunkset_id=0, pitch=CODED_PIECE_BYTES, stream=None):
    """ChunkSet::new's commitment (chunkset.rs:54-63) for n device-resident chunksets: per coded row
    the BLAKE3 chunk digest (chunk.rs:40-46), per chunkset the 16-leaf Merkle root and proofs."""
    _need(coded, (n * N - 1) * pitch + CODED_PIECE_BYTES, "coded")
    _need(digests, n * N * 32, "digests")
    _need(roots, n * 32, "roots")
    _need(proofs, n * N * 4 * 32, "proofs")
    check(lib().decds_commit_batch(ctx.handle, _ptr(coded), pitch, n, first_chunkset_id, _ptr(digests), _ptr(roots),
                                   _ptr(proofs), _stream(stream)))


def encode_commit_workspace(n, device="cuda"):
    import torch
    return torch.empty(max(1, lib().decds_encode_commit_workspace_bytes(n)), dtype=torch.uint8, device=device)


def encode_commit_batch(ctx, src, n, coeffs, dst, digests, roots, proofs, first_chunkset_id=0,
                        pitch=CODED_PIECE_BYTES, workspace=None, stream=None):
    """ChunkSet::new for n device-resident chunksets (chunkset.rs:37-63): encode_batch + commit_batch
    in one call; on 16-byte-aligned rows (coded_buffer(aligned=True)) the chunk hashing is fused into
    the encode kernel. workspace: encode_commit_workspace(n) (allocated here when None)."""
    _need(src, n * CHUNKSET_BYTES, "src")
    _need(coeffs, n * N * K, "coeffs")
    _need(dst, (n * N - 1) * pitch + CODED_PIECE_BYTES, "dst")
    _need(digests, n * N * 32, "digests")
    _need(roots, n * 32, "roots")
    _need(proofs, n * N * 4 * 32, "proofs")
    if workspace is None:
        workspace = encode_commit_workspace(n, device=dst.device)
    _need(workspace, lib().decds_encode_commit_workspace_bytes(n), "workspace")
    check(lib().decds_encode_commit_batch(ctx.handle, _ptr(src), n, _ptr(coeffs), _ptr(dst), pitch, first_chunkset_id,
                                          _ptr(digests), _ptr(roots), _ptr(proofs), _ptr(workspace), _stream(stream)))


def validate_batch(ctx, coded, n_rows, ids, proofs, proof_len, chunkset_roots, num_chunksets, digests, valid,
                   blob_root=None, pitch=CODED_PIECE_BYTES, stream=None):
    """BlobHeader::validate_chunk (blob.rs:211-215) for n_rows received device-resident rows.
    ids: int64/uint64 tensor (n_rows, 2) = (chunkset_id, global chunk_id); proofs: n_rows x proof_len
    x 32 bytes; chunkset_roots: num_chunksets x 32; blob_root: 32-byte device tensor or None."""
    _need(coded, (n_rows - 1) * pitch + CODED_PIECE_BYTES if n_rows else 0, "coded")
    _need(ids, n_rows * 16, "ids")
    _need(proofs, n_rows * proof_len * 32, "proofs")
    _need(chunkset_roots, num_chunksets * 32, "chunkset_roots")
    _need(digests, n_rows * 32, "digests")
    _need(valid, n_rows, "valid")
    check(lib().decds_validate_batch(ctx.handle, _ptr(coded), pitch, n_rows, _ptr(ids), _ptr(proofs), proof_len,
                                     _ptr(chunkset_roots), num_chunksets,
                                     None if blob_root is None else _ptr(blob_root), _ptr(digests), _ptr(valid),
                                     _stream(stream)))


def fill_random_device(ctx, seed, dst, nbytes=None, byte_offset=0, stream=None):
    nbytes = dst.numel() * dst.element_size() if nbytes is None else nbytes
    check(lib().decds_fill_random_device(ctx.handle, seed, byte_offset, _ptr(dst), nbytes, _stream(stream)))


def fill_random_host(seed, nbytes, byte_offset=0):
    out = np.empty(nbytes, dtype=np.uint8)
    lib().decds_fill_random_host(seed, byte_offset, out.ctypes.data_as(ctypes.c_void_p), nbytes)
    return out


def blob_encode_host(ctx, blob, coeffs, batch=16, out=None):
    """Blob::new's chunkset loop (blob.rs:252-264) on host buffers. Returns (n*16, F) uint8."""
    blob = np.ascontiguousarray(np.frombuffer(blob, dtype=np.uint8) if isinstance(blob, (bytes, bytearray)) else blob)
    n = -(-blob.size // CHUNKSET_BYTES)
    coeffs = np.ascontiguousarray(coeffs, dtype=np.uint8)
    if coeffs.size != n * N * K:
        raise ValueError("coeffs must hold n*16*10 bytes")
    if out is None:
        out = np.empty((n * N, CODED_PIECE_BYTES), dtype=np.uint8)
    vp = ctypes.c_void_p
    check(lib().decds_blob_encode_host(ctx.handle, vp(blob.ctypes.data), blob.size, vp(coeffs.ctypes.data),
                                       vp(out.ctypes.data), batch))
    return out


def blob_repair_host(ctx, coded, cand, blob_len, batch=16, out=None):
    """RepairingBlob add_chunk/get_repaired_chunkset (blob.rs:373-473). Returns (blob, status)."""
    coded = np.ascontiguousarray(coded, dtype=np.uint8)
    n = coded.shape[0] // N
    cand = np.ascontiguousarray(cand, dtype=np.uint8).reshape(n, N)
    if out is None:
        out = np.empty(blob_len, dtype=np.uint8)
    status = np.empty(n, dtype=np.int32)
    vp = ctypes.c_void_p
    check(lib().decds_blob_repair_host(ctx.handle, vp(coded.ctypes.data), n, vp(cand.ctypes.data), blob_len,
                                       vp(out.ctypes.data), vp(status.ctypes.data), batch))
    return out, status


def _ctxs(ctxs):
    arr = (ctypes.c_void_p * len(ctxs))(*[c.handle.value for c in ctxs])
    return arr, len(ctxs)


def blob_encode_host_multi(ctxs, blob, coeffs, batch=16, out=None):
    """blob_encode_host sharded over several contexts (devices) by contiguous chunkset range."""
    blob = np.ascontiguousarray(np.frombuffer(blob, dtype=np.uint8) if isinstance(blob, (bytes, bytearray)) else blob)
    n = -(-blob.size // CHUNKSET_BYTES)
    coeffs = np.ascontiguousarray(coeffs, dtype=np.uint8)
    if out is None:
        out = np.empty((n * N, CODED_PIECE_BYTES), dtype=np.uint8)
    arr, k = _ctxs(ctxs)
    vp = ctypes.c_void_p
    check(lib().decds_blob_encode_host_multi(arr, k, vp(blob.ctypes.data), blob.size, vp(coeffs.ctypes.data),
                                             vp(out.ctypes.data), batch))
    return out


def blob_repair_host_multi(ctxs, coded, cand, blob_len, batch=16, out=None):
    """blob_repair_host sharded over several contexts (devices) by contiguous chunkset range."""
    coded = np.ascontiguousarray(coded, dtype=np.uint8)
    n = coded.shape[0] // N
    cand = np.ascontiguousarray(cand, dtype=np.uint8).reshape(n, N)
    if out is None:
        out = np.empty(blob_len, dtype=np.uint8)
    status = np.empty(n, dtype=np.int32)
    arr, k = _ctxs(ctxs)
    vp = ctypes.c_void_p
    check(lib().decds_blob_repair_host_multi(arr, k, vp(coded.ctypes.data), n, vp(cand.ctypes.data), blob_len,
                                             vp(out.ctypes.data), vp(status.ctypes.data), batch))
    return out, status


def host_register(arr):
    """page-lock a numpy buffer for repeated host-path calls (decds_host_register)"""
    check(lib().decds_host_register(ctypes.c_void_p(arr.ctypes.data), arr.nbytes))


def host_unregister(arr):
    check(lib().decds_host_unregister(ctypes.c_void_p(arr.ctypes.data)))


__all__ = ["coded_buffer", "commit_batch", "encode_batch", "repair_plan_batch", "decode_batch", "repair_batch", "repair_info",
           "decoded_bytes", "REPAIR_INFO_BYTES", "fill_random_device",
           "fill_random_host", "blob_encode_host", "blob_repair_host", "blob_encode_host_multi",
           "blob_repair_host_multi", "host_register", "host_unregister",
           "NO_CANDIDATE"]

"""decds-bin's file flow over the device path: `break` a blob file into
`metadata.commit` + `chunkset.N/shareXX.data` (handle_break.rs:5-106) and `repair` it back
(handle_repair.rs:5-155), with the same layout, wire format (decds_amd/wire.py) and error
handling, but Blob::new / RepairingBlob run as device batches:

  break : whole-blob BLAKE3 (host, tree-parallel) | per batch of chunksets: H2D, encode,
          commitment (digests, chunkset roots, proofs) on the GPU, D2H | blob-level Merkle tree
          over the chunkset roots (host, blob.rs:266-273) | serialise + write the share files
  repair: read + parse share files | per batch: H2D, validate every row (decds_validate_batch =
          BlobHeader::validate_chunk), plan over the valid rows in share order, decode, D2H |
          write chunkset.N.data and repaired.data, check the repaired blob's BLAKE3 digest

The reference reads shares 0..15 per chunkset and stops once the chunkset is ready; invalid,
unparsable and undecodable chunks are skipped (handle_repair.rs:57-76). Here every present share
is read and validated, and the plan replays the same arrival order, so the accepted chunks are
the ones the reference would accept.
"""
import ctypes
import os
import time

import numpy as np

from . import codec, wire
from ._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N, NO_CANDIDATE, DecdsError, check, lib

PROOF_SIZE = 4


def _blake3(buf, threads=16):
    out = ctypes.create_string_buffer(32)
    b = np.ascontiguousarray(buf)
    lib().decds_blake3_parallel(b.ctypes.data_as(ctypes.c_void_p), b.size, out, threads)
    return out.raw


def _merkle(leaves):
    n = len(leaves)
    depth = max(0, (n - 1).bit_length())
    lv = np.frombuffer(b"".join(leaves), np.uint8).copy()
    root = ctypes.create_string_buffer(32)
    proofs = np.empty(max(1, n * depth * 32), np.uint8)
    d = lib().decds_merkle_tree(lv.ctypes.data_as(ctypes.c_void_p), n, root, proofs.ctypes.data_as(ctypes.c_void_p))
    if d < 0:
        check(d)
    return root.raw, proofs[:n * depth * 32].reshape(n, depth * 32) if depth else np.zeros((n, 0), np.uint8)


def break_blob(ctx, blob, target_dir, batch=64, coeffs=None, timings=None):
    """Blob::new + handle_break: `blob` is a path or a uint8 array. coeffs: n x 16 x 10 coding vectors
    or None (drawn from os.urandom, as the reference draws from rand::rng()). Returns the header."""
    import torch
    t = {} if timings is None else timings
    t0 = time.perf_counter()
    data = np.fromfile(blob, dtype=np.uint8) if isinstance(blob, (str, os.PathLike)) else np.ascontiguousarray(blob)
    if data.size == 0:
        raise DecdsError(8, "empty data for blob")
    t["read_s"] = time.perf_counter() - t0
    n = -(-data.size // CS)
    if coeffs is None:
        coeffs = np.frombuffer(os.urandom(n * N * K), np.uint8)
    coeffs = np.ascontiguousarray(coeffs, dtype=np.uint8).reshape(-1)
    t0 = time.perf_counter()
    digest = _blake3(data)                                             # blob.rs:249
    t["digest_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    dev = torch.device("cuda", ctx.device)
    coded_h = np.empty((n * N, F), np.uint8)
    roots_h = np.empty((n, 32), np.uint8)
    proofs_h = np.empty((n * N, PROOF_SIZE * 32), np.uint8)
    bmax = min(batch, n)
    src = torch.empty(bmax * CS, dtype=torch.uint8, device=dev)
    coded = torch.empty(bmax * N * F, dtype=torch.uint8, device=dev)
    dig = torch.empty(bmax * N * 32, dtype=torch.uint8, device=dev)
    roots = torch.empty(bmax * 32, dtype=torch.uint8, device=dev)
    proofs = torch.empty(bmax * N * 128, dtype=torch.uint8, device=dev)
    for c0 in range(0, n, bmax):
        b = min(bmax, n - c0)
        lo, hi = c0 * CS, min(data.size, (c0 + b) * CS)
        src[:hi - lo].copy_(torch.from_numpy(data[lo:hi]))
        if hi - lo < b * CS:
            src[hi - lo:b * CS].zero_()                               # blob.rs:252-254 zero padding
        cv = torch.from_numpy(coeffs[c0 * N * K:(c0 + b) * N * K].copy()).to(dev)
        codec.encode_batch(ctx, src, b, cv, coded)
        codec.commit_batch(ctx, coded, b, dig, roots, proofs, first_chunkset_id=c0)
        coded_h[c0 * N:(c0 + b) * N] = coded[:b * N * F].view(b * N, F).cpu().numpy()
        roots_h[c0:c0 + b] = roots[:b * 32].view(b, 32).cpu().numpy()
        proofs_h[c0 * N:(c0 + b) * N] = proofs[:b * N * 128].view(b * N, 128).cpu().numpy()
    torch.cuda.synchronize()
    t["device_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    cs_roots = [roots_h[c].tobytes() for c in range(n)]
    blob_root, blob_proofs = _merkle(cs_roots)                         # blob.rs:266-273
    header = wire.BlobHeader(data.size, n, digest, blob_root, cs_roots)
    os.makedirs(target_dir, exist_ok=True)
    with open(os.path.join(target_dir, "metadata.commit"), "wb") as f:  # handle_break.rs:49-64
        f.write(header.to_bytes())
    depth = blob_proofs.shape[1] // 32
    plen = PROOF_SIZE + depth
    cap = lib().decds_pcc_encoded_len(n, n * N, F, plen)
    out = ctypes.create_string_buffer(cap)
    w = ctypes.c_size_t()
    pf = np.empty(plen * 32, np.uint8)
    for c in range(n):                                                 # handle_break.rs:66-106
        d = os.path.join(target_dir, "chunkset.%d" % c)
        os.makedirs(d, exist_ok=True)
        pf[PROOF_SIZE * 32:] = blob_proofs[c]
        for j in range(N):
            r = c * N + j
            pf[:PROOF_SIZE * 32] = proofs_h[r]
            check(lib().decds_pcc_to_bytes(c, r, coded_h[r].ctypes.data_as(ctypes.c_void_p), F,
                                           pf.ctypes.data_as(ctypes.c_void_p), plen, out, cap, ctypes.byref(w)))
            with open(os.path.join(d, "share%02d.data" % j), "wb") as f:
                f.write(memoryview(out)[:w.value])
    t["write_s"] = time.perf_counter() - t0
    return header


def read_blob_metadata(chunk_dir):
    """decds-bin utils.rs:20-44: the file must hold exactly one header."""
    b = open(os.path.join(chunk_dir, "metadata.commit"), "rb").read()
    h, used = wire.BlobHeader.from_bytes(b)
    if used != len(b):
        raise DecdsError(13, "erasure-coded blob metadata file is %d bytes longer than it should be" % (len(b) - used))
    return h


def repair_blob(ctx, chunk_dir, target_dir, batch=64, timings=None):
    """handle_repair over device batches. Returns the repaired bytes' path; raises DecdsError if a
    chunkset cannot be repaired or the repaired digest differs (handle_repair.rs:79-84, 129-151)."""
    import torch
    t = {} if timings is None else timings
    header = read_blob_metadata(chunk_dir)
    n = header.get_num_chunksets()
    dev = torch.device("cuda", ctx.device)
    roots_d = torch.from_numpy(np.frombuffer(b"".join(header.chunkset_root_commitments), np.uint8).copy()).to(dev)
    broot_d = torch.from_numpy(np.frombuffer(header.root_commitment, np.uint8).copy()).to(dev)
    os.makedirs(target_dir, exist_ok=True)
    out_path = os.path.join(target_dir, "repaired.data")
    repaired = np.empty(n * CS, np.uint8)
    t_read = t_dev = 0.0
    bmax = min(batch, n)
    for c0 in range(0, n, bmax):
        b = min(bmax, n - c0)
        t0 = time.perf_counter()
        rows, ids, prf, owner = [], [], [], []                          # owner: (chunkset slot, share id)
        plen = None
        for c in range(c0, c0 + b):
            for j in range(N):
                p = os.path.join(chunk_dir, "chunkset.%d" % c, "share%02d.data" % j)
                if not os.path.isfile(p):
                    continue
                raw = open(p, "rb").read()
                try:
                    ch, used = wire.pcc_from_bytes(raw)
                except DecdsError:
                    continue                                           # unreadable share: skipped
                if used != len(raw) or len(ch.erasure_coded_data) != F:
                    continue
                if plen is None:
                    plen = len(ch.proof)
                if len(ch.proof) != plen:
                    continue
                rows.append(ch.erasure_coded_data)
                ids.append((ch.chunkset_id, ch.chunk_id))
                prf.append(b"".join(ch.proof))
                owner.append((c - c0, j))
        t_read += time.perf_counter() - t0
        t0 = time.perf_counter()
        m = len(rows)
        cand = np.full((b, N), NO_CANDIDATE, np.uint8)
        if m:
            rows_d = torch.from_numpy(np.frombuffer(b"".join(rows), np.uint8).copy()).to(dev)
            ids_d = torch.tensor(ids, dtype=torch.int64, device=dev)
            prf_d = torch.from_numpy(np.frombuffer(b"".join(prf), np.uint8).copy()).to(dev)
            dig = torch.empty(m * 32, dtype=torch.uint8, device=dev)
            valid = torch.empty(m, dtype=torch.uint8, device=dev)
            codec.validate_batch(ctx, rows_d, m, ids_d, prf_d, plen, roots_d, n, dig, valid, blob_root=broot_d)
            v = valid.cpu().numpy()
            # RepairingBlob::add_chunk routes by the chunk's own chunkset id (blob.rs:374-379): a valid
            # chunk in another chunkset's directory belongs to that chunkset, which the reference
            # would repair from it only if it were read there; keep it only in its own directory
            fill = [0] * b
            coded = torch.empty(b * N * F, dtype=torch.uint8, device=dev)
            for k in range(m):
                s, j = owner[k]
                if v[k] and ids[k][0] == c0 + s and fill[s] < N:
                    coded[(s * N + fill[s]) * F:(s * N + fill[s] + 1) * F].copy_(rows_d[k * F:(k + 1) * F])
                    cand[s, fill[s]] = fill[s]
                    fill[s] += 1
        else:
            coded = torch.empty(b * N * F, dtype=torch.uint8, device=dev)
        plan = torch.empty(b * 128, dtype=torch.uint8, device=dev)
        verd = torch.empty(b * N, dtype=torch.int8, device=dev)
        status = torch.empty(b, dtype=torch.int32, device=dev)
        dst = torch.empty(b * CS, dtype=torch.uint8, device=dev)
        codec.repair_batch(ctx, coded, b, torch.from_numpy(cand).to(dev), plan, verd, dst, status)
        st = status.cpu().numpy()
        bad = [c0 + s for s in range(b) if st[s] != 0]
        if bad:
            raise DecdsError(6 if any(st[s] == 6 for s in range(b)) else 5,
                             "failed to repair chunkset(s) %s" % bad[:8])
        repaired[c0 * CS:(c0 + b) * CS] = dst.cpu().numpy()
        t_dev += time.perf_counter() - t0
    t0 = time.perf_counter()
    blob = repaired[:header.get_blob_size()]
    for c in range(n):                                                  # handle_repair.rs:86-96
        lo, hi = c * CS, min(header.get_blob_size(), (c + 1) * CS)
        blob[lo:hi].tofile(os.path.join(target_dir, "chunkset.%d.data" % c))
    blob.tofile(out_path)
    t["write_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    ok = _blake3(blob) == header.get_blob_digest()                      # handle_repair.rs:129-151
    t["digest_s"] = time.perf_counter() - t0
    t["read_s"], t["device_s"] = t_read, t_dev
    if not ok:
        raise DecdsError(6, "repaired blob digest does not match the header")
    return out_path

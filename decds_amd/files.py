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
the ones the reference would accept. A share whose chunk claims ANOTHER chunkset's id is routed by
the reference to that chunkset (blob.rs:374-379) — or ends the repair, when that chunkset is already
repaired or out of range — so when the batched pass meets one, the repair is redone by the
reference's own sequential loop over the incremental RepairingBlob (repair_blob_sequential).
"""
import ctypes
import os
import time
from concurrent.futures import ThreadPoolExecutor

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


def _pinned(shape, torch):
    return torch.empty(shape, dtype=torch.uint8, pin_memory=True)


def _map(path):
    """a read-only view of a file's pages, prefaulted in one pass (MAP_POPULATE) instead of one fault
    per page while it is hashed or copied"""
    import mmap
    with open(path, "rb") as f:
        size = os.fstat(f.fileno()).st_size
        mm = mmap.mmap(f.fileno(), size, flags=mmap.MAP_SHARED | getattr(mmap, "MAP_POPULATE", 0), prot=mmap.PROT_READ)
    return np.frombuffer(mm, np.uint8)


def break_blob(ctx, blob, target_dir, batch=16, coeffs=None, timings=None, threads=16, device_store=None):
    """Blob::new + handle_break: `blob` is a path or a uint8 array. coeffs: n x 16 x 10 coding vectors
    or None (drawn from os.urandom, as the reference draws from rand::rng()). Returns the header.

    Pipelined over two page-locked slots per direction (no page-locked copy of the whole blob):
      1. the blob file is memory-mapped; batch k is copied into input slot k % 2 (once that slot's
         previous H2D copy is done) and queued — H2D, encode, commitment — on one stream, so the
         device works on batch k while batch k + 1 is copied in; the whole-blob digest (blob.rs:249)
         runs on a helper thread over the mapping meanwhile;
      2. the coded rows stay in HBM (device_store, default: when they fit in half the free device
         memory; else they go to one page-locked host store) until the blob-level tree over the
         chunkset roots (blob.rs:266-273) gives every chunk its proof;
      3. batch k's rows come back into output slot k % 2 while `threads` workers serialise and write
         batch k - 1's share files (handle_break.rs:66-106, one chunkset per task)."""
    import threading
    import torch
    t = {} if timings is None else timings
    t_start = time.perf_counter()
    from_file = isinstance(blob, (str, os.PathLike))
    size = os.path.getsize(blob) if from_file else np.asarray(blob).size
    if size == 0:
        raise DecdsError(8, "empty data for blob")
    data = _map(blob) if from_file else np.ascontiguousarray(blob).reshape(-1)
    n = -(-size // CS)
    if coeffs is None:
        coeffs = np.frombuffer(os.urandom(n * N * K), np.uint8)
    coeffs = np.ascontiguousarray(coeffs, dtype=np.uint8).reshape(-1)
    dev = torch.device("cuda", ctx.device)
    bmax = min(batch, n)
    if device_store is None:
        device_store = n * N * F <= torch.cuda.mem_get_info(dev)[0] // 2
    digest = [None]

    def whole_digest():
        t0 = time.perf_counter()
        digest[0] = _blake3(data, threads)                              # blob.rs:249
        t["digest_s"] = time.perf_counter() - t0

    dth = threading.Thread(target=whole_digest)
    dth.start()
    stream = torch.cuda.Stream(dev)
    pool = ThreadPoolExecutor(max_workers=max(1, threads))
    try:
        t0 = time.perf_counter()
        slots_in = [_pinned(bmax * CS, torch) for _ in range(2)]
        in_free = [None, None]                                         # event: the slot's H2D is done
        with torch.cuda.stream(stream):
            cv = torch.from_numpy(coeffs).to(dev, non_blocking=False)
            src = torch.empty(bmax * CS, dtype=torch.uint8, device=dev)
            store = torch.empty(n * N * F if device_store else bmax * N * F, dtype=torch.uint8, device=dev)
            dig = torch.empty(bmax * N * 32, dtype=torch.uint8, device=dev)
            roots_d = torch.empty(n * 32, dtype=torch.uint8, device=dev)
            proofs_d = torch.empty(n * N * 128, dtype=torch.uint8, device=dev)
        host_store = None if device_store else _pinned((n * N, F), torch)
        t["alloc_s"] = time.perf_counter() - t0

        def copy_in(dst, lo, hi):                                      # a batch's bytes into a slot, 4 threads
            q = -(-(hi - lo) // 4)
            list(pool.map(lambda i: np.copyto(dst[i * q:min(hi - lo, (i + 1) * q)],
                                              data[lo + i * q:lo + min(hi - lo, (i + 1) * q)]), range(4)))

        t0 = time.perf_counter()
        for k, c0 in enumerate(range(0, n, bmax)):                     # 1. in, encode, commit
            b = min(bmax, n - c0)
            lo, hi = c0 * CS, min(size, (c0 + b) * CS)
            sl = k % 2
            if in_free[sl] is not None:
                in_free[sl].synchronize()
            copy_in(slots_in[sl].numpy(), lo, hi)
            with torch.cuda.stream(stream):
                src[:hi - lo].copy_(slots_in[sl][:hi - lo], non_blocking=True)
                in_free[sl] = torch.cuda.Event()
                in_free[sl].record(stream)
                if hi - lo < b * CS:
                    src[hi - lo:b * CS].zero_()                       # blob.rs:252-254 zero padding
                coded = store[c0 * N * F:] if device_store else store
                codec.encode_batch(ctx, src, b, cv[c0 * N * K:], coded, stream=stream)
                codec.commit_batch(ctx, coded, b, dig, roots_d[c0 * 32:], proofs_d[c0 * N * 128:], first_chunkset_id=c0,
                                   stream=stream)
                if not device_store:
                    host_store[c0 * N:(c0 + b) * N].view(-1).copy_(coded[:b * N * F], non_blocking=True)
        stream.synchronize()                                           # (.cpu() below runs on the default stream)
        roots_np = roots_d.cpu().numpy()
        proofs_np = proofs_d.cpu().numpy().reshape(n * N, PROOF_SIZE * 32)
        t["in_device_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        cs_roots = [roots_np[c * 32:(c + 1) * 32].tobytes() for c in range(n)]
        blob_root, blob_proofs = _merkle(cs_roots)                     # blob.rs:266-273
        os.makedirs(target_dir, exist_ok=True)
        depth = blob_proofs.shape[1] // 32
        plen = PROOF_SIZE + depth
        cap = lib().decds_pcc_encoded_len(n, n * N, F, plen)

        def write_chunkset(c, rows):                                   # handle_break.rs:66-106
            d = os.path.join(target_dir, "chunkset.%d" % c)
            os.makedirs(d, exist_ok=True)
            out = ctypes.create_string_buffer(cap)
            w = ctypes.c_size_t()
            pf = np.empty(plen * 32, np.uint8)
            pf[PROOF_SIZE * 32:] = blob_proofs[c]
            for j in range(N):
                r = c * N + j
                pf[:PROOF_SIZE * 32] = proofs_np[r]
                check(lib().decds_pcc_to_bytes(c, r, rows[j].ctypes.data_as(ctypes.c_void_p), F,
                                               pf.ctypes.data_as(ctypes.c_void_p), plen, out, cap, ctypes.byref(w)))
                with open(os.path.join(d, "share%02d.data" % j), "wb") as f:
                    f.write(memoryview(out)[:w.value])

        if device_store:                                               # 3. rows out, shares written
            slots_out = [_pinned((bmax * N, F), torch) for _ in range(2)]
            writing = [[], []]
            for k, c0 in enumerate(range(0, n, bmax)):
                b = min(bmax, n - c0)
                sl = k % 2
                for fut in writing[sl]:
                    fut.result()                                       # the slot's previous shares are out
                with torch.cuda.stream(stream):
                    slots_out[sl][:b * N].view(-1).copy_(store[c0 * N * F:(c0 + b) * N * F], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(stream)
                ev.synchronize()
                rows = slots_out[sl].numpy()
                writing[sl] = [pool.submit(write_chunkset, c0 + s, rows[s * N:(s + 1) * N]) for s in range(b)]
            for w_ in writing:
                for fut in w_:
                    fut.result()
        else:
            rows = host_store.numpy()
            list(pool.map(lambda c: write_chunkset(c, rows[c * N:(c + 1) * N]), range(n)))
        dth.join()
        header = wire.BlobHeader(size, n, digest[0], blob_root, cs_roots)
        with open(os.path.join(target_dir, "metadata.commit"), "wb") as f:  # handle_break.rs:49-64
            f.write(header.to_bytes())
        t["out_write_s"] = time.perf_counter() - t0
    finally:
        pool.shutdown(wait=True)
        if dth.is_alive():
            dth.join()
        stream.synchronize()
    t["device_store"] = bool(device_store)
    t["total_s"] = time.perf_counter() - t_start
    return header


def read_blob_metadata(chunk_dir):
    """decds-bin utils.rs:20-44: the file must hold exactly one header."""
    b = open(os.path.join(chunk_dir, "metadata.commit"), "rb").read()
    h, used = wire.BlobHeader.from_bytes(b)
    if used != len(b):
        raise DecdsError(13, "erasure-coded blob metadata file is %d bytes longer than it should be" % (len(b) - used))
    return h


class _ForeignChunk(Exception):
    """a parsed share claims another chunkset's id: only the sequential loop reproduces the reference"""


def repair_blob_sequential(ctx, chunk_dir, target_dir):
    """handle_repair.rs:41-92 exactly: chunkset directories in order, shares 0..15 of each until the
    chunkset is ready, every parsed chunk through RepairingBlob::add_chunk (the C-ABI incremental
    object: routing by the chunk's own chunkset id, validation, rank test), InvalidProofInChunk /
    InvalidChunkMetadata / ChunkDecodingFailed ignored and any other error fatal (the reference
    exits 1), then get_repaired_chunkset; finally repaired.data and its digest check."""
    from .blob import RepairingBlob
    header = read_blob_metadata(chunk_dir)
    n = header.get_num_chunksets()
    rep = RepairingBlob(ctx, header)
    os.makedirs(target_dir, exist_ok=True)
    parts = []
    for c in range(n):
        for j in range(N):
            if rep.is_chunkset_ready_to_repair(c):
                break
            path = os.path.join(chunk_dir, "chunkset.%d" % c, "share%02d.data" % j)
            if not os.path.isfile(path):
                continue
            try:
                raw = open(path, "rb").read()
                chunk, used = wire.pcc_from_bytes(raw)
            except (OSError, DecdsError):
                continue                                               # unreadable: skipped (utils.rs:47-65)
            if used != len(raw):
                continue
            try:
                rep.add_chunk(chunk)
            except DecdsError as e:
                if e.kind not in ("InvalidProofInChunk", "InvalidChunkMetadata", "ChunkDecodingFailed"):
                    raise                                              # handle_repair.rs:64-67: exit(1)
        if not rep.is_chunkset_ready_to_repair(c):
            raise DecdsError(5, "failed to repair chunkset %d" % c)    # handle_repair.rs:77-80
        data = rep.get_repaired_chunkset(c)
        with open(os.path.join(target_dir, "chunkset.%d.data" % c), "wb") as f:
            f.write(data)
        parts.append(data)
    out_path = os.path.join(target_dir, "repaired.data")
    blob = b"".join(parts)
    with open(out_path, "wb") as f:
        f.write(blob)
    if _blake3(np.frombuffer(blob, np.uint8)) != header.get_blob_digest():   # handle_repair.rs:129-151
        raise DecdsError(6, "repaired blob digest does not match the header")
    return out_path


def repair_blob(ctx, chunk_dir, target_dir, batch=16, timings=None, threads=16):
    """handle_repair over device batches (see _repair_batched); falls back to the reference's
    sequential loop (repair_blob_sequential) when a share claims another chunkset's id."""
    try:
        return _repair_batched(ctx, chunk_dir, target_dir, batch, timings, threads)
    except _ForeignChunk:
        if timings is not None:
            timings["sequential"] = True
        return repair_blob_sequential(ctx, chunk_dir, target_dir)


def _repair_batched(ctx, chunk_dir, target_dir, batch, timings, threads):
    """handle_repair over device batches. Returns the repaired bytes' path; raises DecdsError if a
    chunkset cannot be repaired or the repaired digest differs (handle_repair.rs:79-84, 129-151).
    Share files are read and parsed by `threads` workers straight into a page-locked staging
    buffer laid out as the chunksets' 16 coded-row slots (share j of chunkset slot s at row
    s*16 + j), so validation, plan and decode run on it in place after one H2D copy."""
    import torch
    t = {} if timings is None else timings
    header = read_blob_metadata(chunk_dir)
    n = header.get_num_chunksets()
    blob_size = header.get_blob_size()
    dev = torch.device("cuda", ctx.device)
    roots_d = torch.from_numpy(np.frombuffer(b"".join(header.chunkset_root_commitments), np.uint8).copy()).to(dev)
    broot_d = torch.from_numpy(np.frombuffer(header.root_commitment, np.uint8).copy()).to(dev)
    os.makedirs(target_dir, exist_ok=True)
    out_path = os.path.join(target_dir, "repaired.data")
    plen = PROOF_SIZE + max(0, (n - 1).bit_length())                   # 4 chunkset + blob-level hashes
    t_start = time.perf_counter()
    bmax = min(batch, n)
    # page-locked staging for one batch of shares and two batches of repaired chunksets (no
    # page-locked copy of the whole blob: pinning costs ~0.25 s per GiB on the GPU box)
    rows_h = _pinned((bmax * N, F), torch)
    prf_h = _pinned((bmax * N, plen * 32), torch)
    outs_h = [_pinned(bmax * CS, torch) for _ in range(2)]
    rows_np, prf_np = rows_h.numpy(), prf_h.numpy()
    ids_np = np.empty((bmax * N, 2), np.int64)
    filled = np.zeros(bmax * N, bool)
    stream = torch.cuda.Stream(dev)
    with torch.cuda.stream(stream):
        rows_d = torch.empty(bmax * N * F, dtype=torch.uint8, device=dev)
        prf_d = torch.empty(bmax * N * plen * 32, dtype=torch.uint8, device=dev)
        ids_d = torch.empty(bmax * N * 2, dtype=torch.int64, device=dev)
        dig = torch.empty(bmax * N * 32, dtype=torch.uint8, device=dev)
        valid = torch.empty(bmax * N, dtype=torch.uint8, device=dev)
        plan = torch.empty(bmax * 128, dtype=torch.uint8, device=dev)
        verd = torch.empty(bmax * N, dtype=torch.int8, device=dev)
        status = torch.empty(bmax, dtype=torch.int32, device=dev)
        dst = torch.empty(bmax * CS, dtype=torch.uint8, device=dev)
    t["alloc_s"] = time.perf_counter() - t_start
    t_read = t_dev = 0.0
    foreign = [False]

    def read_chunkset(c0, s):                                          # handle_repair.rs:53-76
        cs, ch = ctypes.c_uint64(), ctypes.c_uint64()
        dp, pp = ctypes.c_void_p(), ctypes.c_void_p()
        dl, pl, used = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        for j in range(N):
            r = s * N + j
            filled[r] = False
            ids_np[r] = (n, 0)                                         # never valid unless overwritten
            try:
                with open(os.path.join(chunk_dir, "chunkset.%d" % (c0 + s), "share%02d.data" % j), "rb") as f:
                    raw = bytearray(f.read())
            except OSError:
                continue                                               # missing share: skipped
            src = (ctypes.c_char * len(raw)).from_buffer(raw)
            st = lib().decds_pcc_from_bytes(src, len(raw), ctypes.byref(cs), ctypes.byref(ch), ctypes.byref(dp),
                                            ctypes.byref(dl), ctypes.byref(pp), ctypes.byref(pl), ctypes.byref(used))
            if st == 0 and used.value == len(raw) and cs.value != c0 + s:
                foreign[0] = True                                      # routed elsewhere by the reference
            if st != 0 or used.value != len(raw) or dl.value != F or pl.value != plen:
                continue                                               # unreadable / malformed: skipped
            base = ctypes.addressof(src)
            mv = memoryview(raw)
            rows_np[r] = np.frombuffer(mv[dp.value - base:dp.value - base + F], np.uint8)
            prf_np[r] = np.frombuffer(mv[pp.value - base:pp.value - base + plen * 32], np.uint8)
            ids_np[r] = (cs.value, ch.value)
            filled[r] = True

    fd = os.open(out_path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)

    def write_part(c, part):                                           # handle_repair.rs:86-96
        with open(os.path.join(target_dir, "chunkset.%d.data" % c), "wb") as f:
            f.write(part)
        os.pwrite(fd, part, c * CS)                                    # repaired.data, in place

    writing = [[], []]
    # the repaired blob's digest (handle_repair.rs:129-151), hashed batch by batch from the output
    # slots in blob order on its own thread (incremental BLAKE3) while the workers write
    hasher = lib().decds_blake3_stream_new()
    t_hash = [0.0]

    def hash_part(part):
        t1 = time.perf_counter()
        lib().decds_blake3_stream_update(hasher, part.ctypes.data, part.size, max(1, threads // 2))
        t_hash[0] += time.perf_counter() - t1

    hpool = ThreadPoolExecutor(max_workers=1)
    try:
        with ThreadPoolExecutor(max_workers=max(1, threads)) as pool:
            for k, c0 in enumerate(range(0, n, bmax)):
                b = min(bmax, n - c0)
                t0 = time.perf_counter()
                list(pool.map(lambda s: read_chunkset(c0, s), range(b)))
                t_read += time.perf_counter() - t0
                if foreign[0]:
                    stream.synchronize()
                    raise _ForeignChunk()
                t0 = time.perf_counter()
                m = b * N
                with torch.cuda.stream(stream):
                    rows_d[:m * F].copy_(rows_h[:m].view(-1), non_blocking=True)
                    prf_d[:m * plen * 32].copy_(prf_h[:m].view(-1), non_blocking=True)
                    ids_d[:m * 2].copy_(torch.from_numpy(ids_np[:m].reshape(-1)), non_blocking=False)
                    codec.validate_batch(ctx, rows_d, m, ids_d, prf_d, plen, roots_d, n, dig, valid, blob_root=broot_d,
                                         stream=stream)
                    v = valid[:m].cpu().numpy().astype(bool)           # (on `stream`: waits for it)
                    cand = np.full((b, N), NO_CANDIDATE, np.uint8)
                    for s in range(b):
                        ok = np.nonzero(filled[s * N:(s + 1) * N] & v[s * N:(s + 1) * N]
                                        & (ids_np[s * N:(s + 1) * N, 0] == c0 + s))[0]
                        cand[s, :ok.size] = ok
                    codec.repair_batch(ctx, rows_d, b, torch.from_numpy(cand).to(dev), plan, verd, dst, status,
                                       stream=stream)
                    st = status[:b].cpu().numpy()
                    bad = [c0 + s for s in range(b) if st[s] != 0]
                    if bad:
                        raise DecdsError(6 if any(st[s] == 6 for s in range(b)) else 5,
                                         "failed to repair chunkset(s) %s" % bad[:8])
                    sl = k % 2
                    for fut in writing[sl]:
                        fut.result()                                   # the slot's previous batch is written
                    outs_h[sl][:b * CS].copy_(dst[:b * CS], non_blocking=True)
                stream.synchronize()
                t_dev += time.perf_counter() - t0
                ob = outs_h[sl].numpy()
                writing[sl] = [pool.submit(write_part, c0 + s,
                                           memoryview(ob[s * CS:s * CS + min(CS, blob_size - (c0 + s) * CS)]))
                               for s in range(b)]
                writing[sl].append(hpool.submit(hash_part, ob[:min(b * CS, blob_size - c0 * CS)]))
            t0 = time.perf_counter()
            for w_ in writing:
                for fut in w_:
                    fut.result()
            t["write_tail_s"] = time.perf_counter() - t0
        dg = ctypes.create_string_buffer(32)
        lib().decds_blake3_stream_finalize(hasher, dg)
        digest = [dg.raw]
        t["digest_s"] = t_hash[0]
    finally:
        hpool.shutdown(wait=True)
        lib().decds_blake3_stream_free(hasher)
        os.close(fd)
    ok = digest[0] == header.get_blob_digest()                          # handle_repair.rs:129-151
    t["read_s"], t["device_s"] = t_read, t_dev
    t["total_s"] = time.perf_counter() - t_start
    if not ok:
        raise DecdsError(6, "repaired blob digest does not match the header")
    return out_path

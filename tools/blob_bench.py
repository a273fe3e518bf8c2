"""The reference's public blob API at the C-ABI, timed end to end from host memory (SURVEY.md §8a
rows a9/a10): Blob::new over a random blob (whole-blob BLAKE3 on host threads, encode + commitment on
the device, blob-level tree, chunks back in host memory), then the incremental RepairingBlob the way
decds-bin's repair loop drives it (handle_repair.rs:41-92): per chunkset, chunks of 10 random shares
one add_chunk call at a time (each validated: chunk digest + two Merkle paths on the host), then
get_repaired_chunkset for every chunkset (ready chunksets decoded in device batches), checked
against the blob. Also the batched add_chunks form (validation on the device). One JSON line.

usage: python tools/blob_bench.py [--gib 1]"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=1.0)
    ap.add_argument("--share-major", action="store_true",
                    help="chunks arrive share by share over all chunksets (every chunkset open at once, as "
                         "Blob::get_share hands them out) instead of chunkset by chunkset")
    ap.add_argument("--budgets-mb", default="", help="comma list of RepairingBlob device budgets (MiB) to time "
                                                       "the sequential add_chunk path under, e.g. 0,512")
    ap.add_argument("--contexts", type=int, default=1, help="RepairingBlob over this many contexts of device 0")
    a = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (torch's HIP runtime first, as the other tools)
    import decds_amd
    from decds_amd import codec
    from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N, check, lib
    from decds_amd.blob import Blob, HostBuffer, RepairingBlob

    L = lib()
    ctx = decds_amd.Context(0)
    size = int(a.gib * (1 << 30))
    data = HostBuffer(size)
    data.array[:] = codec.fill_random_host(0xB10B, size)
    n = -(-size // CS)
    res = {"blob_GiB": a.gib, "chunksets": n}

    t0 = time.perf_counter()
    blob = Blob(ctx, data.array)
    res["blob_new_s"] = round(time.perf_counter() - t0, 3)
    res["blob_new_GiBps"] = round(a.gib / res["blob_new_s"], 2)
    header = blob.get_blob_header()
    plen = blob.proof_len()
    rng = np.random.default_rng(7)
    picks = [rng.permutation(N)[:K] for _ in range(n)]
    # pointers to every picked chunk inside the blob (zero-copy) and its proof
    dp = ctypes.c_void_p()
    chunks = []
    order = [(c, k) for k in range(K) for c in range(n)] if a.share_major else [(c, k) for c in range(n) for k in range(K)]
    res["arrival"] = "share-major" if a.share_major else "chunkset-major"
    for c, k in order:
        j = picks[c][k]
        proof = ctypes.create_string_buffer(32 * plen)
        check(L.decds_blob_get_chunk(blob._h, c, int(j), ctypes.byref(dp), proof, len(proof)))
        chunks.append((c, c * N + int(j), dp.value, proof))
    ctxs = [ctx] + [decds_amd.Context(0) for _ in range(a.contexts - 1)]
    res["contexts"] = a.contexts

    def repair(batched, budget=None):
        rb = RepairingBlob(ctxs if len(ctxs) > 1 else ctx, header, device_budget=budget)
        t0 = time.perf_counter()
        if batched:
            m = len(chunks)
            rows = np.empty((m, F), np.uint8)
            ids = np.empty((m, 2), np.uint64)
            prf = np.empty((m, plen * 32), np.uint8)
            for i, (c, gid, p, proof) in enumerate(chunks):
                rows[i] = np.ctypeslib.as_array((ctypes.c_uint8 * F).from_address(p))
                ids[i] = (c, gid)
                prf[i] = np.frombuffer(proof.raw, np.uint8)
            t0 = time.perf_counter()  # the batch call alone (the row gather above is the caller's)
            st = rb.add_rows(rows, ids, prf, plen)
            assert (st == 0).sum() >= n * (K - 1), "too many rejected chunks"
        else:
            for c, gid, p, proof in chunks:
                s = L.decds_repairing_blob_add_chunk(rb._h, c, gid, ctypes.c_void_p(p), F, proof, plen)
                if s not in (0, 4):  # 4: ChunkDecodingFailed (a dependent chunk), which the reference tolerates
                    check(s)
        t_add = time.perf_counter() - t0
        mem = rb.memory()
        out = HostBuffer(CS)
        t_get = 0.0
        ok = 0
        for c in range(n):
            t0 = time.perf_counter()
            if not rb.is_chunkset_ready_to_repair(c):
                t_get += time.perf_counter() - t0
                continue
            got = rb.get_repaired_chunkset(c, out=out.array)
            t_get += time.perf_counter() - t0  # the check below is the caller's, outside the timing
            lo = c * CS
            assert np.array_equal(got, data.array[lo:lo + got.size]), c
            ok += 1
        del got
        out.free()
        rb.free()
        return t_add, t_get, ok, mem

    runs = [("add_chunk", False, None), ("add_chunks_batch", True, None)]
    runs += [("add_chunk_budget_%sMiB" % b, False, int(b) << 20) for b in a.budgets_mb.split(",") if b != ""]
    for name, batched, budget in runs:
        t_add, t_get, ok, mem = repair(batched, budget)
        gib_ok = ok * CS / (1 << 30)
        res[name] = {"add_s": round(t_add, 3), "get_repaired_s": round(t_get, 3), "repaired_chunksets": ok,
                     "GiBps": round(gib_ok / (t_add + t_get), 2),
                     "per_chunk_add_us": round(t_add / len(chunks) * 1e6, 1),
                     "device_chunksets": mem["device_chunksets"], "spilled_chunksets": mem["spilled_chunksets"],
                     "device_MiB": round(mem["device_bytes"] / 2 ** 20, 1)}
    # a second Blob::new of the same size after the first is freed: its coded store comes from the
    # library's page-locked block cache instead of being page-locked again
    t0 = time.perf_counter()
    blob.free()
    res["blob_free_s"] = round(time.perf_counter() - t0, 3)
    t0 = time.perf_counter()
    blob2 = Blob(ctx, data.array)
    res["blob_new_cached_s"] = round(time.perf_counter() - t0, 3)
    res["blob_new_cached_GiBps"] = round(a.gib / res["blob_new_cached_s"], 2)
    h2 = blob2.get_blob_header()  # fresh random coding vectors: only the data-derived fields agree
    assert (h2.get_blob_size(), h2.get_num_chunksets(), h2.get_blob_digest()) == \
        (header.get_blob_size(), header.get_num_chunksets(), header.get_blob_digest())
    blob2.free()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

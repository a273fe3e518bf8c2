"""Throughput of the per-chunkset drop-in path (decds_chunkset_new = ChunkSet::new with its commitment,
decds_repairing_chunkset_repair = RepairingChunkSet::repair) under T concurrent host threads — the
reference calls ChunkSet::new from rayon workers (blob.rs:256-264) — next to the blob-level host
paths (decds_blob_encode_host / _repair_host) with pageable (staged) and registered caller memory.
Host memory -> host memory, PCIe included. One JSON line per measurement.

usage: python tools/mirror_bench.py [--threads 1,4,16] [--seconds 2] [--blob-gib 2]"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GIB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,4,8,16")
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--blob-gib", type=float, default=2.0)
    ap.add_argument("--reps", type=int, default=5, help="timed blob-path repetitions per mode (median)")
    ap.add_argument("--modes", default="pageable,host_alloc,host_register")
    ap.add_argument("--blob-only", action="store_true")
    ap.add_argument("--no-blob", action="store_true", help="only the per-chunkset mirror rows")
    a = ap.parse_args()
    import numpy as np
    import decds_amd
    from decds_amd import codec
    from decds_amd._capi import CHUNKSET_BYTES as CS, K, N

    ctx = decds_amd.Context(0)
    for T in ([] if a.blob_only else [int(t) for t in a.threads.split(",")]):
        datas = [codec.fill_random_host(0x77 + t, CS).tobytes() for t in range(T)]
        coeffs = [codec.fill_random_host(0x88 + t, N * K).tobytes() for t in range(T)]
        # one warm call per thread slot (lane creation: stream, device buffers, pinned staging)
        for t in range(T):
            decds_amd.ChunkSet(ctx, t, datas[t], coeffs[t])
        counts = [0] * T
        stop = time.perf_counter() + a.seconds

        def enc(t):
            while time.perf_counter() < stop:
                decds_amd.ChunkSet(ctx, t, datas[t], coeffs[t])
                counts[t] += 1

        t0 = time.perf_counter()
        th = [threading.Thread(target=enc, args=(t,)) for t in range(T)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        dt = time.perf_counter() - t0
        print(json.dumps({"path": "decds_chunkset_new (ChunkSet::new + commitment)", "threads": T,
                          "coalesced": os.environ.get("DECDS_CHUNKSET_COALESCE", "0").strip() not in ("", "0"),
                          "chunksets": sum(counts), "GiBps": round(sum(counts) * CS / GIB / dt, 2)}), flush=True)
        # repair: RepairingChunkSet with 10 chunks already added, repair() timed
        cs = [decds_amd.ChunkSet(ctx, t, datas[t], coeffs[t]) for t in range(T)]
        chunks = [[c.get_chunk(j) for j in range(K)] for c in cs]
        counts = [0] * T
        stop = time.perf_counter() + a.seconds

        def rep(t):
            while time.perf_counter() < stop:
                r = decds_amd.RepairingChunkSet(ctx, t)
                for ch in chunks[t]:
                    r.add_chunk_unvalidated(ch)
                r.repair()
                counts[t] += 1

        t0 = time.perf_counter()
        th = [threading.Thread(target=rep, args=(t,)) for t in range(T)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        dt = time.perf_counter() - t0
        print(json.dumps({"path": "decds_repairing_chunkset_repair (add 10 chunks + repair)", "threads": T,
                          "chunksets": sum(counts), "GiBps": round(sum(counts) * CS / GIB / dt, 2)}), flush=True)

    if a.no_blob:
        return
    # blob-level host paths over the same kind of data: pageable (staged through the library's rings),
    # library page-locked memory (decds_host_alloc) and registered caller memory (decds_host_register)
    n = max(1, int(a.blob_gib * GIB) // CS)
    blob = codec.fill_random_host(0x99, n * CS)
    cv = codec.fill_random_host(0x9A, n * N * K)
    cand = np.stack([np.random.default_rng(c).permutation(N) for c in range(n)]).astype(np.uint8)
    for mode in a.modes.split(","):
        bufs, regs = [], []
        if mode == "host_alloc":
            hb = [decds_amd.HostBuffer(blob.nbytes), decds_amd.HostBuffer(n * N * codec.CODED_PIECE_BYTES),
                  decds_amd.HostBuffer(blob.nbytes)]
            hb[0].array[:] = blob
            b_in, coded_out, rep_out = hb[0].array, hb[1].array.reshape(n * N, -1), hb[2].array
            bufs = hb
        else:
            b_in, coded_out, rep_out = blob, np.empty((n * N, codec.CODED_PIECE_BYTES), np.uint8), np.empty(blob.nbytes, np.uint8)
            coded_out[:] = 0
            rep_out[:] = 0
            if mode == "host_register":
                regs = [blob, coded_out, rep_out]
                for r in regs:
                    codec.host_register(r)
        codec.blob_encode_host(ctx, b_in, cv, out=coded_out)  # warm (slot buffers, rings)
        codec.blob_repair_host(ctx, coded_out, cand, blob.nbytes, out=rep_out)
        te, tr = [], []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            codec.blob_encode_host(ctx, b_in, cv, out=coded_out)
            te.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            _, st = codec.blob_repair_host(ctx, coded_out, cand, blob.nbytes, out=rep_out)
            tr.append(time.perf_counter() - t0)
        assert (st == 0).all() and np.array_equal(rep_out, blob)
        te, tr = float(np.median(te)), float(np.median(tr))
        print(json.dumps({"path": "decds_blob_encode_host / _repair_host", "memory": mode, "chunksets": n, "reps": a.reps,
                          "encode_GiBps": round(n * CS / GIB / te, 2), "repair_GiBps": round(n * CS / GIB / tr, 2)}),
              flush=True)
        for r in regs:
            codec.host_unregister(r)
        for b in bufs:
            b.free()


if __name__ == "__main__":
    main()

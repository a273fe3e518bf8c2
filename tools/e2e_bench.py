"""Host-memory end-to-end rate of the blob-level path (blob file bytes in host RAM -> coded chunks in
host RAM -> repaired blob in host RAM): decds_blob_encode_host / decds_blob_repair_host with
page-locked caller buffers and H2D / kernel / D2H overlapped on two streams. PCIe-inclusive, so it
is bounded by the host link, not HBM (DESIGN.md "End-to-end rate"). Prints one JSON line.
usage: python tools/e2e_bench.py --gib 4 --batch 32"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--memory", choices=("register", "alloc"), default="register",
                    help="caller buffers page-locked by decds_host_register (default) or allocated by decds_host_alloc")
    ap.add_argument("--with-torch", action="store_true", help="initialise torch on the device first (as bench.py does)")
    ap.add_argument("--with-pattern", action="store_true", help="load and use the pattern-ceiling build first (as bench.py does)")
    ap.add_argument("--device-gib", type=float, default=0.0,
                    help="hold this much device memory (torch) before the page-locked buffers are allocated")
    ap.add_argument("--pre-streams", type=int, default=0,
                    help="create this many HIP streams (torch.cuda.Stream) before the library's, and keep them")
    ap.add_argument("--cand", choices=("random", "first", "all"), default="random",
                    help="the rows repair gets: 10 random of 16 (default), rows 0-9, or all 16 in order")
    ap.add_argument("--cpus", default=None, help="run on these CPUs only (e.g. 0-15 or 128-143): NUMA placement of the "
                                                    "page-locked buffers")
    a = ap.parse_args()
    if a.cpus:
        lo, _, hi = a.cpus.partition("-")
        os.sched_setaffinity(0, range(int(lo), int(hi or lo) + 1))
    import numpy as np
    if a.with_torch or a.with_pattern or a.device_gib or a.pre_streams:
        import torch
        torch.cuda.init()
        torch.zeros(1, device="cuda")
        print(json.dumps({"stream_priority_range": torch.cuda.Stream.priority_range()}))
        streams = [torch.cuda.Stream() for _ in range(a.pre_streams)]
        for s_ in streams:  # a stream takes its hardware queue when first used
            with torch.cuda.stream(s_):
                torch.zeros(1, device="cuda")
        torch.cuda.synchronize()
        held = torch.empty(int(a.device_gib * (1 << 30)), dtype=torch.uint8, device="cuda") if a.device_gib else None
    if a.with_pattern:
        import ctypes
        Lp = ctypes.CDLL(os.path.join(ROOT, "tools", "bin", "libdecds_pattern.so"))
        h = ctypes.c_void_p()
        Lp.decds_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        Lp.decds_ctx_destroy.argtypes = [ctypes.c_void_p]
        assert Lp.decds_ctx_create(0, ctypes.byref(h)) == 0
        Lp.decds_ctx_destroy(h)
    import decds_amd
    from decds_amd import codec
    from decds_amd._capi import CHUNKSET_BYTES as CS, K, N

    ctx = decds_amd.Context(0)
    blob_len = int(a.gib * (1 << 30))
    n = -(-blob_len // CS)
    t = time.time()
    blob = codec.fill_random_host(0xDEC05003, blob_len)
    coeffs = codec.fill_random_host(0xC0EF0003, n * N * K)
    rng = np.random.default_rng(0x5EED0003)
    cand = np.full((n, N), 0xFF, np.uint8)
    for c in range(n):
        if a.cand == "random":
            cand[c, :K] = rng.permutation(N)[:K]
        elif a.cand == "first":
            cand[c, :K] = np.arange(K)
        else:
            cand[c, :] = np.arange(N)
    gen_s = time.time() - t
    # cold: every call pins/unpins the caller buffers itself (first rep); warm: buffers pinned once
    enc, rep = [], []
    if a.memory == "alloc":  # page-locked from the start: every call is warm
        from decds_amd.blob import HostBuffer
        hbs = [HostBuffer(blob_len), HostBuffer(n * N * (CS // K + 1 + K)), HostBuffer(blob_len)]
        hbs[0].array[:] = blob
        blob, coded_buf, out_buf = hbs[0].array, hbs[1].array.reshape(n * N, -1), hbs[2].array
    else:
        coded_buf = np.empty((n * N, CS // K + 1 + K), dtype=np.uint8)
        out_buf = np.empty(blob_len, dtype=np.uint8)
    for rep_i in range(a.reps + 1):
        if rep_i == 1 and a.memory == "register":
            for b in (blob, coeffs, coded_buf, out_buf):
                codec.host_register(b)
        t = time.perf_counter()
        coded = codec.blob_encode_host(ctx, blob, coeffs, batch=a.batch, out=coded_buf)
        enc.append(time.perf_counter() - t)
        t = time.perf_counter()
        out, status = codec.blob_repair_host(ctx, coded, cand, blob_len, batch=a.batch, out=out_buf)
        rep.append(time.perf_counter() - t)
    ok = status == 0
    good = all(np.array_equal(out[c * CS:min((c + 1) * CS, blob_len)], blob[c * CS:min((c + 1) * CS, blob_len)])
               for c in np.nonzero(ok)[0][:8])
    cold_e, cold_r = enc[0], rep[0]
    e, r = min(enc[1:]), min(rep[1:])
    e_med, r_med = float(np.median(enc[1:])), float(np.median(rep[1:]))
    print(json.dumps({"blob_gib": a.gib, "memory": a.memory, "cpus": a.cpus, "device_gib": a.device_gib, "pre_streams": a.pre_streams, "cand": a.cand, "chunksets": n, "batch": a.batch,
                      "encode_median_s": round(e_med, 4), "repair_median_s": round(r_med, 4), "encode_s": round(e, 4),
                      "repair_s": round(r, 4), "encode_blob_GiBps": round(blob_len / (1 << 30) / e, 2),
                      "repair_blob_GiBps": round(blob_len / (1 << 30) / r, 2),
                      "encode_pcie_GBps": round((blob_len + n * N * (CS // K + 1 + K)) / e / 1e9, 2),
                      "repair_pcie_GBps": round((n * K * (CS // K + 1 + K) + blob_len) / r / 1e9, 2),
                      "cold_encode_blob_GiBps": round(blob_len / (1 << 30) / cold_e, 2),
                      "cold_repair_blob_GiBps": round(blob_len / (1 << 30) / cold_r, 2), "ready": int(ok.sum()), "spot_check_ok": bool(good), "host_gen_s": round(gen_s, 1)}))


if __name__ == "__main__":
    main()

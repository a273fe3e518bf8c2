"""Where Blob::new's time goes: decds_blob_new against its parts on one blob size,
each the median of `--repeats` warm calls. One JSON line.

  encode_host_pinned     decds_blob_encode_host, page-locked blob in / coded rows out (bench's end_to_end)
  encode_host_pageable   the same on plain (pageable) numpy memory: staged through the bounce rings
  blake3_16              decds_blake3_parallel over the blob on 16 host threads, alone
  encode_plus_blake3     encode_host_pinned with the blake3 running beside it on a second host thread
  blob_new_pinned        decds_blob_new on a page-locked blob (first call = cold, reported apart)
  blob_new_pageable      decds_blob_new on a pageable blob (what a Rust Vec<u8> is)

usage: python tools/blob_breakdown.py [--gib 1] [--repeats 5]"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=1.0)
    ap.add_argument("--repeats", type=int, default=5)
    ap.add_argument("--only", default="", help="comma list of the parts to time (default: all)")
    a = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (torch's HIP runtime first, as the other tools)
    import decds_amd
    from decds_amd import codec
    from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N, lib
    from decds_amd.blob import Blob, HostBuffer

    L = lib()
    ctx = decds_amd.Context(0)
    size = int(a.gib * (1 << 30))
    n = -(-size // CS)
    pin_in, pin_out = HostBuffer(size), HostBuffer(n * N * F)
    pin_in.array[:] = codec.fill_random_host(0xB10B, size)
    page_in = np.array(pin_in.array, copy=True)
    page_out = np.empty(n * N * F, np.uint8)
    coeffs = codec.fill_random_host(0xC0EF, n * N * K)
    res = {"blob_bytes": size, "chunksets": n, "repeats": a.repeats}

    def throttled():
        """cgroup v2 cpu.stat: (nr_throttled, throttled_usec), None where unreadable"""
        try:
            with open("/sys/fs/cgroup/cpu.stat") as f:
                kv = dict(ln.split() for ln in f if ln.strip())
            return int(kv.get("nr_throttled", 0)), int(kv.get("throttled_usec", 0))
        except (OSError, ValueError):
            return None

    def med(fn, reps=a.repeats, warm=1):
        for _ in range(warm):
            fn()
        ts = []
        th0 = throttled()
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        th1 = throttled()
        res.setdefault("cgroup_throttled", []).append(None if th0 is None else [th1[0] - th0[0], (th1[1] - th0[1]) / 1e3])
        return round(float(np.median(ts)) * 1e3, 3), [round(min(ts) * 1e3, 3), round(max(ts) * 1e3, 3)]

    out32 = ctypes.create_string_buffer(32)
    b3 = lambda: L.decds_blake3_parallel(ctypes.c_void_p(pin_in.array.ctypes.data), size, out32, 16)
    enc_pin = lambda: codec.blob_encode_host(ctx, pin_in.array, coeffs, out=pin_out.array.reshape(n * N, F))
    enc_page = lambda: codec.blob_encode_host(ctx, page_in, coeffs, out=page_out.reshape(n * N, F))

    def enc_plus_b3():
        t = threading.Thread(target=b3)
        t.start()
        enc_pin()
        t.join()

    only = set(x for x in a.only.split(",") if x)
    for name, fn in (("encode_host_pinned", enc_pin), ("encode_host_pageable", enc_page), ("blake3_16", b3),
                     ("encode_plus_blake3", enc_plus_b3)):
        if only and name not in only:
            continue
        ms, spread = med(fn)
        res[name] = {"throttled_periods_ms": res["cgroup_throttled"][-1], "ms": ms, "spread_ms": spread, "GiBps": round(size / (1 << 30) / (ms * 1e-3), 2)}

    def blob_new(src):
        def run():
            Blob(ctx, src).free()
        return run

    for name, src in (("blob_new_pinned", pin_in.array), ("blob_new_pageable", page_in)):
        if only and name not in only:
            continue
        t0 = time.perf_counter()
        Blob(ctx, src).free()
        cold = round((time.perf_counter() - t0) * 1e3, 3)
        ms, spread = med(blob_new(src), warm=0)
        res[name] = {"throttled_periods_ms": res["cgroup_throttled"][-1], "cold_ms": cold, "ms": ms, "spread_ms": spread, "GiBps": round(size / (1 << 30) / (ms * 1e-3), 2)}
    if "blob_new_pinned" in res and "encode_host_pinned" in res:
        res["ratio_blob_new_pinned_over_encode_host"] = round(res["blob_new_pinned"]["ms"] / res["encode_host_pinned"]["ms"], 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

"""decds_commit_batch (chunk digests + Merkle roots + proofs) on HBM-resident coded rows, in-process
A/B of library builds (rounds alternate between builds): cfg2's 103 chunksets in the bench's
payload-aligned layout (+118) and the message-aligned one (+16). Every build's roots must equal the
first build's. One JSON line per build and layout.

usage: python tools/digestbench.py --n 103 build/ab/lib_a.so build/ab/lib_b.so ...
"""
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
    ap.add_argument("--n", type=int, default=103)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--offsets", default="118,16")
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    import numpy as np
    import torch
    from decds_amd._capi import CODED_PITCH_ALIGNED as P, N, _declare

    n = a.n
    vp = ctypes.c_void_p
    st = torch.cuda.Stream()
    sp = vp(st.cuda_stream)
    builds = []
    for path in a.libs:
        L = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
        _declare(L)
        h = ctypes.c_void_p()
        assert L.decds_ctx_create(0, ctypes.byref(h)) == 0
        builds.append({"tag": os.path.basename(path)[:-3], "lib": L, "ctx": h})
    buf = torch.empty(n * N * P + 256, dtype=torch.uint8, device="cuda")
    builds[0]["lib"].decds_fill_random_device(builds[0]["ctx"], 7, 0, vp(buf.data_ptr()), buf.numel(), sp)
    dig = torch.empty(n * N * 32, dtype=torch.uint8, device="cuda")
    roots = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    proofs = torch.empty(n * N * 128, dtype=torch.uint8, device="cuda")
    st.synchronize()
    for o in [int(x) for x in a.offsets.split(",")]:
        off = (o - buf.data_ptr()) % 128
        coded = vp(buf.data_ptr() + off)

        def run(b):
            assert b["lib"].decds_commit_batch(b["ctx"], coded, P, n, 0, vp(dig.data_ptr()), vp(roots.data_ptr()),
                                               vp(proofs.data_ptr()), sp) == 0

        ref = None
        for b in builds:
            run(b)
            st.synchronize()
            if ref is None:
                ref = roots.clone()
            assert torch.equal(ref, roots), b["tag"] + ": roots differ from the first build's"
            b["t"] = []
        t0 = time.time()
        while time.time() - t0 < 1.0:
            for b in builds:
                run(b)
            st.synchronize()
        for r in range(a.rounds):
            for b in (builds if r % 2 == 0 else builds[::-1]):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                run(b)
                e1.record(st)
                st.synchronize()
                b["t"].append(e0.elapsed_time(e1))
        for b in builds:
            ms = float(np.median(b["t"]))
            print(json.dumps({"tag": b["tag"], "n": n, "row_offset": o, "commit_ms": round(ms, 4),
                              "GBps_coded": round(n * N * P / (ms * 1e-3) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()

"""ChunkSet::new on the device, in-process A/B of library builds (cdna_hip_programming.md §5.4 rule 24):
per build, decds_encode_commit_batch on rows 16 bytes past a 128-byte boundary (the fused kernel)
against decds_encode_batch + decds_commit_batch (separate kernels), rounds alternating between
builds. Every build's roots must equal the first build's. One JSON line per build.

usage: python tools/fusebench.py --n 103 --rounds 8 build/ab/lib_a.so build/ab/lib_b.so ...
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
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--warmup-s", type=float, default=2.0)
    ap.add_argument("--no-check", action="store_true", help="timing-only builds: skip the roots comparison")
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    import numpy as np
    import torch
    from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, CODED_PITCH_ALIGNED as P, K, N, _declare

    n = a.n
    vp = ctypes.c_void_p
    st = torch.cuda.Stream()
    sp = vp(st.cuda_stream)
    builds = []
    for path in a.libs:
        if path == "default":  # the in-tree library, as in tools/abbench.py
            from decds_amd import build as _build
            path = _build.LIB
        L = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
        _declare(L)
        h = ctypes.c_void_p()
        assert L.decds_ctx_create(0, ctypes.byref(h)) == 0
        builds.append({"tag": os.path.basename(path)[:-3], "lib": L, "ctx": h, "fused": [], "sep": []})
    src = torch.empty(n * CS, dtype=torch.uint8, device="cuda")
    builds[0]["lib"].decds_fill_random_device(builds[0]["ctx"], 5, 0, vp(src.data_ptr()), src.numel(), sp)
    cv = torch.from_numpy(np.random.default_rng(6).integers(0, 256, n * N * K, dtype=np.uint8)).cuda()
    buf = torch.empty(n * N * P + 256, dtype=torch.uint8, device="cuda")
    off = (16 - buf.data_ptr()) % 128
    coded = buf[off:]
    dig = torch.empty(n * N * 32, dtype=torch.uint8, device="cuda")
    roots = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    proofs = torch.empty(n * N * 128, dtype=torch.uint8, device="cuda")
    ws = torch.empty(max(b["lib"].decds_encode_commit_workspace_bytes(n) for b in builds), dtype=torch.uint8, device="cuda")
    ptrs = [vp(t.data_ptr()) for t in (src, cv, coded, dig, roots, proofs, ws)]

    def fused(b):
        assert b["lib"].decds_encode_commit_batch(b["ctx"], ptrs[0], n, ptrs[1], ptrs[2], P, 0, ptrs[3], ptrs[4], ptrs[5],
                                                  ptrs[6], sp) == 0

    def sep(b):
        assert b["lib"].decds_encode_batch(b["ctx"], ptrs[0], n, ptrs[1], ptrs[2], P, sp) == 0
        assert b["lib"].decds_commit_batch(b["ctx"], ptrs[2], P, n, 0, ptrs[3], ptrs[4], ptrs[5], sp) == 0

    ref = None
    for b in ([] if a.no_check else builds):
        fused(b)
        st.synchronize()
        r = roots.clone()
        sep(b)
        st.synchronize()
        assert torch.equal(r, roots), b["tag"] + ": fused roots differ from the separate kernels'"
        if ref is None:
            ref = r
        assert torch.equal(ref, r), b["tag"] + ": roots differ from the first build's"
    t0 = time.time()
    while time.time() - t0 < a.warmup_s:
        for b in builds:
            fused(b)
            sep(b)
        st.synchronize()
    for r in range(a.rounds):
        for b in (builds if r % 2 == 0 else builds[::-1]):
            for kind, fn in (("fused", fused), ("sep", sep)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                fn(b)
                e1.record(st)
                st.synchronize()
                b[kind].append(e0.elapsed_time(e1))
    for b in builds:
        f, s = np.median(b["fused"]), np.median(b["sep"])
        print(json.dumps({"tag": b["tag"], "n": n, "fused_ms": round(float(f), 4), "separate_ms": round(float(s), 4),
                          "fused_blob_GiBps": round(n * CS / 2 ** 30 / (f * 1e-3), 1)}), flush=True)


if __name__ == "__main__":
    main()

"""Per-workgroup phase timeline of a small repair from a DECDS_PHASE_TRACE build: the fused plan + decode
(rlnc_plan_decode_kernel) against the plan kernel then the one-tile decode (rlnc_decode_kernel). Wave 0 of
each workgroup stamps the 100 MHz real-time counter (slots: 0 entry, 1 coding vectors in and plan tables
built, 2 plan's fast path done, 3 plan in LDS for the workgroup, 4 decode tables built, 5 lookups and stores
issued, 6 stores drained). One JSON line per (form, n, run): per slot the 0 / 50 / 100th percentiles over
workgroups in µs from the earliest entry.

build: python -c "from decds_amd import build as b; b.build(force=True, defines=['DECDS_PHASE_TRACE=1'], out='tools/bin/lib_ptrace.so')"
usage: DECDS_LIB=$PWD/tools/bin/lib_ptrace.so python tools/repair_phases.py --sizes 1,2"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PT_WGS, PT_SLOTS = 8192, 32


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,2")
    ap.add_argument("--runs", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch
    import decds_amd
    from decds_amd import codec
    from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N, lib

    L = lib()
    L.decds_debug_phase_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
    sizes = [int(x) for x in a.sizes.split(",")]
    nmax = max(sizes)
    ctx = decds_amd.Context(0)
    st = torch.cuda.Stream()
    src = torch.empty(nmax * CS, dtype=torch.uint8, device="cuda")
    codec.fill_random_device(ctx, 7, src, stream=st)
    cv = torch.from_numpy(codec.fill_random_host(8, nmax * N * K)).cuda()
    coded = torch.empty(nmax * N * F, dtype=torch.uint8, device="cuda")
    codec.encode_batch(ctx, src, nmax, cv, coded, stream=st)
    rng = np.random.default_rng(3)
    cand = np.full((nmax, N), 0xFF, np.uint8)
    for c in range(nmax):
        cand[c, :K] = rng.permutation(N)[:K]
    cand = torch.from_numpy(cand).cuda()
    plan = torch.empty(nmax * 128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(nmax * N, dtype=torch.int8, device="cuda")
    status = torch.empty(nmax, dtype=torch.int32, device="cuda")
    out = torch.empty(nmax * CS, dtype=torch.uint8, device="cuda")
    buf = np.zeros(PT_WGS * PT_SLOTS, dtype=np.uint64)
    forms = {
        "fused": lambda n: codec.repair_batch(ctx, coded, n, cand, plan, verd, out, status, stream=st),
        "plan+decode": lambda n: (codec.repair_plan_batch(ctx, coded, n, cand, plan, verd, status, stream=st),
                                  codec.decode_batch(ctx, coded, n, plan, out, status, stream=st)),
    }
    L.decds_tuning(b"DECDS_PLAN_DECODE_MAX_N", 1 << 62, 1)
    for n in sizes:
        for form, fn in forms.items():
            for _ in range(30):
                fn(n)
            st.synchronize()
            for run in range(a.runs):
                assert L.decds_debug_phase_trace(None, 1) == 0
                torch.cuda.synchronize()
                fn(n)
                st.synchronize()
                assert L.decds_debug_phase_trace(buf.ctypes.data, 0) == 0
                wgs = n * 256
                t = buf[: wgs * PT_SLOTS].reshape(wgs, PT_SLOTS).astype(np.int64)
                ent = t[:, 0]
                t0 = ent[ent > 0].min()
                res = {"form": form, "n": n, "run": run, "status_ok": int((status[:n] == 0).sum().item())}
                for slot in range(7):
                    v = t[:, slot]
                    v = v[v > 0]
                    if len(v):
                        res["s%d" % slot] = [round((float(x) - t0) / 100.0, 2) for x in np.percentile(v, (0, 50, 100))]
                print(json.dumps(res), flush=True)
    L.decds_tuning(b"DECDS_PLAN_DECODE_MAX_N", (1 << 64) - 1, 1)


if __name__ == "__main__":
    main()

"""ChunkSet::new for a batch as two overlapped kernels: the encode of sub-batch i+1 (HBM-bound) runs
beside the commitment of sub-batch i (VALU-bound) on a second stream, against the fused kernel
(decds_encode_commit_batch) and the two kernels back to back. Roots are checked against the
back-to-back form. One JSON line per sub-batch size.

usage: python tools/pipecommit.py --n 103 --subs 103,52,26,13,8
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
    ap.add_argument("--subs", default="103,52,35,26,13,8")
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--priority", action="store_true", help="commitment stream at high priority")
    a = ap.parse_args()
    import numpy as np
    import torch
    from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PITCH_ALIGNED as P, K, N, lib
    import decds_amd

    L = lib()
    n = a.n
    vp = ctypes.c_void_p
    ctx = decds_amd.Context(0)
    h = ctx._h
    sa = torch.cuda.Stream()
    sb = torch.cuda.Stream(priority=-1) if a.priority else torch.cuda.Stream()
    src = torch.empty(n * CS, dtype=torch.uint8, device="cuda")
    L.decds_fill_random_device(h, 5, 0, vp(src.data_ptr()), src.numel(), vp(sa.cuda_stream))
    cv = torch.from_numpy(np.random.default_rng(6).integers(0, 256, n * N * K, dtype=np.uint8)).cuda()
    buf = torch.empty(n * N * P + 256, dtype=torch.uint8, device="cuda")
    off = (16 - buf.data_ptr()) % 128
    coded = buf[off:]
    dig = torch.empty(n * N * 32, dtype=torch.uint8, device="cuda")
    roots = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    proofs = torch.empty(n * N * 128, dtype=torch.uint8, device="cuda")
    ws = torch.empty(L.decds_encode_commit_workspace_bytes(n), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()

    def enc(lo, hi, st):
        assert L.decds_encode_batch(h, vp(src.data_ptr() + lo * CS), hi - lo, vp(cv.data_ptr() + lo * N * K),
                                    vp(coded.data_ptr() + lo * N * P), P, vp(st.cuda_stream)) == 0

    def com(lo, hi, st):
        assert L.decds_commit_batch(h, vp(coded.data_ptr() + lo * N * P), P, hi - lo, lo, vp(dig.data_ptr() + lo * N * 32),
                                    vp(roots.data_ptr() + lo * 32), vp(proofs.data_ptr() + lo * N * 128),
                                    vp(st.cuda_stream)) == 0

    def fused():
        assert L.decds_encode_commit_batch(h, vp(src.data_ptr()), n, vp(cv.data_ptr()), vp(coded.data_ptr()), P, 0,
                                           vp(dig.data_ptr()), vp(roots.data_ptr()), vp(proofs.data_ptr()),
                                           vp(ws.data_ptr()), vp(sa.cuda_stream)) == 0

    def piped(S):
        for lo in range(0, n, S):
            hi = min(n, lo + S)
            enc(lo, hi, sa)
            e = torch.cuda.Event()
            e.record(sa)
            sb.wait_event(e)
            com(lo, hi, sb)
        sa.wait_stream(sb)

    enc(0, n, sa)
    com(0, n, sa)
    sa.synchronize()
    ref = roots.clone()

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        sa.synchronize()
        sb.synchronize()
        e0.record(sa)
        sb.wait_event(e0)
        fn()
        e1.record(sa)
        sa.synchronize()
        return e0.elapsed_time(e1)

    subs = [int(s) for s in a.subs.split(",")]
    t0 = time.time()
    while time.time() - t0 < 1.5:
        for S in subs:
            timed(lambda: piped(S))
        timed(fused)
    res = {S: [] for S in subs}
    res["fused"] = []
    for _ in range(a.rounds):
        for S in subs:
            roots.zero_()
            torch.cuda.synchronize()
            res[S].append(timed(lambda: piped(S)))
            assert torch.equal(roots, ref), f"sub-batch {S}: roots differ"
        res["fused"].append(timed(fused))
        assert torch.equal(roots, ref), "fused roots differ"
    for k, v in res.items():
        print(json.dumps({"n": n, "sub_batch": k, "priority": a.priority, "ms": round(float(np.median(v)), 4),
                          "min_ms": round(float(np.min(v)), 4)}), flush=True)


if __name__ == "__main__":
    main()

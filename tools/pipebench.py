"""ChunkSet::new over a batch = encode + commitment (chunkset.rs:37-69). Times the two kernels
back to back on one stream against a two-stream pipeline over sub-batches (encode of sub-batch
k+1 beside the commitment of sub-batch k): encode is HBM-bound, the BLAKE3 digest VALU-bound, so
they can share the chip. Prints one JSON line.
usage: python tools/pipebench.py --n 103 --parts 4 --reps 10"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=103)
    ap.add_argument("--parts", type=int, default=4)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import numpy as np
    import torch
    import decds_amd
    from decds_amd import codec
    from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N
    ctx = decds_amd.Context(0)
    n = a.n
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    src = torch.empty(n * CS, dtype=torch.uint8, device="cuda")
    codec.fill_random_device(ctx, 1, src, stream=s1)
    coeffs = torch.from_numpy(codec.fill_random_host(2, n * N * K)).cuda()
    coded = torch.empty(n * N * F, dtype=torch.uint8, device="cuda")
    dig = torch.empty(n * N * 32, dtype=torch.uint8, device="cuda")
    roots = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    proofs = torch.empty(n * N * 128, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    bounds = [n * p // a.parts for p in range(a.parts + 1)]

    def views(lo, hi):
        return (src[lo * CS:hi * CS], coeffs[lo * N * K:hi * N * K], coded[lo * N * F:hi * N * F],
                dig[lo * N * 32:hi * N * 32], roots[lo * 32:hi * 32], proofs[lo * N * 128:hi * N * 128])

    def sequential():
        codec.encode_batch(ctx, src, n, coeffs, coded, stream=s1)
        codec.commit_batch(ctx, coded, n, dig, roots, proofs, stream=s1)

    def pipelined():
        evs = []
        for p in range(a.parts):
            lo, hi = bounds[p], bounds[p + 1]
            sv, cv, co, dg, rt, pf = views(lo, hi)
            codec.encode_batch(ctx, sv, hi - lo, cv, co, stream=s1)
            e = torch.cuda.Event()
            e.record(s1)
            evs.append(e)
        for p in range(a.parts):
            lo, hi = bounds[p], bounds[p + 1]
            sv, cv, co, dg, rt, pf = views(lo, hi)
            s2.wait_event(evs[p])
            codec.commit_batch(ctx, co, hi - lo, dg, rt, pf, first_chunkset_id=lo, stream=s2)
        s1.wait_stream(s2)

    def timed(fn):
        ts = []
        for r in range(a.reps + 2):
            torch.cuda.synchronize()
            b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            b.record(s1)
            s2.wait_event(b)
            fn()
            e.record(s1)
            torch.cuda.synchronize()
            if r >= 2:
                ts.append(b.elapsed_time(e))
        return float(np.median(ts))

    t_seq = timed(sequential)
    ref = (dig.clone(), roots.clone(), proofs.clone())
    t_pipe = timed(pipelined)
    same = all(torch.equal(x, y) for x, y in zip(ref, (dig, roots, proofs)))
    print(json.dumps({"n": n, "parts": a.parts, "sequential_ms": round(t_seq, 4), "pipelined_ms": round(t_pipe, 4),
                      "speedup": round(t_seq / t_pipe, 3), "build_GiBps_seq": round(n * CS / (1 << 30) / t_seq * 1e3, 1),
                      "build_GiBps_pipe": round(n * CS / (1 << 30) / t_pipe * 1e3, 1), "results_equal": same}))


if __name__ == "__main__":
    main()

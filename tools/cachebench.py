"""Encode + repair of one batch as S sequential sub-batches on ONE stream (encode k, plan k, decode k,
then k+1), so that decode k re-reads coded rows that encode k wrote a moment earlier: with sub-batches
small enough, those rows may still sit in the memory-side Infinity Cache (MALL) and decode's reads
leave DRAM alone. Prints one JSON line per S: median step time over rounds, per-kernel-type sums
from HIP events, and the repaired-data check.

usage: python tools/cachebench.py --n 103 --subs 1 2 4 8 13
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=103)
    ap.add_argument("--subs", type=int, nargs="+", default=[1, 2, 4, 8, 13])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    import numpy as np
    import torch
    import decds_amd
    from decds_amd import codec
    from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N

    n = a.n
    ctx = decds_amd.Context(0)
    s0 = torch.cuda.Stream()
    src = torch.empty(n * CS, dtype=torch.uint8, device="cuda")
    codec.fill_random_device(ctx, 0xDEC05002, src, stream=s0)
    coeffs = torch.from_numpy(codec.fill_random_host(0xC0EF0002, n * N * K)).cuda()
    rng = np.random.default_rng(0x5EED0002)
    cand_h = np.full((n, N), 0xFF, np.uint8)
    for c in range(n):
        cand_h[c, :K] = rng.permutation(N)[:K]
    cand = torch.from_numpy(cand_h).cuda()
    coded = torch.empty(n * N * F, dtype=torch.uint8, device="cuda")
    plan = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(n * N, dtype=torch.int8, device="cuda")
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    out = torch.empty(n * CS, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()

    def parts(S):
        b = [n * k // S for k in range(S + 1)]
        return [(b[k], b[k + 1] - b[k]) for k in range(S)]

    def step(S, ev=None):
        for k, (c0, m) in enumerate(parts(S)):
            if ev is not None:
                ev[k][0].record(s0)
            codec.encode_batch(ctx, src[c0 * CS:], m, coeffs[c0 * N * K:], coded[c0 * N * F:], stream=s0)
            if ev is not None:
                ev[k][1].record(s0)
            codec.repair_plan_batch(ctx, coded[c0 * N * F:], m, cand[c0:], plan[c0 * 128:], verd[c0 * N:],
                                    status[c0:], stream=s0)
            if ev is not None:
                ev[k][2].record(s0)
            codec.decode_batch(ctx, coded[c0 * N * F:], m, plan[c0 * 128:], out[c0 * CS:], status[c0:], stream=s0)
            if ev is not None:
                ev[k][3].record(s0)

    # clock settle
    t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t[0].record(s0)
    for _ in range(400):
        step(1)
    t[1].record(s0)
    s0.synchronize()
    res = {S: [] for S in a.subs}
    split = {S: [] for S in a.subs}
    for _ in range(a.rounds):
        for S in a.subs:
            for _ in range(3):
                step(S)
            b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            b[0].record(s0)
            for _ in range(a.steps):
                step(S)
            b[1].record(s0)
            ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(S)]
            step(S, ev)
            s0.synchronize()
            res[S].append(b[0].elapsed_time(b[1]) / a.steps)
            split[S].append([sum(e[i].elapsed_time(e[i + 1]) for e in ev) for i in range(3)])
    st = status.cpu().numpy()
    ok = all(torch.equal(out[c * CS:(c + 1) * CS], src[c * CS:(c + 1) * CS]) for c in np.nonzero(st == 0)[0].tolist())
    for S in a.subs:
        ms = statistics.median(res[S])
        sp = [round(statistics.median(x[i] for x in split[S]), 4) for i in range(3)]
        print(json.dumps({"n": n, "subs": S, "step_ms": round(ms, 4), "min_ms": round(min(res[S]), 4),
                          "encode_ms": sp[0], "plan_ms": sp[1], "decode_ms": sp[2],
                          "blob_GiBps": round(n * CS / 2**30 / (ms * 1e-3), 1), "repair_ok": ok}), flush=True)


if __name__ == "__main__":
    main()

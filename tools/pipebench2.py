"""Encode + repair of one batch, sequential on one stream against pipelined over S sub-batches on two
streams (stream 0 encodes sub-batch k while stream 1 plans and decodes sub-batch k-1, joined by
events), so one kernel's ramp-down and the launch gaps overlap the next kernel's work. Prints one
JSON line per S: median step time over rounds, and the repaired data check.

usage: python tools/pipebench2.py --n 103 --subs 1 2 3 4 --steps 20
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=103)
    ap.add_argument("--subs", type=int, nargs="+", default=[1, 2, 3, 4])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--events", type=int, nargs="+", default=[0],
                    help="sequential steps with 0 / 2 (around encode) / 4 timing events per step")
    a = ap.parse_args()
    import numpy as np
    import torch
    import decds_amd
    from decds_amd import codec
    from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N

    n = a.n
    ctx = decds_amd.Context(0)
    s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
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

    def step(S, nev=0):
        if S == 1:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(nev)]
            if nev:
                ev[0].record(s0)
            codec.encode_batch(ctx, src, n, coeffs, coded, stream=s0)
            if nev:
                ev[1].record(s0)
            codec.repair_plan_batch(ctx, coded, n, cand, plan, verd, status, stream=s0)
            if nev == 4:
                ev[2].record(s0)
            codec.decode_batch(ctx, coded, n, plan, out, status, stream=s0)
            if nev == 4:
                ev[3].record(s0)
            return
        for c0, m in parts(S):
            codec.encode_batch(ctx, src[c0 * CS:], m, coeffs[c0 * N * K:], coded[c0 * N * F:], stream=s0)
            ev = torch.cuda.Event()
            ev.record(s0)
            s1.wait_event(ev)
            codec.repair_plan_batch(ctx, coded[c0 * N * F:], m, cand[c0:], plan[c0 * 128:], verd[c0 * N:],
                                    status[c0:], stream=s1)
            codec.decode_batch(ctx, coded[c0 * N * F:], m, plan[c0 * 128:], out[c0 * CS:], status[c0:], stream=s1)
        ev = torch.cuda.Event()
        ev.record(s1)
        s0.wait_event(ev)

    cfgs = [(S, 0) for S in a.subs if S > 1] + [(1, e) for e in a.events]
    res = {c: [] for c in cfgs}
    for c in cfgs:  # warm-up
        for _ in range(3):
            step(*c)
    torch.cuda.synchronize()
    for r in range(a.rounds):
        for c in (cfgs if r % 2 == 0 else cfgs[::-1]):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step(*c)
            torch.cuda.synchronize()
            res[c].append((time.perf_counter() - t0) / a.steps * 1e3)
    st = status.cpu().numpy()
    ok = all(torch.equal(out[c * CS:(c + 1) * CS], src[c * CS:(c + 1) * CS]) for c in np.nonzero(st == 0)[0].tolist())
    for (S, e) in cfgs:
        ms = float(np.median(res[(S, e)]))
        print(json.dumps({"n": n, "sub_batches": S, "events_per_step": e, "ms_per_step": round(ms, 4),
                          "GiBps": round(n * CS / 2**30 / (ms * 1e-3), 1), "repaired_ok": ok}), flush=True)


if __name__ == "__main__":
    main()

"""Step pipelining across consecutive encode+repair steps: stream A encodes step s+1 into the other
of two coded buffers while stream B plans and decodes step s (events order encode(s) -> plan(s) and
decode(s-1) -> encode(s+1), the coded buffer's last reader). Full-size launches only, so the gain
can only come from one kernel's ramp-up / drain overlapping the other's. Against the sequential
one-stream step, and against S independent sub-batch streams (split2/3/4: each stream its own
encode -> plan -> decode chain, as S processes sharing the card). Prints one JSON line per mode.

usage: python tools/overlapbench.py --n 103 --steps 40 --rounds 5
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
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--graph", action="store_true", help="sequential steps against one step captured as a HIP graph")
    a = ap.parse_args()
    import numpy as np
    import torch
    import decds_amd
    from decds_amd import codec
    from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N

    n = a.n
    ctx = decds_amd.Context(0)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    src = torch.empty(n * CS, dtype=torch.uint8, device="cuda")
    codec.fill_random_device(ctx, 0xDEC05002, src, stream=sa)
    coeffs = torch.from_numpy(codec.fill_random_host(0xC0EF0002, n * N * K)).cuda()
    rng = np.random.default_rng(0x5EED0002)
    cand_h = np.full((n, N), 0xFF, np.uint8)
    for c in range(n):
        cand_h[c, :K] = rng.permutation(N)[:K]
    cand = torch.from_numpy(cand_h).cuda()
    coded = [torch.empty(n * N * F, dtype=torch.uint8, device="cuda") for _ in range(2)]
    plan = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(n * N, dtype=torch.int8, device="cuda")
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    out = torch.empty(n * CS, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()

    def run_seq(k):
        for _ in range(k):
            codec.encode_batch(ctx, src, n, coeffs, coded[0], stream=sa)
            codec.repair_plan_batch(ctx, coded[0], n, cand, plan, verd, status, stream=sa)
            codec.decode_batch(ctx, coded[0], n, plan, out, status, stream=sa)

    def run_pipe(k):
        enc_done = [torch.cuda.Event() for _ in range(k)]
        dec_done = [torch.cuda.Event() for _ in range(k)]
        sb.wait_stream(sa)
        for s in range(k):
            c = coded[s % 2]
            if s >= 2:
                sa.wait_event(dec_done[s - 2])  # coded[s % 2]'s last reader
            codec.encode_batch(ctx, src, n, coeffs, c, stream=sa)
            enc_done[s].record(sa)
            sb.wait_event(enc_done[s])
            codec.repair_plan_batch(ctx, c, n, cand, plan, verd, status, stream=sb)
            codec.decode_batch(ctx, c, n, plan, out, status, stream=sb)
            dec_done[s].record(sb)
        sa.wait_stream(sb)

    streams = [torch.cuda.Stream() for _ in range(4)]

    def run_split(S, k):
        # S independent sub-batches, each on its own stream with its own encode -> plan -> decode
        # chain (as S processes sharing the card would issue them); no cross-stream waits
        b = [n * j // S for j in range(S + 1)]
        for st in streams[:S]:
            st.wait_stream(sa)
        for _ in range(k):
            for j in range(S):
                c0, m, st = b[j], b[j + 1] - b[j], streams[j]
                codec.encode_batch(ctx, src[c0 * CS:], m, coeffs[c0 * N * K:], coded[0][c0 * N * F:], stream=st)
                codec.repair_plan_batch(ctx, coded[0][c0 * N * F:], m, cand[c0:], plan[c0 * 128:], verd[c0 * N:],
                                        status[c0:], stream=st)
                codec.decode_batch(ctx, coded[0][c0 * N * F:], m, plan[c0 * 128:], out[c0 * CS:], status[c0:],
                                   stream=st)
        for st in streams[:S]:
            sa.wait_stream(st)

    def timed(fn):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(sa)
        fn(a.steps)
        e1.record(sa)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.steps

    for _ in range(40):
        run_seq(10)
        run_pipe(10)
    torch.cuda.synchronize()
    # one step captured as a HIP graph (the three launches), replayed per step
    graph = None
    if a.graph:
        gs = torch.cuda.Stream()
        gs.wait_stream(sa)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=gs):
            codec.encode_batch(ctx, src, n, coeffs, coded[0], stream=gs)
            codec.repair_plan_batch(ctx, coded[0], n, cand, plan, verd, status, stream=gs)
            codec.decode_batch(ctx, coded[0], n, plan, out, status, stream=gs)
        torch.cuda.synchronize()

    def run_graph(k):
        with torch.cuda.stream(sa):
            for _ in range(k):
                graph.replay()

    fns = {"seq": run_seq, "pipe": run_pipe, "split2": lambda k: run_split(2, k),
           "split3": lambda k: run_split(3, k), "split4": lambda k: run_split(4, k)}
    if a.graph:
        fns = {"seq": run_seq, "graph": run_graph}
    for _ in range(10):
        for f in fns.values():
            f(4)
    res = {m: [] for m in fns}
    for r in range(a.rounds):
        for m in (list(fns) if r % 2 == 0 else list(fns)[::-1]):
            res[m].append(timed(fns[m]))
    st = status.cpu().numpy()
    ok = all(torch.equal(out[c * CS:(c + 1) * CS], src[c * CS:(c + 1) * CS]) for c in np.nonzero(st == 0)[0].tolist())
    for m, v in res.items():
        ms = statistics.median(v)
        print(json.dumps({"n": n, "mode": m, "step_ms": round(ms, 4), "min_ms": round(min(v), 4),
                          "blob_GiBps": round(n * CS / 2**30 / (ms * 1e-3), 1), "repair_ok": ok}), flush=True)


if __name__ == "__main__":
    main()

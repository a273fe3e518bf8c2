"""Kernel-level timing of one library build (DECDS_LIB selects a variant .so): encode, plan and
decode launches on one stream, HIP events per launch, median over reps. Prints one JSON line.
usage: DECDS_LIB=build/variants/lib_X.so python tools/kbench.py --n 103 --reps 20 --tag X"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=103)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tag", default=os.path.basename(os.environ.get("DECDS_LIB", "default")))
    ap.add_argument("--pitch", type=int, default=0)
    ap.add_argument("--dst-off", type=int, default=0, help="byte offset of the coded buffer (alignment study)")
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--commit", action="store_true", help="also time decds_commit_batch (BLAKE3 + Merkle)")
    ap.add_argument("--repair", action="store_true",
                    help="also time decds_repair_batch (plan + decode in one call; one launch up to "
                         "DECDS_PLAN_DECODE_MAX_N chunksets, rlnc_plan_decode_kernel)")
    a = ap.parse_args()
    import numpy as np
    import torch
    import decds_amd
    from decds_amd import codec
    from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N
    ctx = decds_amd.Context(0)
    n, pitch = a.n, a.pitch or F
    st = torch.cuda.Stream()
    src = torch.empty(n * CS, dtype=torch.uint8, device="cuda")
    codec.fill_random_device(ctx, 1, src, stream=st)
    coeffs = torch.from_numpy(codec.fill_random_host(2, n * N * K)).cuda()
    rng = np.random.default_rng(3)
    cand = np.full((n, N), 0xFF, np.uint8)
    for c in range(n):
        cand[c, :K] = rng.permutation(N)[:K]
    cand = torch.from_numpy(cand).cuda()
    coded_buf = torch.empty((n * N - 1) * pitch + F + a.dst_off, dtype=torch.uint8, device="cuda")
    coded = coded_buf[a.dst_off:]
    plan = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(n * N, dtype=torch.int8, device="cuda")
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    out = torch.empty(n * CS, dtype=torch.uint8, device="cuda")
    if a.commit:
        dig = torch.empty(n * N * 32, dtype=torch.uint8, device="cuda")
        roots = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
        proofs = torch.empty(n * N * 128, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(6)] for _ in range(a.reps + 3)]
    for r in range(a.reps + 3):
        e = ev[r]
        e[0].record(st)
        codec.encode_batch(ctx, src, n, coeffs, coded, pitch, stream=st)
        e[1].record(st)
        codec.repair_plan_batch(ctx, coded, n, cand, plan, verd, status, pitch, stream=st)
        e[2].record(st)
        codec.decode_batch(ctx, coded, n, plan, out, status, pitch, stream=st)
        e[3].record(st)
        if a.commit:
            codec.commit_batch(ctx, coded, n, dig, roots, proofs, pitch=pitch, stream=st)
            e[4].record(st)
        if a.repair:
            if not a.commit:  # (with --commit, e[4] already marks the commit's end)
                e[4].record(st)
            codec.repair_batch(ctx, coded, n, cand, plan, verd, out, status, pitch, stream=st)
            e[5].record(st)
    torch.cuda.synchronize()
    t = np.array([[e[0].elapsed_time(e[1]), e[1].elapsed_time(e[2]), e[2].elapsed_time(e[3])] for e in ev[3:]])
    med = np.median(t, axis=0)
    s = status.cpu().numpy()
    nr = int((s == 0).sum())
    res = {"tag": a.tag, "n": n, "pitch": pitch, "dst_off": a.dst_off, "encode_ms": round(med[0], 4), "plan_ms": round(med[1], 4),
           "decode_ms": round(med[2], 4),
           "encode_GBps": round(n * (CS + N * F) / med[0] / 1e6, 1),
           "decode_GBps": round(nr * (K * F + CS) / med[2] / 1e6, 1),
           "encode_min_ms": round(t[:, 0].min(), 4), "decode_min_ms": round(t[:, 2].min(), 4)}
    if a.commit:
        tc = np.array([e[3].elapsed_time(e[4]) for e in ev[3:]])
        res["commit_ms"] = round(float(np.median(tc)), 4)
        res["commit_GBps"] = round(n * N * F / res["commit_ms"] / 1e6, 1)
    if a.repair:
        from decds_amd._capi import lib
        tr = np.array([e[4].elapsed_time(e[5]) for e in ev[3:]])
        res["repair_ms"] = round(float(np.median(tr)), 4)
        res["repair_kernel"] = lib().decds_repair_kernel_name(n).decode()
    if a.check:
        good = True
        for c in np.nonzero(s == 0)[0].tolist():
            good &= bool(torch.equal(out[c * CS:(c + 1) * CS], src[c * CS:(c + 1) * CS]))
        res["roundtrip_ok"] = good
        if a.commit:  # spot-check digests of a few rows against the CPU restatement
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as o
            d = dig.cpu().numpy()
            ok = True
            for row in sorted({0, 1, 17, n * N - 1}):
                piece = coded[row * pitch:row * pitch + F].cpu().numpy()
                ok &= d[row * 32:(row + 1) * 32].tobytes() == o.chunk_digest(row // N, row, piece)
            res["digest_ok"] = ok
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

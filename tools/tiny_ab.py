"""In-process A/B of small-batch kernel forms as bench.py's sweep times them: per round and knob value,
0.2 s of warm launches, then `reps` launches each between its own torch events (recorded back to back, one
synchronize), the median; rounds alternate between the knob set to 0 and to 2^30. Forms: encode (--enc-knob,
default DECDS_ENC_SMALL_MAX_N), decode and the fused repair (--dec-knob, default DECDS_DEC_NARROW_MAX_N), on
chunkset 0 of an n_alloc-chunkset aligned layout. One JSON line per (form, knob value). (Round 6 used it
with the 4-column one-chunkset forms' knobs, DECDS_ENC_TINY_MAX_N / DECDS_DEC_TINY_MAX_N, since removed:
profiles/r09zj_tiny_forms_ab.jsonl.)

usage: python tools/tiny_ab.py [--n 1] [--rounds 6] [--reps 20] [--n-alloc 64] [--enc-knob K] [--dec-knob K]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--n-alloc", type=int, default=64)
    ap.add_argument("--enc-knob", default="DECDS_ENC_SMALL_MAX_N")
    ap.add_argument("--dec-knob", default="DECDS_DEC_NARROW_MAX_N")
    a = ap.parse_args()
    ek, dk = a.enc_knob.encode(), a.dec_knob.encode()
    import numpy as np
    import torch
    import decds_amd
    from decds_amd import codec
    from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N, lib

    L = lib()
    n, na = a.n, max(a.n, a.n_alloc)
    ctx = decds_amd.Context(0)
    st = torch.cuda.Stream()
    src = torch.empty(na * CS, dtype=torch.uint8, device="cuda")
    codec.fill_random_device(ctx, 7, src, stream=st)
    cv = torch.from_numpy(codec.fill_random_host(8, na * N * K)).cuda()
    dst, pitch = codec.coded_buffer(na)
    rng = np.random.default_rng(3)
    cand = np.full((n, N), 0xFF, np.uint8)
    for c in range(n):
        cand[c, :K] = rng.permutation(N)[:K]
    cand = torch.from_numpy(cand).cuda()
    plan = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(n * N, dtype=torch.int8, device="cuda")
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    out = torch.empty(n * CS, dtype=torch.uint8, device="cuda")
    codec.encode_batch(ctx, src, n, cv, dst, pitch, stream=st)
    codec.repair_plan_batch(ctx, dst, n, cand, plan, verd, status, pitch, stream=st)
    st.synchronize()
    forms = {
        "encode": (ek, lambda: codec.encode_batch(ctx, src, n, cv, dst, pitch, stream=st),
                   n * (CS + N * F)),
        "decode": (dk, lambda: codec.decode_batch(ctx, dst, n, plan, out, status, pitch, stream=st),
                   n * (K * F + CS)),
        "repair_fused": (dk,
                         lambda: codec.repair_batch(ctx, dst, n, cand, plan, verd, out, status, pitch, stream=st),
                         n * (K * F + CS)),
    }
    res = {}
    for r in range(a.rounds):
        for form, (knob, fn, byts) in forms.items():
            for val in ((0, 1 << 30) if r % 2 == 0 else (1 << 30, 0)):
                L.decds_tuning(knob, val, 1)
                t_w = time.perf_counter()
                while time.perf_counter() - t_w < 0.2:
                    for _ in range(4):
                        fn()
                    st.synchronize()
                ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(a.reps)]
                for e in ev:
                    e[0].record(st)
                    fn()
                    e[1].record(st)
                st.synchronize()
                res.setdefault((form, val), []).append(float(np.median([x.elapsed_time(y) for x, y in ev])))
    for k in (ek, dk):
        L.decds_tuning(k, (1 << 64) - 1, 1)
    for (form, val), ms in sorted(res.items()):
        byts = forms[form][2]
        med = float(np.median(ms))
        print(json.dumps({"form": form, "n": n, "knob": (ek if form == "encode" else dk).decode(), "knob_on": val != 0, "ms_median_of_rounds": round(med, 5),
                          "ms_rounds": [round(x, 5) for x in ms], "frac": round(byts / (med * 1e-3) / 8e12, 4)}))


if __name__ == "__main__":
    main()

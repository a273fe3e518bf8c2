"""Where a small encode batch's time goes: per batch size, the median of single launches each bracketed
by its own HIP events (bench.py's encode_batch_sweep) against back-to-back launches between two
events (the dispatch latency of all but the first launch hidden behind the previous kernel), for both
encode forms (DECDS_ENC_SMALL_MAX_N). Prints one JSON line per (form, n).

usage: python tools/smallbatch.py [--sizes 1,2,4,8,16,32,64]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,2,4,8,16,32,64")
    ap.add_argument("--reps", type=int, default=40)
    a = ap.parse_args()
    import numpy as np
    import torch
    import decds_amd
    from decds_amd import codec
    from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N, lib

    sizes = [int(x) for x in a.sizes.split(",")]
    nmax = max(sizes)
    ctx = decds_amd.Context(0)
    st = torch.cuda.Stream()
    src = torch.empty(nmax * CS, dtype=torch.uint8, device="cuda")
    codec.fill_random_device(ctx, 7, src, stream=st)
    cv = torch.from_numpy(codec.fill_random_host(8, nmax * N * K)).cuda()
    dst, pitch = codec.coded_buffer(nmax)
    st.synchronize()
    for form, knob in (("cols16", 0), ("cols8", 1 << 30)):
        lib().decds_tuning(b"DECDS_ENC_SMALL_MAX_N", knob, 1)
        for n in sizes:
            for _ in range(50):
                codec.encode_batch(ctx, src, n, cv, dst, pitch, stream=st)
            st.synchronize()
            single = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                codec.encode_batch(ctx, src, n, cv, dst, pitch, stream=st)
                e1.record(st)
                st.synchronize()
                single.append(e0.elapsed_time(e1))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.reps):
                codec.encode_batch(ctx, src, n, cv, dst, pitch, stream=st)
            e1.record(st)
            st.synchronize()
            b2b = e0.elapsed_time(e1) / a.reps
            ms = float(np.median(single))
            byts = n * (CS + N * F)
            print(json.dumps({"form": form, "n": n, "single_ms": round(ms, 4), "back_to_back_ms": round(b2b, 4),
                              "single_frac": round(byts / (ms * 1e-3) / 8e12, 4),
                              "back_to_back_frac": round(byts / (b2b * 1e-3) / 8e12, 4)}), flush=True)
    lib().decds_tuning(b"DECDS_ENC_SMALL_MAX_N", (1 << 64) - 1, 1)


if __name__ == "__main__":
    main()

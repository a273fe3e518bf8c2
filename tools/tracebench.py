"""Per-wave timeline of the codec kernels from a DECDS_TIMING_TRACE build: start / end stamps of every
wave (100 MHz real-time counter) for one encode and one decode launch, summarised as start skew,
end-time percentiles and the tail (how long the last waves run after the median wave ended).
usage: python tools/tracebench.py build/ab/lib_trace.so --n 103"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


TRACE_WAVES = 65536


def summarise(st, n_waves):
    import numpy as np
    s = st.reshape(-1, 2)[:n_waves].astype(np.int64)
    s = s[(s[:, 0] > 0) & (s[:, 1] > 0)]
    n_waves = len(s)
    t0 = s[:, 0].min()
    start, end = (s[:, 0] - t0) / 100.0, (s[:, 1] - t0) / 100.0   # microseconds
    q = np.percentile(end, [0, 10, 50, 90, 99, 100])
    # resident waves over time (20 bins over the launch) and per-wave durations
    bins = np.linspace(0, q[5], 21)
    mid = (bins[:-1] + bins[1:]) / 2
    resident = [int(((start <= t) & (end > t)).sum()) for t in mid]
    dur = end - start
    return {"waves": n_waves, "start_max_us": round(float(start.max()), 2),
            "end_us_p0_p10_p50_p90_p99_p100": [round(float(v), 1) for v in q],
            "tail_us": round(float(q[5] - q[2]), 1), "busy_frac": round(float(dur.sum() / (n_waves * q[5])), 3),
            "wave_us_p10_p50_p90": [round(float(v), 1) for v in np.percentile(dur, [10, 50, 90])],
            "first_end_us": round(float(end.min()), 1), "last_start_us": round(float(start.max()), 1),
            "resident_20bins": resident}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--n", type=int, default=103)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--dump", default="", help="save the last run's raw stamps (.npz)")
    a = ap.parse_args()
    import numpy as np
    import torch
    from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N, _declare
    L = ctypes.CDLL(os.path.abspath(a.lib), mode=ctypes.RTLD_LOCAL)
    _declare(L)
    L.decds_debug_trace.argtypes = [ctypes.c_int, ctypes.c_void_p]
    h = ctypes.c_void_p()
    assert L.decds_ctx_create(0, ctypes.byref(h)) == 0
    n, vp = a.n, ctypes.c_void_p
    st = torch.cuda.Stream()
    src = torch.empty(n * CS, dtype=torch.uint8, device="cuda")
    L.decds_fill_random_device(h, 1, 0, vp(src.data_ptr()), src.numel(), vp(st.cuda_stream))
    coeffs = torch.from_numpy(np.random.default_rng(2).integers(0, 256, n * N * K, dtype=np.uint8)).cuda()
    rng = np.random.default_rng(3)
    cand = np.full((n, N), 0xFF, np.uint8)
    for c in range(n):
        cand[c, :K] = rng.permutation(N)[:K]
    cand = torch.from_numpy(cand).cuda()
    coded = torch.empty(n * N * F, dtype=torch.uint8, device="cuda")
    plan = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(n * N, dtype=torch.int8, device="cuda")
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    out = torch.empty(n * CS, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    sp = vp(st.cuda_stream)
    res = {"lib": os.path.basename(a.lib), "n": n, "runs": []}
    for r in range(a.reps):
        assert L.decds_encode_batch(h, vp(src.data_ptr()), n, vp(coeffs.data_ptr()), vp(coded.data_ptr()), F, sp) == 0
        st.synchronize()
        enc = np.zeros(2 * TRACE_WAVES, np.uint64)
        assert L.decds_debug_trace(0, enc.ctypes.data) == 0
        assert L.decds_repair_plan_batch(h, vp(coded.data_ptr()), F, n, vp(cand.data_ptr()), vp(plan.data_ptr()),
                                         vp(verd.data_ptr()), vp(status.data_ptr()), sp) == 0
        assert L.decds_decode_batch(h, vp(coded.data_ptr()), F, n, vp(plan.data_ptr()), vp(out.data_ptr()),
                                    vp(status.data_ptr()), None, sp) == 0
        st.synchronize()
        dec = np.zeros(2 * TRACE_WAVES, np.uint64)
        assert L.decds_debug_trace(1, dec.ctypes.data) == 0
        if r >= 2:
            res["runs"].append({"encode": summarise(enc, TRACE_WAVES), "decode": summarise(dec, TRACE_WAVES)})
    if a.dump:
        np.savez(a.dump, encode=enc, decode=dec)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

"""How much of a small encode batch's event-bracketed time is the timing events' own cost. bench.py's
encode_batch_sweep brackets each launch with a pair of torch events (hipEventCreateWithFlags(0)):
recording one performs a system-scope fence — an L2 writeback and invalidate — that
hipEventDisableSystemFence skips ("can improve the accuracy of timing measurements", hip_runtime_api.h)
and hipEventReleaseToDevice narrows to device scope. Per batch size: the median of single launches
each between its own event pair, recorded back to back on one stream exactly as the sweep does, for
each event kind. Prints one JSON line per (events, n).

usage: python tools/eventbench.py [--sizes 1,2,4,8,16,32,64] [--reps 40]"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KINDS = {"torch default (flags 0)": None, "hipEventDisableSystemFence": 0x20000000,
         "hipEventReleaseToDevice": 0x40000000}


def hip_runtime():
    """the libamdhip64 torch already loaded (the library binds to the same one)"""
    with open("/proc/self/maps") as f:
        paths = sorted({ln.split()[-1] for ln in f if "libamdhip64.so" in ln})
    assert paths, "no HIP runtime mapped"
    return ctypes.CDLL(paths[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,2,4,8,16,32,64")
    ap.add_argument("--reps", type=int, default=40)
    a = ap.parse_args()
    import numpy as np
    import torch
    import decds_amd
    from decds_amd import codec
    from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N

    sizes = [int(x) for x in a.sizes.split(",")]
    nmax = max(sizes)
    ctx = decds_amd.Context(0)
    st = torch.cuda.Stream()
    src = torch.empty(nmax * CS, dtype=torch.uint8, device="cuda")
    codec.fill_random_device(ctx, 7, src, stream=st)
    cv = torch.from_numpy(codec.fill_random_host(8, nmax * N * K)).cuda()
    dst, pitch = codec.coded_buffer(nmax, aligned=True)
    st.synchronize()
    hip = hip_runtime()
    vp = ctypes.c_void_p
    hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
    hip.hipEventRecord.argtypes = [vp, vp]
    hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), vp, vp]
    hip.hipEventDestroy.argtypes = [vp]
    sptr = vp(st.cuda_stream)
    for n in sizes:
        byts = n * (CS + N * F)
        for _ in range(3):  # warm, as the sweep does
            for _ in range(50):
                codec.encode_batch(ctx, src, n, cv, dst, pitch, stream=st)
            st.synchronize()
        for kind, flags in KINDS.items():
            ms = []
            if flags is None:
                ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(a.reps)]
                for r in range(a.reps):
                    ev[r][0].record(st)
                    codec.encode_batch(ctx, src, n, cv, dst, pitch, stream=st)
                    ev[r][1].record(st)
                st.synchronize()
                ms = [x.elapsed_time(y) for x, y in ev]
            else:
                ev = []
                for r in range(2 * a.reps):
                    h = vp()
                    assert hip.hipEventCreateWithFlags(ctypes.byref(h), flags) == 0
                    ev.append(h)
                for r in range(a.reps):
                    assert hip.hipEventRecord(ev[2 * r], sptr) == 0
                    codec.encode_batch(ctx, src, n, cv, dst, pitch, stream=st)
                    assert hip.hipEventRecord(ev[2 * r + 1], sptr) == 0
                st.synchronize()
                for r in range(a.reps):
                    t = ctypes.c_float()
                    assert hip.hipEventElapsedTime(ctypes.byref(t), ev[2 * r], ev[2 * r + 1]) == 0
                    ms.append(t.value)
                for h in ev:
                    hip.hipEventDestroy(h)
            m = float(np.median(ms))
            print(json.dumps({"events": kind, "n": n, "encode_ms": round(m, 4),
                              "frac": round(byts / (m * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()

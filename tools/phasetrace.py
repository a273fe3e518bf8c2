"""Per-workgroup phase timeline of one encode launch from a DECDS_PHASE_TRACE build: wave 0 of every
workgroup stamps the 100 MHz real-time counter at entry, after the edge pass, when its first tables are
ready, after its last lookups and once its stores have drained (rlnc_encode_sweep_kernel). Prints one
JSON line per (n, run): percentiles of each phase in µs from the first workgroup's entry, beside the
launch's HIP-event time.

build: python -m decds_amd.build --variant ptrace -DDECDS_PHASE_TRACE=1
usage: DECDS_LIB=build/variants/lib_ptrace.so python tools/phasetrace.py --sizes 1,16 [--knob NAME=V]"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PT_WGS, PT_SLOTS = 8192, 32


def pct(v, qs=(0, 50, 90, 100)):
    import numpy as np
    return [round(float(x), 2) for x in np.percentile(v, qs)] if len(v) else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,2,16")
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--knob", action="append", default=[])
    a = ap.parse_args()
    import numpy as np
    import torch
    import decds_amd
    from decds_amd import codec
    from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N, lib

    L = lib()
    L.decds_debug_phase_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for kv in a.knob:
        k, v = kv.split("=")
        L.decds_tuning(k.encode(), int(v), 1)
    sizes = [int(x) for x in a.sizes.split(",")]
    nmax = max(sizes)
    ctx = decds_amd.Context(0)
    st = torch.cuda.Stream()
    src = torch.empty(nmax * CS, dtype=torch.uint8, device="cuda")
    codec.fill_random_device(ctx, 7, src, stream=st)
    cv = torch.from_numpy(codec.fill_random_host(8, nmax * N * K)).cuda()
    dst, pitch = codec.coded_buffer(nmax)
    st.synchronize()
    buf = np.zeros(PT_WGS * PT_SLOTS, dtype=np.uint64)
    for n in sizes:
        for _ in range(30):
            codec.encode_batch(ctx, src, n, cv, dst, pitch, stream=st)
        st.synchronize()
        for run in range(a.runs):
            assert L.decds_debug_phase_trace(None, 1) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            codec.encode_batch(ctx, src, n, cv, dst, pitch, stream=st)
            e1.record(st)
            st.synchronize()
            assert L.decds_debug_phase_trace(buf.ctypes.data, 0) == 0
            s = buf.reshape(PT_WGS, PT_SLOTS).astype(np.int64)
            s = s[s[:, 0] > 0]
            t0 = s[:, 0].min()
            us = lambda c: (s[:, c] - t0) / 100.0
            tile = s[:, 2] > 0
            edge = (~tile) & (s[:, 4] > 0)
            rec = {"n": n, "run": run, "event_us": round(e0.elapsed_time(e1) * 1e3, 2), "workgroups": int(len(s)),
                   "tile_wgs": int(tile.sum()), "edge_or_idle_wgs": int(edge.sum()),
                   "entry_p0_50_90_100": pct(us(0)),
                   "edge_done": pct(us(1)[tile]),
                   "coeffs_in": pct(us(24)[tile & (s[:, 24] > 0)]),
                   "first_build_done": pct(us(25)[tile & (s[:, 25] > 0)]),
                   "tables_ready": pct(us(2)[tile]),
                   "lookups_done": pct(us(3)[tile]),
                   "drained": pct(us(4)[tile]),
                   "edge_wgs_drained": pct(us(4)[edge]),
                   "tiles_min_max": [int(s[tile, 5].min()), int(s[tile, 5].max())] if tile.any() else None,
                   "round_start_p50": [round(float(np.median(us(8 + k)[tile & (s[:, 8 + k] > 0)])), 2)
                                       for k in range(16) if (tile & (s[:, 8 + k] > 0)).sum() > len(s) // 2],
                   "by_tiles": {int(k): [int((tile & (s[:, 5] == k)).sum()),
                                         round(float(np.median(us(3)[tile & (s[:, 5] == k)])), 2)]
                                for k in sorted(set(s[tile, 5].tolist()))},
                   "edge_wgs_first_tile_p50": round(float(np.median(us(2)[tile & (s[:, 1] - s[:, 0] > 200)])), 2)
                   if (tile & (s[:, 1] - s[:, 0] > 200)).any() else None,
                   "span_us": round(float((s[:, 4].max() - t0) / 100.0), 2),
                   "algorithmic_frac_of_span": round(n * (CS + N * F) / ((s[:, 4].max() - t0) * 1e-8) / 8e12, 4)}
            if (s[:, 6] != 0).any():  # placement (HW_ID / XCC_ID, trace builds that record them)
                key = (s[:, 7] << 16) | ((s[:, 6] >> 8) & 0xFF)
                fin = us(3)
                tiles_wg = s[:, 5]
                pair_dt, pair_dfin, lone = [], [], 0
                for k in np.unique(key[tile]):
                    m = np.nonzero(tile & (key == k))[0]
                    if len(m) == 2:
                        pair_dt.append(abs(int(tiles_wg[m[0]]) - int(tiles_wg[m[1]])))
                        pair_dfin.append(abs(float(fin[m[0]] - fin[m[1]])))
                    else:
                        lone += 1
                rec["placement"] = {
                    "cus": int(len(np.unique(key[tile]))), "cus_not_two_wgs": lone,
                    "pair_tile_diff_hist": {int(v): int(c) for v, c in zip(*np.unique(pair_dt, return_counts=True))},
                    "pair_finish_diff_us_p50_90_max": pct(pair_dfin, (50, 90, 100)),
                    "finish_us_by_xcd_p50": {int(x): round(float(np.median(fin[tile & (s[:, 7] == x)])), 2)
                                             for x in np.unique(s[tile, 7])},
                    "tiles_by_xcd_mean": {int(x): round(float(np.mean(tiles_wg[tile & (s[:, 7] == x)])), 2)
                                          for x in np.unique(s[tile, 7])}}
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()

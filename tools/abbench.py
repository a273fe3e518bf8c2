"""Interleaved A/B timing of several library builds in ONE process (cdna_hip_programming.md §5.4
rule 24): every build is loaded with its own ctypes handle; rounds alternate between builds so DVFS
and device drift hit all of them alike. Prints one JSON line per build (median / min over rounds).

usage: python tools/abbench.py --n 1639 --rounds 12 lib_a.so lib_b.so[:pitch[+offset]][@KNOB=V] ...
  "default" = the in-tree library; @KNOB=V sets a launch-shape threshold (decds_tuning, e.g.
  @DECDS_ENC_SMALL_MAX_N=64) before each of that build's runs, so forms of one build A/B in-process.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1639)
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--warmup-s", type=float, default=3.0)
    ap.add_argument("--alloc-n", type=int, default=0, help="size the buffers for this many chunksets (>= n)")
    ap.add_argument("--at", type=int, default=0, help="run on chunksets [at, at + n) of the buffers")
    ap.add_argument("--check", action="store_true", help="verify every build's repaired chunksets against the source")
    ap.add_argument("--check-reps", type=int, default=1, help="repeat the output check this many times")
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    import numpy as np
    import torch
    from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N, _declare

    n = a.n
    na = max(a.alloc_n, n + a.at)
    builds = []
    for spec in a.libs:
        spec, _, knob = spec.partition("@")
        path, _, rest = spec.partition(":")
        if path == "default":
            from decds_amd import build as _build
            path = _build.LIB
        pitch, _, off = rest.partition("+")  # lib.so[:pitch[+offset]]: coded rows start `offset` bytes in
        L = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
        _declare(L)
        h = ctypes.c_void_p()
        assert L.decds_ctx_create(0, ctypes.byref(h)) == 0, L.decds_last_error()
        kname, _, kval = knob.partition("=")
        builds.append({"tag": os.path.basename(path)[:-3] + (":%s" % rest if rest else "") + ("@%s" % knob if knob else ""),
                       "lib": L, "ctx": h, "knob": (kname.encode(), int(kval)) if knob else None,
                       "pitch": int(pitch) if pitch else F, "off": int(off) if off else 0, "cs": CS,
                       "t": []})
    maxcs = max(b["cs"] for b in builds)
    maxpitch = max(b["pitch"] for b in builds)
    st = torch.cuda.Stream()
    vp = ctypes.c_void_p
    src_all = torch.empty(na * maxcs + 64, dtype=torch.uint8, device="cuda")
    src = src_all[a.at * maxcs:]
    builds[0]["lib"].decds_fill_random_device(builds[0]["ctx"], 1, 0, vp(src.data_ptr()), src.numel(), vp(st.cuda_stream))
    coeffs = torch.from_numpy(np.random.default_rng(2).integers(0, 256, n * N * K, dtype=np.uint8)).cuda()
    rng = np.random.default_rng(3)
    cand = np.full((n, N), 0xFF, np.uint8)
    for c in range(n):
        cand[c, :K] = rng.permutation(N)[:K]
    cand = torch.from_numpy(cand).cuda()
    coded_all = torch.empty(na * N * maxpitch + 512, dtype=torch.uint8, device="cuda")
    coded0 = coded_all[a.at * N * maxpitch:]
    plan = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(n * N, dtype=torch.int8, device="cuda")
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    out_all = torch.empty(na * maxcs + 64, dtype=torch.uint8, device="cuda")
    out = out_all[a.at * maxcs:]
    torch.cuda.synchronize()
    sp = vp(st.cuda_stream)

    # every knob any build sets, per library handle: a build that does not set one must run at its default
    # (knobs are process-wide per loaded library, and two specs of one .so share that library)
    knob_names = sorted({b["knob"][0] for b in builds if b["knob"]})

    def run(b, ev=None, encode=True):
        L, h, p = b["lib"], b["ctx"], b["pitch"]
        for name in knob_names:
            L.decds_tuning(name, b["knob"][1] if b["knob"] and b["knob"][0] == name else (1 << 64) - 1, 1)
        coded = coded0[b["off"]:]
        if ev:
            ev[0].record(st)
        assert not encode or L.decds_encode_batch(h, vp(src.data_ptr()), n, vp(coeffs.data_ptr()), vp(coded.data_ptr()), p, sp) == 0
        if ev:
            ev[1].record(st)
        assert L.decds_repair_plan_batch(h, vp(coded.data_ptr()), p, n, vp(cand.data_ptr()), vp(plan.data_ptr()),
                                         vp(verd.data_ptr()), vp(status.data_ptr()), sp) == 0
        if ev:
            ev[2].record(st)
        assert L.decds_decode_batch(h, vp(coded.data_ptr()), p, n, vp(plan.data_ptr()), vp(out.data_ptr()),
                                    vp(status.data_ptr()), None, sp) == 0
        if ev:
            ev[3].record(st)

    t0 = time.time()
    while time.time() - t0 < a.warmup_s:
        for b in builds:
            run(b)
        st.synchronize()
    for r in range(a.rounds):
        for b in (builds if r % 2 == 0 else builds[::-1]):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            run(b, ev)
            st.synchronize()
            b["t"].append([ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2]), ev[2].elapsed_time(ev[3])])
    if a.check:  # every ready chunkset must repair to its source bytes
        for b, _ in [(b, r) for r in range(a.check_reps) for b in builds]:
            out.fill_(0xA5)
            torch.cuda.synchronize()  # the fill runs on torch's stream, the codec on st
            run(b)
            st.synchronize()
            ok = status[:n].cpu().numpy() == 0
            same = (out[:n * CS].view(n, CS) == src[:n * CS].view(n, CS)).all(dim=1).cpu().numpy()
            st_np = status[:n].cpu().numpy()
            idle = (st_np != 0) & (st_np != 6)  # not ready: the decode must leave the output alone
            kept = (out[:n * CS].view(n, CS) == 0xA5).all(dim=1).cpu().numpy()
            prev = b.get("check")
            b["check"] = {"ready": int(ok.sum()), "bad": int((ok & ~same).sum()), "not_ready": int(idle.sum()),
                          "not_ready_written": int((idle & ~kept).sum())}
            where = []  # first bad chunksets: (chunkset, mismatching bytes, first/last piece:column)
            for c in np.nonzero(ok & ~same)[0][:8]:
                d = np.nonzero((out[c * CS:(c + 1) * CS] != src[c * CS:(c + 1) * CS]).cpu().numpy())[0]
                Lp = (CS + K - 1) // K + 1  # piece length L
                where.append([int(c), int(d.size), "%d:%d" % divmod(int(d[0]), Lp), "%d:%d" % divmod(int(d[-1]), Lp)])
            if where:
                b["check"]["where"] = where
                # the same coded rows planned and decoded again: a decode race comes out different
                out.fill_(0xA5)
                torch.cuda.synchronize()
                run(b, encode=False)
                st.synchronize()
                again = (out[:n * CS].view(n, CS) == src[:n * CS].view(n, CS)).all(dim=1).cpu().numpy()
                b["check"]["bad_redecode"] = int((ok & ~again).sum())
            if prev:  # repeated checks: bad counts per repetition, first failure kept
                b["check"]["bad_reps"] = prev.get("bad_reps", [prev["bad"]]) + [b["check"]["bad"]]
                if "where" in prev:
                    b["check"]["where"] = prev["where"]
    for b in builds:
        t = np.array(b["t"])
        med, mn = np.median(t, axis=0), t.min(axis=0)
        print(json.dumps({"tag": b["tag"], "n": n, "alloc_n": na, "at": a.at, "pitch": b["pitch"], "encode_ms": round(med[0], 4),
                          "encode_min_ms": round(mn[0], 4), "plan_ms": round(med[1], 4), "decode_ms": round(med[2], 4),
                          "decode_min_ms": round(mn[2], 4), "encode_GBps": round(n * (CS + N * F) / med[0] / 1e6, 1),
                          "decode_GBps": round(n * (K * F + CS) / med[2] / 1e6, 1), **({"check": b["check"]} if "check" in b else {})}),
              flush=True)


if __name__ == "__main__":
    main()

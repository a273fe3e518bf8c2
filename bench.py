"""bench.py — device-resident RLNC encode+repair throughput on MI355X (BASELINE.json metric).

Step = one pass of the hot path over one batch: encode the rank's chunksets (10 -> 16,
chunkset.rs:43-52) and repair every chunkset from exactly 10 random surviving coded chunks
(plan + decode, chunkset.rs:173-208), all resident in HBM. Default workload = BASELINE configs 3 + 4,
the largest single-GPU configuration: a 16 GiB random blob = 1639 chunksets per GPU, all in one
batch, encoded and repaired from exactly 10 random survivors per chunkset (--config cfg2: the 1 GiB
blob of config 2). For N > 1 each rank owns its own 16 GiB slice of a 16N GiB blob (contiguous
chunkset-index shard, no collective on the data path; N = 8 is config 5, the 128 GiB blob);
value = blob bytes of all ranks / max-over-ranks time ("scaling": "weak").

Launched with torchrun for N > 1 (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* from the environment).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
HBM_COPY_GBS = 6290.0  # MI355X_MICROARCH.md: 6.29 TB/s measured float4 copy (SURVEY.md §8d second denominator)
SWEEP = (1, 16, 64, 256, 1024, 1639)  # encode batch sweep: chunksets per launch

CONFIGS = {
    # name: (blob bytes per GPU, description)
    "cfg2": (1 << 30, "1 GiB random blob (103 x 10 MiB chunksets) encode + repair from 10 random survivors, one batch"),
    "cfg3": (16 << 30, "16 GiB random blob (1639 chunksets) encode + repair from 10 random survivors, one batch"),
}


class FenceFreeEvents:
    """HIP timing events created with hipEventDisableSystemFence, recorded on a torch stream through the
    HIP runtime torch already loaded. A default event (torch.cuda.Event) performs a system-scope fence —
    an L2 writeback and invalidate — when it is recorded; these skip it ("can improve the accuracy of
    timing measurements", hip_runtime_api.h), which matters only for launches of a few microseconds."""
    DISABLE_SYSTEM_FENCE = 0x20000000

    def __init__(self, k):
        import ctypes
        with open("/proc/self/maps") as f:
            paths = sorted({ln.split()[-1] for ln in f if "libamdhip64.so" in ln})
        # the runtime that owns torch's streams: the one under torch's own lib directory when torch
        # bundles one, else the only one mapped (two runtimes and neither torch's: refuse)
        import torch
        tlib = os.path.realpath(os.path.join(os.path.dirname(torch.__file__), "lib"))
        own = [p for p in paths if os.path.realpath(os.path.dirname(p)) == tlib]
        if own:
            paths = own
        if len(paths) != 1:
            raise RuntimeError("FenceFreeEvents: expected one HIP runtime mapped, found %s" % paths)
        self.hip = h = ctypes.CDLL(paths[0])  # already mapped: the same runtime, no second copy
        vp = ctypes.c_void_p
        h.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
        h.hipEventRecord.argtypes = [vp, vp]
        h.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), vp, vp]
        h.hipEventDestroy.argtypes = [vp]
        self.ev = []
        for _ in range(k):
            e = vp()
            if h.hipEventCreateWithFlags(ctypes.byref(e), self.DISABLE_SYSTEM_FENCE) != 0:
                raise RuntimeError("hipEventCreateWithFlags(hipEventDisableSystemFence) failed")
            self.ev.append(e)

    def record(self, i, stream):
        import ctypes
        if self.hip.hipEventRecord(self.ev[i], ctypes.c_void_p(stream.cuda_stream)) != 0:
            raise RuntimeError("hipEventRecord failed")

    def elapsed_ms(self, i, j):
        import ctypes
        t = ctypes.c_float()
        if self.hip.hipEventElapsedTime(ctypes.byref(t), self.ev[i], self.ev[j]) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return t.value

    def close(self):
        for e in self.ev:
            self.hip.hipEventDestroy(e)
        self.ev = []


def shard_range(n_total, world, rank):
    """contiguous chunkset-index shard of rank"""
    per = -(-n_total // world)
    lo = min(rank * per, n_total)
    return lo, min(lo + per, n_total)


def shard_arg(v):
    """--rehearse-shard R/W: integers with 0 <= R < W (checked before anything touches the device)"""
    try:
        r, w = (int(x) for x in v.split("/"))
    except ValueError:
        raise argparse.ArgumentTypeError("expected R/W, e.g. 7/8, got %r" % v)
    if not 0 <= r < w:
        raise argparse.ArgumentTypeError("--rehearse-shard R/W needs 0 <= R < W, got %r" % v)
    return r, w


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--settle-s", type=float, default=0.5,
                   help="after the W warmup steps, keep running untimed steps until this many seconds passed")
    p.add_argument("--config", default="cfg3", choices=sorted(CONFIGS),
                   help="cfg3 (default): BASELINE's largest single-GPU configuration, 16 GiB per GPU "
                        "(configs 3 + 4; at N = 8 the whole job is config 5, the 128 GiB blob)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-commit", action="store_true", help="skip timing the commitment kernels (row f1)")
    p.add_argument("--no-sweep", action="store_true", help="skip the encode batch sweep (256..1639 chunksets)")
    p.add_argument("--cpu-sample", type=int, default=0, help="chunksets in the CPU sample (0 = auto)")
    p.add_argument("--no-extras", action="store_true",
                   help="skip the pattern ceilings and the end-to-end (PCIe-inclusive) host-path rate")
    p.add_argument("--no-api-shapes", action="store_true",
                   help="skip the reference's build_blob / repair_blob shapes through the blob API (1 MiB .. 4 GiB)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    p.add_argument("--rehearse-shard", default=None, metavar="R/W", type=shard_arg,
                   help="one process, no process group: run only rank R's shard of a W-GPU job on this GPU "
                        "(cfg5, the 128 GiB blob over 8 GPUs, is --config cfg3 --rehearse-shard R/8)")
    p.add_argument("--spot-out", default=None, metavar="PATH.npz",
                   help="after the timed region, save the source bytes, coding vectors and coded rows of the "
                        "shard's first, middle and last chunkset (the GPU tests check them against the oracle)")
    p.add_argument("--digest-out", default=None, metavar="PATH.npy",
                   help="after the timed region, save the chunk digest (chunk.rs:40-46, decds_commit_batch) of every "
                        "coded row of the shard: the GPU tests compare all of them with the oracle's rows' digests")
    p.add_argument("--packed", action="store_true",
                   help="coded rows packed at pitch 1,048,587 instead of the recommended 128-B-aligned layout")
    return p.parse_args(argv)


def usable_cpus():
    """the CPUs this process may run on (sched affinity; os.cpu_count() if unavailable)"""
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cgroup_cpus():
    """the cgroup v2 CPU quota in CPUs (cpu.max "quota period"), None when unlimited or unreadable"""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        return None if quota == "max" else int(quota) / int(period)
    except (OSError, ValueError):
        return None


def cpu_threads():
    """the thread counts the CPU baseline measures: all usable CPUs (rayon's pool on every core,
    blob.rs:256-264), the count Rust's available_parallelism() — rayon's default pool size — gives
    (usable CPUs capped by the cgroup quota), and 16 (the box's nominal CPU share per GPU)"""
    allc = max(1, usable_cpus())
    q = cgroup_cpus()
    rayon = max(1, min(allc, int(-(-q // 1)))) if q else allc
    return {"all_cores": allc, "rayon_default": rayon, "threads_16": min(16, allc)}


def host_cpu():
    """the host's CPU model and the CPU counts this process sees"""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"model": model, "cpus_online": os.cpu_count(), "cpus_usable": usable_cpus(), "cgroup_cpu_quota": cgroup_cpus()}


def cpu_baseline(n_sample, seed, repeats=5, cfg2_chunksets=103):
    """The CPU restatement (oracle/, "port") on the host cores: chunkset-parallel encode
    (blob.rs:256-264) + per-chunkset repair from 10 survivors (chunkset.rs:173-208).

    Codec = the strongest restatement: column-blocked GFNI affine multiplies on AVX-512
    (oracle/rlnc_cpu_fast.c; coefficient-only rank + inverse, then one blocked pass for the repair),
    the median of `repeats` runs (each at least 1 s of passes over the sample) with their spread, at
    each of the thread counts cpu_threads() names: `all_cores` (every usable CPU — the reference's
    shape, rayon over all cores), `rayon_default` (what rayon's default pool takes: usable CPUs capped
    by the cgroup quota; measured only when it differs) and `threads_16`. The sample holds at least
    one chunkset per thread. `value` is the strongest of them (its thread count in `cores`): the
    GPU/CPU ratio is quoted against the fastest CPU configuration measured. Beside it (BASELINE.md's
    plan): the same codec on 1 thread, on config 2's sample (the 1 GiB blob's 103 chunksets) with the
    headline's thread count and on config 1's single chunkset (one thread: the work is chunkset-parallel); one run each
    of the row-pass forms (AVX2 nibble tables; the scalar table-driven loop rlnc 0.4.0 is recalled to
    use) on 16 threads. All produce the same bytes (tests/test_oracle.py)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as o
    counts = cpu_threads()
    allc, t16 = counts["all_cores"], counts["threads_16"]
    if n_sample <= 0:
        n_sample = max(256, allc)  # >= one chunkset per thread

    def sample(n, sd):
        blob = o.fill_random(sd, n * o.CS)
        coeffs = o.fill_random(sd + 1, n * o.N * o.K)
        rng = np.random.default_rng(sd)
        cand = np.full((n, o.N), 0xFF, np.uint8)
        for c in range(n):
            cand[c, :o.K] = rng.permutation(o.N)[:o.K]
        return blob, coeffs, cand

    def run(enc, rep, smp, nthreads, min_s=0.0):
        """encode + repair of the sample, repeated until min_s seconds have passed (a GFNI pass over 256
        chunksets on 16 threads is ~60 ms: single passes measured +-14 % run to run, BENCH_r03)"""
        blob, coeffs, cand = smp
        n = cand.shape[0]
        gib = n * o.CS / GIB
        t_enc = t_rep = 0.0
        reps = 0
        while reps == 0 or t_enc + t_rep < min_s:
            t0 = time.perf_counter()
            coded = enc(blob, coeffs, nthreads=nthreads)
            t1 = time.perf_counter()
            out, status = rep(coded, cand, blob.size, nthreads=nthreads)
            t2 = time.perf_counter()
            if reps == 0:
                ok = status == 0
                assert np.array_equal(out.reshape(n, o.CS)[ok], blob.reshape(n, o.CS)[ok])
            del coded, out
            t_enc += t1 - t0
            t_rep += t2 - t1
            reps += 1
        # encode + repair GiB/s as the GPU's value: (blob bytes encoded + repaired) / 2 per second
        return {"value": reps * gib / (t_enc + t_rep), "encode_gib_s": reps * gib / t_enc,
                "repair_gib_s": reps * gib / t_rep, "passes": reps}

    rnd = lambda d: {k: (round(v, 2) if isinstance(v, float) else v) for k, v in d.items()}

    def median(runs):
        med = lambda k: float(np.median([r[k] for r in runs]))
        return {"value": med("value"), "encode_gib_s": med("encode_gib_s"), "repair_gib_s": med("repair_gib_s"),
                "runs": len(runs), "passes": sum(r["passes"] for r in runs), "spread": [round(min(r["value"] for r in runs), 2),
                                              round(max(r["value"] for r in runs), 2)]}

    smp = sample(n_sample, seed)
    desc = lambda n, th: "%d chunksets (%.0f MiB) encode + repair from 10 survivors, %d threads (chunkset-parallel)" % (
        n, n * o.CS / 2 ** 20, th)
    rows = {}
    o.set_simd(0)
    rows["scalar tables, row passes"] = dict(rnd(run(o.blob_encode, o.blob_repair, smp, t16)), cores=t16)
    if o.set_simd(1):
        rows["avx2 nibble tables, row passes"] = dict(rnd(run(o.blob_encode, o.blob_repair, smp, t16)), cores=t16)
    o.set_simd(0)
    extra = {}
    if not o.fast_supported():
        head_name = max(rows, key=lambda k: rows[k]["value"])
        head = dict(rows[head_name], runs=1, spread=None)
        return {"value": head["value"], "unit": "GiB/s", "cores": t16, "kind": "port", "variant": head_name,
                "sample": desc(n_sample, t16), "host": host_cpu(), "thread_counts": counts, "other_variants": rows}
    head_name = "avx512 gfni affine, column-blocked"
    measured = {}
    for key in ("all_cores", "rayon_default", "threads_16"):
        th = counts[key]
        same = [k for k, v in measured.items() if v["cores"] == th]
        if same:  # the same thread count as a figure already measured
            extra[key] = {"same_as": same[0], "cores": th}
            continue
        m = median([run(o.fast_blob_encode, o.fast_blob_repair, smp, th, min_s=1.0) for _ in range(max(1, repeats))])
        measured[key] = dict(rnd(m), cores=th, sample=desc(n_sample, th))
        extra[key] = measured[key]
    best = max(measured, key=lambda k: measured[k]["value"])
    head = measured[best]
    del smp
    smp2 = sample(cfg2_chunksets, seed + 2)
    cfg2_tag = " (config 2: the 1 GiB blob)" if cfg2_chunksets == 103 else ""
    extra["threads_1"] = dict(rnd(run(o.fast_blob_encode, o.fast_blob_repair, smp2, 1, min_s=1.0)), cores=1,
                              sample="%d chunksets%s, 1 thread" % (cfg2_chunksets, cfg2_tag))
    th2 = min(head["cores"], cfg2_chunksets)  # the headline's thread count (more threads than the cgroup quota throttle, r07a)
    extra["cfg2"] = dict(rnd(median([run(o.fast_blob_encode, o.fast_blob_repair, smp2, th2, min_s=1.0)
                                     for _ in range(max(1, repeats))])), cores=th2,
                         sample="%d chunksets%s, %d threads" % (cfg2_chunksets, cfg2_tag, th2))
    del smp2
    # config 1: one chunkset (chunkset-parallel, so one thread does all of it), median of repeats
    smp1 = sample(1, seed + 3)
    extra["cfg1"] = dict(rnd(median([run(o.fast_blob_encode, o.fast_blob_repair, smp1, 1, min_s=0.5)
                                     for _ in range(max(1, repeats))])), cores=1,
                         sample="1 chunkset (config 1), 1 thread")
    del smp1
    # the reference's bench shapes (build_blob.rs / repair_blob.rs, API_SIZES) on the same codec and the
    # headline's thread count: encode of the whole blob (Blob::new's RLNC part) and repair of every
    # chunkset from the first 10 useful of shares 0..11 in a shuffled order (RepairingBlob's add_chunk
    # rank step + decode). RLNC only: the restatement carries no SIMD BLAKE3, so the commitment and the
    # chunk validation the GPU figures (api_shapes) include are not in these.
    th = head["cores"]
    api = []
    for size in API_SIZES:
        n = -(-size // o.CS)
        blob = o.fill_random(0xA91 + size.bit_length(), size)
        coeffs = o.fill_random(0xC0EF0A91, n * o.N * o.K)
        rng = np.random.default_rng(0x5EED + size.bit_length())
        cand = np.full((n, o.N), 0xFF, np.uint8)
        for c in range(n):
            cand[c, :12] = rng.permutation(12)
        t_enc, t_rep, reps = 0.0, 0.0, 0
        while reps < 3 or t_enc + t_rep < 0.5:
            t0 = time.perf_counter()
            coded = o.fast_blob_encode(blob, coeffs, nthreads=th)
            t1 = time.perf_counter()
            out, status = o.fast_blob_repair(coded, cand, size, nthreads=th)
            t2 = time.perf_counter()
            if reps == 0:
                assert (status == 0).all() and np.array_equal(out, blob), "CPU repair of the api shape differs"
            del coded, out
            t_enc, t_rep, reps = t_enc + t1 - t0, t_rep + t2 - t1, reps + 1
        api.append({"blob_bytes": size, "chunksets": n, "encode_ms": round(t_enc / reps * 1e3, 3),
                    "repair_ms": round(t_rep / reps * 1e3, 3), "encode_GiBps": round(reps * size / GIB / t_enc, 2),
                    "repair_GiBps": round(reps * size / GIB / t_rep, 2), "passes": reps})
        del blob
    extra["api_shapes"] = {"cores": th, "what": "GFNI restatement, RLNC encode / repair only (no commitment, no "
                                                "validation), the reference's build_blob / repair_blob sizes",
                           "sizes": api}
    return dict({"value": head["value"], "unit": "GiB/s", "cores": head["cores"], "kind": "port",
                 "variant": head_name, "headline": best, "median_of": head["runs"], "passes": head["passes"],
                 "spread": head["spread"], "sample": head["sample"],
                 "encode_gib_s": head["encode_gib_s"], "repair_gib_s": head["repair_gib_s"],
                 "host": host_cpu(), "thread_counts": counts, "other_variants": rows}, **extra)


def pattern_ceilings(torch, stream, device, n, src, coeffs, coded, pitch, plan, out, status, reps=10):
    """Each streaming kernel's own access-pattern ceiling, timed on the headline's buffers after the
    timed region: tools/bin/libdecds_pattern.so is the product's kernel source built with
    DECDS_STUDY_PATTERN (rlnc_kernels.hip: the same loads, stores, tile order and table builds, the LDS
    lookups replaced by one XOR per input dword). It writes wrong bytes by design, so it runs after the
    repaired data was checked: decode first (on the real plans and coded rows, so its edge pass sees
    intact tails), then encode. Median of `reps` launches, each between its own events on the bench
    stream. Loaded privately (RTLD_LOCAL) beside the product library."""
    import ctypes
    import numpy as np
    path = os.path.join(ROOT, "tools", "bin", "libdecds_pattern.so")
    if not os.path.exists(path):
        return {"error": "tools/bin/libdecds_pattern.so not built (decds_amd.build.build_pattern)"}
    L = ctypes.CDLL(path)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    L.decds_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.decds_ctx_destroy.argtypes = [vp]
    L.decds_encode_batch.argtypes = [vp, vp, sz, vp, vp, sz, vp]
    L.decds_decode_batch.argtypes = [vp, vp, sz, sz, vp, vp, vp, vp, vp]
    ctx = vp()
    if L.decds_ctx_create(device, ctypes.byref(ctx)) != 0:
        return {"error": "decds_ctx_create failed in the pattern build"}
    st = vp(stream.cuda_stream)

    def timed(launch):
        t_w = time.perf_counter()
        while time.perf_counter() - t_w < 0.2:
            for _ in range(4):
                assert launch() == 0
            stream.synchronize()
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(reps)]
        for e in ev:
            e[0].record(stream)
            assert launch() == 0
            e[1].record(stream)
        stream.synchronize()
        return float(np.median([a.elapsed_time(b) for a, b in ev]))

    dec_ms = timed(lambda: L.decds_decode_batch(ctx, coded.data_ptr(), pitch, n, plan.data_ptr(), out.data_ptr(),
                                                status.data_ptr(), None, st))
    enc_ms = timed(lambda: L.decds_encode_batch(ctx, src.data_ptr(), n, coeffs.data_ptr(), coded.data_ptr(), pitch, st))
    L.decds_ctx_destroy(ctx)
    return {"library": "tools/bin/libdecds_pattern.so (DECDS_STUDY_PATTERN)", "launches": reps,
            "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4)}


def copy_pattern_ceiling(torch, stream, n, coded, pitch, plan, out, reps=10):
    """The decode's copy ceiling (tools/copypattern.hip, built into tools/bin/libdecds_copypattern.so): the
    decode's exact HBM address stream — per ready chunkset the plan's ten selected coded rows read at
    their payload offsets, ten byte-misaligned piece stores at i*L — with no tables, no arithmetic and
    no tile counter, in each of its launch geometries; the fastest is the ceiling. Timed on the
    headline's own plans and coded rows after the repaired bytes were checked (it overwrites the repaired
    output). Median of `reps` launches per geometry, each between its own events on the bench stream."""
    import ctypes
    import numpy as np
    path = os.path.join(ROOT, "tools", "bin", "libdecds_copypattern.so")
    if not os.path.exists(path):
        return {"error": "tools/bin/libdecds_copypattern.so not built (decds_amd.build.build_copypattern)"}
    L = ctypes.CDLL(path)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    L.decds_copy_pattern_decode.argtypes = [vp, sz, sz, vp, vp, ctypes.c_int, vp]
    L.decds_copy_pattern_variant_name.restype = ctypes.c_char_p
    st = vp(stream.cuda_stream)
    res = {}
    for v in range(4):
        launch = lambda: L.decds_copy_pattern_decode(coded.data_ptr(), pitch, n, plan.data_ptr(), out.data_ptr(), v, st)
        t_w = time.perf_counter()
        while time.perf_counter() - t_w < 0.2:
            for _ in range(4):
                assert launch() == 0
            stream.synchronize()
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(reps)]
        for e in ev:
            e[0].record(stream)
            assert launch() == 0
            e[1].record(stream)
        stream.synchronize()
        res[L.decds_copy_pattern_variant_name(v).decode()] = round(float(np.median([a.elapsed_time(b) for a, b in ev])), 4)
    best = min(res, key=res.get)
    return {"library": "tools/bin/libdecds_copypattern.so (tools/copypattern.hip)", "launches": reps,
            "variants_ms": res, "best": best, "decode_ms": res[best]}


def end_to_end(ctx, chunksets=103, repeats=5, batch=16):
    """The PCIe-inclusive rate north_star asks for (blob in host memory -> coded chunks in host memory
    -> repaired blob in host memory): decds_blob_encode_host and decds_blob_repair_host (handle_break.rs
    / handle_repair.rs's device work, blob.rs:252-264 / 373-473) at config 2's 1 GiB blob, every caller
    buffer from decds_host_alloc (page-locked: direct DMA), H2D / kernels / D2H overlapped over three
    slots in the library. One warm-up call each, then the median of `repeats` calls; the repaired
    chunksets are compared with the blob."""
    import numpy as np
    from decds_amd import codec
    from decds_amd.blob import HostBuffer
    from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N
    blob_len = chunksets * CS if chunksets != 103 else 1 << 30
    n = -(-blob_len // CS)
    hb_blob, hb_coded, hb_out = HostBuffer(blob_len), HostBuffer(n * N * F), HostBuffer(blob_len)
    blob = hb_blob.array
    blob[:] = codec.fill_random_host(0xDEC05004, blob_len)
    coeffs = codec.fill_random_host(0xC0EF0004, n * N * K)
    rng = np.random.default_rng(0x5EED0004)
    cand = np.full((n, N), 0xFF, np.uint8)
    for c in range(n):
        cand[c, :K] = rng.permutation(N)[:K]
    coded_out = hb_coded.array.reshape(n * N, F)
    enc, rep = [], []
    for i in range(repeats + 1):
        t0 = time.perf_counter()
        codec.blob_encode_host(ctx, blob, coeffs, batch=batch, out=coded_out)
        t1 = time.perf_counter()
        _, status = codec.blob_repair_host(ctx, coded_out, cand, blob_len, batch=batch, out=hb_out.array)
        t2 = time.perf_counter()
        if i:
            enc.append(t1 - t0)
            rep.append(t2 - t1)
    ok = np.nonzero(status == 0)[0]
    out = hb_out.array
    for c in ok.tolist():
        lo, hi = c * CS, min((c + 1) * CS, blob_len)
        assert np.array_equal(out[lo:hi], blob[lo:hi]), "end-to-end repaired chunkset %d differs" % c
    rep_len = sum(min(CS, blob_len - c * CS) for c in ok.tolist())
    e, r = float(np.median(enc)), float(np.median(rep))
    res = {"what": "decds_blob_encode_host + decds_blob_repair_host, host memory to host memory (PCIe-inclusive)",
           "blob_bytes": blob_len, "chunksets": n, "batch": batch, "memory": "decds_host_alloc (page-locked) caller buffers",
           "calls": repeats, "encode_ms": round(e * 1e3, 3), "repair_ms": round(r * 1e3, 3),
           "encode_spread_ms": [round(min(enc) * 1e3, 3), round(max(enc) * 1e3, 3)],
           "repair_spread_ms": [round(min(rep) * 1e3, 3), round(max(rep) * 1e3, 3)],
           "encode_blob_GiBps": round(blob_len / GIB / e, 2), "repair_blob_GiBps": round(rep_len / GIB / r, 2),
           "value_GiBps": round((blob_len + rep_len) / 2 / GIB / (e + r), 2),
           "encode_pcie_GBps": round((blob_len + n * N * F) / e / 1e9, 2),
           "repair_pcie_GBps": round((len(ok) * K * F + rep_len) / r / 1e9, 2),
           "ready_chunksets": int(len(ok)), "repaired_checked": int(len(ok))}
    del coded_out, out, blob
    for hb in (hb_blob, hb_coded, hb_out):
        hb.free()
    return res


API_SIZES = (1 << 20, 1 << 24, 1 << 28, 1 << 30, 1 << 32)  # decds-lib/benches/build_blob.rs:38-44, repair_blob.rs:35-41


def api_shapes(ctx, sizes=API_SIZES, repeats=5, repair_repeats=3):
    """The reference's own benchmarks through the reference-facing C-ABI, at their five blob sizes
    (1 MiB .. 4 GiB), on one GPU, host memory in and out:

    * build_blob (decds-lib/benches/build_blob.rs:47-55): Blob::new(Vec<u8>) = decds_blob_new on a
      plain (pageable) random blob — whole-blob BLAKE3, encode + commitment of every chunkset, the
      blob-level tree, coded chunks in host memory. `cold_ms`: the first call at that size (the
      coded store is page-locked then; later calls reuse it from the library's block cache);
      `warm_ms`: the median of `repeats` further calls.
    * repair_blob (decds-lib/benches/repair_blob.rs:47-65): the header and shares 0..11 of a Blob,
      their chunks shuffled (seeded), then RepairingBlob::new + add_chunk of every chunk in that order
      (each validated: chunk digest + both proofs; chunks of a chunkset already at rank 10 are refused
      ChunksetReadyToRepair, which the reference ignores) — and, beyond the reference's timed region
      (its add_chunk already decodes), get_repaired_chunkset of every chunkset, each compared with the
      blob after the timing. `add_chunk_ms` / `get_ms` split the median run; `batched` times the same
      arrivals through decds_repairing_blob_add_chunks (validation as device batches).
    Python calls the C-ABI through ctypes with pointers into numpy arrays (no per-chunk copies)."""
    import ctypes
    import numpy as np
    from decds_amd import codec
    from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, N, check, lib
    from decds_amd.blob import Blob, RepairingBlob
    L = lib()
    vp = ctypes.c_void_p
    ptr = lambda a: vp(a.ctypes.data)
    rows = []
    for size in sizes:
        n = -(-size // CS)
        data = codec.fill_random_host(0xA91 + size.bit_length(), size)
        t0 = time.perf_counter()
        blob = Blob(ctx, data)
        cold = time.perf_counter() - t0
        warm = []
        for _ in range(repeats):
            blob.free()
            t0 = time.perf_counter()
            blob = Blob(ctx, data)
            warm.append(time.perf_counter() - t0)
        header = blob.get_blob_header()
        plen = blob.proof_len()
        shares, proofs = np.empty((12, n, F), np.uint8), np.empty((12, n, plen * 32), np.uint8)
        for sh in range(12):  # DECDS_NUM_ERASURE_CODED_SHARES - 4 (repair_blob.rs:51)
            check(L.decds_blob_get_share(blob._h, sh, ptr(shares[sh]), shares[sh].nbytes, ptr(proofs[sh]), proofs[sh].nbytes))
        blob.free()
        del blob
        arrivals = [(sh, c) for sh in range(12) for c in range(n)]
        np.random.default_rng(0x5EED + size.bit_length()).shuffle(arrivals)
        out = np.empty(size, np.uint8)

        def repair_seq():
            t0 = time.perf_counter()
            rb = RepairingBlob(ctx, header)
            h = rb._h
            for sh, c in arrivals:
                st = L.decds_repairing_blob_add_chunk(h, c, c * N + sh, ptr(shares[sh, c]), F, ptr(proofs[sh, c]), plen)
                if st not in (0, 3, 4):  # ok, ChunksetReadyToRepair, ChunkDecodingFailed (repair_blob.rs:62 ignores them)
                    check(st)
            t1 = time.perf_counter()
            ok = 0
            for c in range(n):
                if rb.is_chunkset_ready_to_repair(c):
                    rb.get_repaired_chunkset(c, out=out[c * CS:min(size, (c + 1) * CS)])
                    ok += 1
            t2 = time.perf_counter()
            rb.free()
            return t1 - t0, t2 - t1, ok

        rows_a = np.ascontiguousarray(shares[[a[0] for a in arrivals], [a[1] for a in arrivals]])
        ids = np.array([(c, c * N + sh) for sh, c in arrivals], np.uint64)
        prf_a = np.ascontiguousarray(proofs[[a[0] for a in arrivals], [a[1] for a in arrivals]])

        def repair_batched():
            t0 = time.perf_counter()
            rb = RepairingBlob(ctx, header)
            st = rb.add_rows(rows_a, ids, prf_a, plen)
            assert set(np.unique(st).tolist()) <= {0, 3, 4}, np.unique(st)
            t1 = time.perf_counter()
            ok = 0
            for c in range(n):
                if rb.is_chunkset_ready_to_repair(c):
                    rb.get_repaired_chunkset(c, out=out[c * CS:min(size, (c + 1) * CS)])
                    ok += 1
            t2 = time.perf_counter()
            rb.free()
            return t1 - t0, t2 - t1, ok

        rec = {"blob_bytes": size, "chunksets": n,
               "blob_new": {"cold_ms": round(cold * 1e3, 3), "warm_ms": round(float(np.median(warm)) * 1e3, 3),
                            "warm_spread_ms": [round(min(warm) * 1e3, 3), round(max(warm) * 1e3, 3)],
                            "warm_GiBps": round(size / GIB / float(np.median(warm)), 2), "calls": repeats}}
        for key, fn in (("repair", repair_seq), ("repair_batched", repair_batched)):
            runs = []
            for _ in range(repair_repeats):
                out[:] = 0
                runs.append(fn())
                assert runs[-1][2] == n, "not every chunkset was ready after shares 0..11"
                assert np.array_equal(out, data), "repaired blob differs (%s, %d bytes)" % (key, size)
            tot = sorted(runs, key=lambda r: r[0] + r[1])[len(runs) // 2]
            rec[key] = {"ms": round((tot[0] + tot[1]) * 1e3, 3), "add_chunk_ms": round(tot[0] * 1e3, 3),
                        "get_ms": round(tot[1] * 1e3, 3), "GiBps": round(size / GIB / (tot[0] + tot[1]), 2),
                        "chunks_added": len(arrivals), "runs": repair_repeats}
        rows.append(rec)
        del shares, proofs, rows_a, prf_a, out, data
    return {"what": "the reference's build_blob / repair_blob benches through decds_blob_new / decds_repairing_blob_*",
            "memory": "pageable numpy blob in, the library's own coded store; host-memory end to end (PCIe-inclusive)",
            "sizes": rows}


def init_group(dist, backend, device, rank, world, timeout_s=300):
    """The process group for N > 1 (RCCL; DECDS_BENCH_BACKEND=gloo rehearses the path with ranks
    sharing devices). A failed or stuck rendezvous ends the process with a clear message and a
    non-zero exit instead of hanging the driver's run."""
    import datetime
    try:
        if backend == "gloo":
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=timeout_s))
        else:
            dist.init_process_group("nccl", device_id=device, timeout=datetime.timedelta(seconds=timeout_s))
        dist.barrier()  # the first collective: fails here, not inside the timed region
    except Exception as e:  # noqa: BLE001 - any init failure ends the bench
        sys.stderr.write("bench.py: rank %d/%d: %s process group init failed: %s: %s\n"
                         % (rank, world, "RCCL" if backend == "nccl" else backend, type(e).__name__, e))
        sys.stderr.flush()
        os._exit(3)


def rank_record(torch, rank, local, world, lo, hi, shard_bytes, enc_ms, plan_ms, dec_ms, enc_bytes, dec_bytes,
                n_ready, checked, rep_len, elapsed, steps):
    """one rank's per-GPU figures for the N > 1 line's per_rank (gathered with all_gather_object)"""
    import socket
    props = torch.cuda.get_device_properties(local)
    uuid = getattr(props, "uuid", None)
    enc_gbs = enc_bytes / (enc_ms * 1e-3) / 1e9
    dec_gbs = dec_bytes / (dec_ms * 1e-3) / 1e9 if dec_ms > 0 else 0.0
    return {"rank": rank, "local_rank": local, "host": socket.gethostname(), "device": local,
            "device_uuid": str(uuid) if uuid is not None else None,
            "pci_bus_id": getattr(props, "pci_bus_id", None), "device_name": props.name,
            "chunksets": [lo, hi], "shard_bytes": shard_bytes,
            "encode_ms": round(enc_ms, 4), "plan_ms": round(plan_ms, 4), "decode_ms": round(dec_ms, 4),
            "encode_frac": round(enc_gbs / HBM_PEAK_GBS, 4), "decode_frac": round(dec_gbs / HBM_PEAK_GBS, 4),
            "ready_chunksets": n_ready, "not_ready_chunksets": hi - lo - n_ready,
            "repaired_checked": checked, "repaired_blob_bytes": rep_len,
            "elapsed_s": round(elapsed, 6),
            "gpu_GiBps": round((shard_bytes + rep_len) / 2 * steps / GIB / elapsed, 2)}


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    import decds_amd
    from decds_amd import codec
    from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N
    from decds_amd._capi import lib as _lib

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    rehearse = None
    if args.rehearse_shard:
        if world != 1:
            raise SystemExit("--rehearse-shard runs in a single process")
        rank, world = args.rehearse_shard
        rehearse = {"rank": rank, "world": world}
    # DECDS_BENCH_DIST=1: the process-group path at any N, also N = 1 (a one-rank RCCL group: the only
    # way a one-GPU box runs the N > 1 line's RCCL calls — init, barrier, device all_reduce,
    # all_gather_object — on the device, tests/test_gpu_bench.py)
    dist_on = (world > 1 or os.environ.get("DECDS_BENCH_DIST") == "1") and rehearse is None
    # DECDS_BENCH_BACKEND=gloo is a rehearsal mode for the N > 1 path on a box with fewer GPUs than
    # ranks (ranks share devices round-robin, timing reduced over gloo); the real runs use RCCL.
    backend = os.environ.get("DECDS_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    if dist_on:
        init_group(dist, backend, torch.device("cuda", local), rank, world)

    blob_per_gpu, desc = CONFIGS[args.config]
    n_total = -(-(blob_per_gpu * world) // CS)
    lo, hi = shard_range(n_total, world, rank)
    n = hi - lo
    blob_len_rank = min(blob_per_gpu * world, hi * CS) - lo * CS

    ctx = decds_amd.Context(local)
    stream = torch.cuda.Stream()
    dev = torch.device("cuda", local)
    with torch.cuda.stream(stream):
        src = torch.zeros(n * CS, dtype=torch.uint8, device=dev)
        codec.fill_random_device(ctx, 0xDEC05002, src, nbytes=blob_len_rank, byte_offset=lo * CS, stream=stream)
        coeffs_h = codec.fill_random_host(0xC0EF0002, n * N * K, byte_offset=lo * N * K)
        rng = np.random.default_rng(0x5EED0002 + rank)
        cand_h = np.full((n, N), 0xFF, np.uint8)
        for c in range(n):
            cand_h[c, :K] = rng.permutation(N)[:K]
        coeffs = torch.from_numpy(coeffs_h).to(dev)
        cand = torch.from_numpy(cand_h).to(dev)
        # coded rows in the recommended device layout (include/decds_rlnc.h): pitch 1,048,704 with every
        # payload 128-byte aligned — rlnc's byte-exact full coded pieces, line-aligned encoder stores
        coded, pitch = codec.coded_buffer(n, aligned=not args.packed, device=dev)
        plan = torch.empty(n * 128, dtype=torch.uint8, device=dev)
        verd = torch.empty(n * N, dtype=torch.int8, device=dev)
        status = torch.empty(n, dtype=torch.int32, device=dev)
        out = torch.empty(n * CS, dtype=torch.uint8, device=dev)
    stream.synchronize()

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        codec.encode_batch(ctx, src, n, coeffs, coded, pitch, stream=stream)
        if ev is not None:
            ev[1].record(stream)
        codec.repair_plan_batch(ctx, coded, n, cand, plan, verd, status, pitch, stream=stream)
        if ev is not None:
            ev[2].record(stream)
        codec.decode_batch(ctx, coded, n, plan, out, status, pitch, stream=stream)
        if ev is not None:
            ev[3].record(stream)

    for _ in range(args.warmup):
        step()
    stream.synchronize()
    # clock settle: keep warming (untimed) until the GPU has run the step for SETTLE_S seconds. After
    # a few ms of work the chip is still ramping its clocks: W = 5 alone measured 883 GiB/s against
    # 924 GiB/s after 0.3 s of steps on the same box.
    t_w, settle_steps = time.perf_counter(), 0
    while time.perf_counter() - t_w < args.settle_s and settle_steps < 5000:
        for _ in range(10):
            step()
        settle_steps += 10
        stream.synchronize()
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        step(events[s])
    stream.synchronize()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist_on:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if backend == "gloo" else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    enc_ms = sum(e[0].elapsed_time(e[1]) for e in events) / args.steps
    plan_ms = sum(e[1].elapsed_time(e[2]) for e in events) / args.steps
    dec_ms = sum(e[2].elapsed_time(e[3]) for e in events) / args.steps

    # correctness of the timed work: every repaired chunkset equals its source
    st = status.cpu().numpy()
    assert set(np.unique(st).tolist()) <= {0, 5}, "unexpected repair status"
    for c in np.nonzero(st == 0)[0].tolist():
        assert torch.equal(out[c * CS:(c + 1) * CS], src[c * CS:(c + 1) * CS]), "repaired chunkset %d differs" % c
    n_ready = int((st == 0).sum())
    checked = n_ready  # every ready chunkset's repaired bytes were compared with its source above
    if args.spot_out:
        spots = sorted({0, n // 2, n - 1})
        rows = coded.as_strided((n * N, F), (pitch, 1))
        np.savez(args.spot_out, chunksets=np.array([lo + c for c in spots], np.int64),
                 src=np.stack([src[c * CS:(c + 1) * CS].cpu().numpy() for c in spots]),
                 coeffs=np.stack([coeffs_h[c * N * K:(c + 1) * N * K] for c in spots]),
                 coded=np.stack([rows[c * N:(c + 1) * N].cpu().numpy() for c in spots]),
                 shard_bytes=np.int64(blob_len_rank), pitch=np.int64(pitch))

    if args.digest_out:
        with torch.cuda.stream(stream):
            ddig = torch.empty(n * N * 32, dtype=torch.uint8, device=dev)
            droots = torch.empty(n * 32, dtype=torch.uint8, device=dev)
            dproofs = torch.empty(n * N * 128, dtype=torch.uint8, device=dev)
        codec.commit_batch(ctx, coded, n, ddig, droots, dproofs, first_chunkset_id=lo, pitch=pitch, stream=stream)
        stream.synchronize()
        np.save(args.digest_out, ddig.cpu().numpy().reshape(n * N, 32))
        del ddig, droots, dproofs

    # the next row, timed beside the headline step, never inside it: ChunkSet::new's
    # commitment (BLAKE3 of every coded row + 16-leaf Merkle trees/proofs) over the same coded rows
    commit = None
    if not args.no_commit:
        dig = torch.empty(n * N * 32, dtype=torch.uint8, device=dev)
        roots = torch.empty(n * 32, dtype=torch.uint8, device=dev)
        proofs = torch.empty(n * N * 128, dtype=torch.uint8, device=dev)
        codec.commit_batch(ctx, coded, n, dig, roots, proofs, first_chunkset_id=lo, pitch=pitch, stream=stream)
        cev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
        cev[0].record(stream)
        for s in range(args.steps):
            codec.commit_batch(ctx, coded, n, dig, roots, proofs, first_chunkset_id=lo, pitch=pitch, stream=stream)
            cev[s + 1].record(stream)
        stream.synchronize()
        c_ms = cev[0].elapsed_time(cev[-1]) / args.steps
        # ChunkSet::new as one call (encode + commitment, chunkset.rs:37-63): on rows 16 bytes past a
        # 128-byte boundary the chunk hashing is fused into the encode kernel (rlnc_encode_hash_kernel:
        # every coded 128-byte step hashed from LDS right behind its stores) + commit_fold_kernel
        with torch.cuda.stream(stream):
            mbuf = torch.empty(n * N * codec.CODED_PITCH_ALIGNED + 256, dtype=torch.uint8, device=dev)
            moff = (16 - mbuf.data_ptr()) % 128
            mcoded = mbuf[moff:moff + (n * N - 1) * codec.CODED_PITCH_ALIGNED + F]
            ws = codec.encode_commit_workspace(n, device=dev)
        fused = lambda: codec.encode_commit_batch(ctx, src, n, coeffs, mcoded, dig, roots, proofs, first_chunkset_id=lo,
                                                  pitch=codec.CODED_PITCH_ALIGNED, workspace=ws, stream=stream)
        fused()
        fev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
        fev[0].record(stream)
        for s in range(args.steps):
            fused()
            fev[s + 1].record(stream)
        stream.synchronize()
        f_ms = fev[0].elapsed_time(fev[-1]) / args.steps
        del mbuf, mcoded, ws
        commit = {"kernels": "chunk_digest_kernel + chunkset_merkle_kernel", "ms": round(c_ms, 4),
                  "coded_GBps": round(n * N * F / (c_ms * 1e-3) / 1e9, 1),
                  "blob_GiBps": round(n * CS / GIB / (c_ms * 1e-3), 1), "bound": "valu (BLAKE3 rotates)",
                  "chunkset_new": {"what": "ChunkSet::new = encode + commitment (decds_encode_commit_batch)",
                                   "separate_ms": round(enc_ms + c_ms, 4),
                                   "fused_ms": round(f_ms, 4),
                                   "fused_kernels": "rlnc_encode_hash_kernel + commit_fold_kernel + chunkset_merkle_kernel",
                                   "fused_blob_GiBps": round(n * CS / GIB / (f_ms * 1e-3), 1)}}

    # the kernels' own access-pattern ceilings (decode first: it needs the intact coded rows), then the
    # end-to-end host-memory rate (north_star: written in DESIGN.md §7) — both after the timed region
    patterns, copy_ceiling, e2e, shapes = None, None, None, None
    if world == 1 and not args.no_extras:
        patterns = pattern_ceilings(torch, stream, local, n, src, coeffs, coded, pitch, plan, out, status)
        copy_ceiling = copy_pattern_ceiling(torch, stream, n, coded, pitch, plan, out)
        e2e = end_to_end(ctx)
        if not args.no_api_shapes:
            shapes = api_shapes(ctx)

    # encode batch sweep beside the headline step (north_star: "at batch >= 256"):
    # one HBM-resident 16 GiB blob, encode-only launches of its first n chunksets, HIP events on the
    # bench stream. Single-GPU runs only; never inside the timed step.
    sweep = None
    if world == 1 and not args.no_sweep:
        del out, plan, verd, status
        nmax = max(SWEEP)
        if n >= nmax:  # cfg3: the headline's own 16 GiB blob and coded rows
            big, cbig, obig, bpitch = src, coeffs, coded, pitch
        else:
            with torch.cuda.stream(stream):
                big = torch.empty(nmax * CS, dtype=torch.uint8, device=dev)
                codec.fill_random_device(ctx, 0xDEC05003, big, stream=stream)
                cbig = torch.from_numpy(codec.fill_random_host(0xC0EF0003, nmax * N * K)).to(dev)
                obig, bpitch = codec.coded_buffer(nmax, aligned=not args.packed, device=dev)
        sweep = []
        for ns in SWEEP:
            # warm, then the median of >= 10 launches, each bracketed by its own events
            reps = 10 if ns >= 256 else 20
            t_w = time.perf_counter()
            while time.perf_counter() - t_w < 0.2:
                for _ in range(4):
                    codec.encode_batch(ctx, big, ns, cbig, obig, bpitch, stream=stream)
                stream.synchronize()
            sev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(reps)]
            for r in range(reps):
                sev[r][0].record(stream)
                codec.encode_batch(ctx, big, ns, cbig, obig, bpitch, stream=stream)
                sev[r][1].record(stream)
            stream.synchronize()
            ms = float(np.median([a.elapsed_time(b) for a, b in sev]))
            gbs = ns * (CS + N * F) / (ms * 1e-3) / 1e9
            rec = {"chunksets": ns, "kernel": _lib().decds_encode_kernel_name(ns).decode(),
                   "encode_ms": round(ms, 4), "launches": reps, "encode_GBps": round(gbs, 1),
                   "frac": round(gbs / HBM_PEAK_GBS, 4), "blob_GiBps": round(ns * CS / GIB / (ms * 1e-3), 1)}
            if ns <= 64:
                # beside it (not instead): a stream of back-to-back launches between one event pair, the
                # shape of many small encode calls in a row (each launch's dispatch behind the previous one)
                b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                b0.record(stream)
                for _ in range(4 * reps):
                    codec.encode_batch(ctx, big, ns, cbig, obig, bpitch, stream=stream)
                b1.record(stream)
                stream.synchronize()
                sms = b0.elapsed_time(b1) / (4 * reps)
                rec["stream"] = {"launches": 4 * reps, "encode_ms": round(sms, 4),
                                 "frac": round(ns * (CS + N * F) / (sms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
                # and the same single launches between timing events that skip the system-scope fence
                # (hipEventDisableSystemFence): `frac` above keeps torch's default events, as in every
                # round before; the difference is the events' own L2 writeback + invalidate
                fe = FenceFreeEvents(2 * reps)
                for r in range(reps):
                    fe.record(2 * r, stream)
                    codec.encode_batch(ctx, big, ns, cbig, obig, bpitch, stream=stream)
                    fe.record(2 * r + 1, stream)
                stream.synchronize()
                fms = float(np.median([fe.elapsed_ms(2 * r, 2 * r + 1) for r in range(reps)]))
                fe.close()
                rec["no_system_fence"] = {"launches": reps, "encode_ms": round(fms, 4),
                                          "frac": round(ns * (CS + N * F) / (fms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
            sweep.append(rec)
        del big, cbig, obig

    enc_bytes = n * (CS + N * F)            # algorithmic HBM bytes of one encode launch
    dec_bytes = n_ready * (K * F + CS)      # ... of one decode launch (ready chunksets only)
    enc_gbs = enc_bytes / (enc_ms * 1e-3) / 1e9
    dec_gbs = dec_bytes / (dec_ms * 1e-3) / 1e9
    enc_kernel = _lib().decds_encode_kernel_name(n).decode()
    dec_kernel = _lib().decds_decode_kernel_name(n).decode()
    dominant = enc_kernel if enc_ms >= dec_ms else dec_kernel
    achieved = enc_gbs if dominant == enc_kernel else dec_gbs
    traffic, fused_valu = None, None
    try:
        with open(args.traffic_json) as f:
            tj = json.load(f)
        if tj.get("config") == args.config and dominant in tj.get("kernels", {}):
            traffic = tj["kernels"][dominant]["hbm_bytes_per_launch"]
        if tj.get("config") == args.config:
            fused_valu = tj.get("kernels", {}).get("rlnc_encode_hash_kernel", {}).get("valu")
            if fused_valu:
                fused_valu = dict(fused_valu, source=tj.get("source"))
    except (OSError, ValueError):
        pass
    if commit is not None:
        # the fused ChunkSet::new kernel's own roofline: vector issue (tools/isa_mix.py; PMC of the same
        # command, profiles/): VALU instructions x the built mix's cycles each / (1024 SIMDs x cycles)
        commit["chunkset_new"]["valu_roofline"] = (
            None if not fused_valu else {"kernel": "rlnc_encode_hash_kernel", "bound": "valu", "frac": fused_valu["frac"],
                                         "frac_full_rate": fused_valu["frac_full_rate"],
                                         "cycles_per_valu": fused_valu["cycles_per_valu"],
                                         "insts_per_launch": fused_valu["insts_per_launch"],
                                         "source": fused_valu["source"]})

    # value: blob bytes encoded plus blob bytes repaired (only the chunksets that were ready; the
    # decode kernel skips the rest), halved — encode+repair GiB/s of blob, whole job
    rep_len = sum(min(CS, blob_len_rank - c * CS) for c in np.nonzero(st == 0)[0].tolist())
    # this rank's figures: with N > 1 every rank's are gathered into the line's per_rank (BASELINE
    # configs[4]: per-GPU and whole-node GiB/s), with the device each rank ran on
    mine = rank_record(torch, rank, local, world, lo, hi, blob_len_rank, enc_ms, plan_ms, dec_ms, enc_bytes, dec_bytes,
                       n_ready, checked, rep_len, elapsed, args.steps)
    if dist_on:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
        rep_total = float(sum(r["repaired_blob_bytes"] for r in per_rank))
    else:
        per_rank = [mine]
        rep_total = float(rep_len)
    def pattern_of(nbytes, gbs, key):
        """the kernel's own access-pattern ceiling (pattern_ceilings) and the fraction of it reached"""
        if not patterns or key not in patterns:
            return {}
        p_gbs = nbytes / (patterns[key] * 1e-3) / 1e9
        return {"pattern_GBps": round(p_gbs, 1), "frac_of_pattern": round(gbs / p_gbs, 4)}

    def copy_of(nbytes, gbs):
        """the decode's copy ceiling (copy_pattern_ceiling) and the fraction of it reached"""
        if not copy_ceiling or "decode_ms" not in copy_ceiling:
            return {}
        c_gbs = nbytes / (copy_ceiling["decode_ms"] * 1e-3) / 1e9
        return {"copy_pattern_GBps": round(c_gbs, 1), "frac_of_copy_pattern": round(gbs / c_gbs, 4)}

    if rank == 0 or rehearse:
        # whole-job blob bytes (a rehearsal: this shard's bytes only)
        enc_total = float(blob_len_rank if rehearse else blob_per_gpu * world)
        value = (enc_total + rep_total) / 2 * args.steps / GIB / elapsed
        line = {
            "metric": "RLNC encode+repair GiB/s device-resident, 10MB chunksets; % HBM roofline",
            "value": round(value, 2), "unit": "GiB/s", "n_gpus": 1 if rehearse else world, "steps": args.steps,
            "warmup": args.warmup, "settle_steps": settle_steps, "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (SplitMix64 random blob + coding vectors, seeded)",
            "value_def": "(blob bytes encoded + blob bytes of repaired chunksets) / 2 per second",
            "config": {"workload": args.config + ": " + desc, "chunksets_per_gpu": n,
                       "coded_layout": "pitch %d, payloads %s" % (pitch, "packed" if args.packed else "128-B aligned"),
                       "blob_bytes_per_gpu": blob_per_gpu, "survivors_per_chunkset": K,
                       "parallelism": "chunkset-index shards x%d, no collective" % world},
            "roofline": {"bound": "hbm", "kernel": dominant, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "copy_ceiling": HBM_COPY_GBS, "frac_of_copy": round(achieved / HBM_COPY_GBS, 4),
                         "decode": dict({"kernel": dec_kernel, "achieved": round(dec_gbs, 1),
                                         "frac": round(dec_gbs / HBM_PEAK_GBS, 4),
                                         "bytes_per_launch": dec_bytes, "ms": round(dec_ms, 4)},
                                        **pattern_of(dec_bytes, dec_gbs, "decode_ms"), **copy_of(dec_bytes, dec_gbs)),
                         "encode": dict({"kernel": enc_kernel, "achieved": round(enc_gbs, 1),
                                         "frac": round(enc_gbs / HBM_PEAK_GBS, 4),
                                         "bytes_per_launch": enc_bytes, "ms": round(enc_ms, 4)},
                                        **pattern_of(enc_bytes, enc_gbs, "encode_ms"))},
            "breakdown": {"encode_ms": round(enc_ms, 4), "plan_ms": round(plan_ms, 4), "decode_ms": round(dec_ms, 4),
                          "encode_GBps": round(enc_gbs, 1), "decode_GBps": round(dec_gbs, 1),
                          "encode_blob_GiBps": round(n * CS / GIB / (enc_ms * 1e-3), 1),
                          "repair_blob_GiBps": round(rep_len / GIB / ((plan_ms + dec_ms) * 1e-3), 1),
                          "ready_chunksets": n_ready, "not_ready_chunksets": n - n_ready},
            "rehearsal": None if rehearse is None else dict(rehearse, first_chunkset=lo, chunksets=n,
                                                             blob_bytes=blob_per_gpu * world, shard_bytes=blob_len_rank),
            "commitment": commit,
            "pattern_ceilings": patterns,
            "decode_copy_ceiling": copy_ceiling,
            "end_to_end": e2e,
            "api_shapes": shapes,
            "encode_batch_sweep": sweep,
        }
        line["per_rank"] = per_rank
        if dist_on:
            line["world_size"] = dist.get_world_size()
            line["backend"] = "rccl" if backend == "nccl" else backend
            devs = [r["device_uuid"] or "%s/%d" % (r["host"], r["local_rank"]) for r in per_rank]
            line["scaling_point"] = len(set(devs)) == world
            if not line["scaling_point"]:
                line["scaling_note"] = ("ranks share devices (%d ranks on %d devices): a rehearsal of the N-rank "
                                        "path, not a scaling measurement" % (world, len(set(devs))))
        if world == 1 and not args.no_cpu_baseline:
            cb = line["cpu_baseline"] = cpu_baseline(args.cpu_sample, 0xDEC05002)
            # the GPU/CPU ratio against each CPU figure: `value` (the strongest CPU configuration: the
            # cgroup's 16 CPUs, what rayon's default pool takes on the box) and all usable cores (throttled
            # by that quota on the box) — a reported baseline, not kernel quality
            ac = (cb.get("all_cores") or {}).get("value")
            cb["gpu_over_cpu"] = {"vs_value": round(line["value"] / cb["value"], 2) if cb.get("value") else None,
                                  "vs_all_cores": round(line["value"] / ac, 2) if ac else None}
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

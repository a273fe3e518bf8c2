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
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    p.add_argument("--rehearse-shard", default=None, metavar="R/W", type=shard_arg,
                   help="one process, no process group: run only rank R's shard of a W-GPU job on this GPU "
                        "(cfg5, the 128 GiB blob over 8 GPUs, is --config cfg3 --rehearse-shard R/8)")
    p.add_argument("--spot-out", default=None, metavar="PATH.npz",
                   help="after the timed region, save the source bytes, coding vectors and coded rows of the "
                        "shard's first, middle and last chunkset (the GPU tests check them against the oracle)")
    p.add_argument("--packed", action="store_true",
                   help="coded rows packed at pitch 1,048,587 instead of the recommended 128-B-aligned layout")
    return p.parse_args(argv)


def cpu_threads():
    """the host threads the CPU baseline uses: the CPUs this process may run on, at most 16 (the GPU
    box's CPU share; os.cpu_count() reports the whole machine there)"""
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count() or 1
    return max(1, min(16, avail))


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
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return {"model": model, "cpus_online": os.cpu_count(), "cpus_usable": affinity}


def cpu_baseline(n_sample, seed, repeats=5, cfg2_chunksets=103):
    """The CPU restatement (oracle/, "port") on the host cores: chunkset-parallel encode
    (blob.rs:256-264) + per-chunkset repair from 10 survivors (chunkset.rs:173-208).

    Headline = the strongest restatement: column-blocked GFNI affine multiplies on AVX-512
    (oracle/rlnc_cpu_fast.c; coefficient-only rank + inverse, then one blocked pass for the repair),
    the median of `repeats` runs (each at least 1 s of passes over the sample) with their spread. Beside it (BASELINE.md's plan): the same codec on
    1 thread, on config 2's sample (the 1 GiB blob's 103 chunksets) with all threads and on config 1's
    single chunkset (one thread: the work is chunkset-parallel); one run
    each of the row-pass forms (AVX2 nibble tables; the scalar table-driven loop rlnc 0.4.0 is
    recalled to use). All produce the same bytes (tests/test_oracle.py)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as o
    threads = cpu_threads()
    if n_sample <= 0:
        n_sample = 16 * threads

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
    rows = {}
    o.set_simd(0)
    rows["scalar tables, row passes"] = run(o.blob_encode, o.blob_repair, smp, threads)
    if o.set_simd(1):
        rows["avx2 nibble tables, row passes"] = run(o.blob_encode, o.blob_repair, smp, threads)
    o.set_simd(0)
    extra = {}
    if o.fast_supported():
        head_name = "avx512 gfni affine, column-blocked"
        head = median([run(o.fast_blob_encode, o.fast_blob_repair, smp, threads, min_s=1.0)
                       for _ in range(max(1, repeats))])
        del smp
        smp2 = sample(cfg2_chunksets, seed + 2)
        cfg2_tag = " (config 2: the 1 GiB blob)" if cfg2_chunksets == 103 else ""
        extra["threads_1"] = dict(rnd(run(o.fast_blob_encode, o.fast_blob_repair, smp2, 1, min_s=1.0)), cores=1,
                                  sample="%d chunksets%s, 1 thread" % (cfg2_chunksets, cfg2_tag))
        extra["cfg2"] = dict(rnd(median([run(o.fast_blob_encode, o.fast_blob_repair, smp2, threads, min_s=1.0)
                                         for _ in range(max(1, repeats))])), cores=threads,
                             sample="%d chunksets%s, %d threads" % (cfg2_chunksets, cfg2_tag, threads))
        del smp2
        # config 1: one chunkset (chunkset-parallel, so one thread does all of it), median of repeats
        smp1 = sample(1, seed + 3)
        extra["cfg1"] = dict(rnd(median([run(o.fast_blob_encode, o.fast_blob_repair, smp1, 1, min_s=0.5)
                                         for _ in range(max(1, repeats))])), cores=1,
                             sample="1 chunkset (config 1), 1 thread")
        del smp1
    else:
        head_name = max(rows, key=lambda k: rows[k]["value"])
        head = dict(rows[head_name], runs=1, spread=None)
    return dict({"value": round(head["value"], 2), "unit": "GiB/s", "cores": threads, "kind": "port",
                 "variant": head_name, "median_of": head["runs"], "passes": head.get("passes", 1),
                 "spread": head["spread"],
                 "sample": "%d chunksets (%.0f MiB) encode + repair from 10 survivors, %d threads (chunkset-parallel)"
                           % (n_sample, n_sample * o.CS / 2 ** 20, threads),
                 "encode_gib_s": round(head["encode_gib_s"], 2), "repair_gib_s": round(head["repair_gib_s"], 2),
                 "host": host_cpu(),
                 "other_variants": {k: rnd(v) for k, v in rows.items()}}, **extra)

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
    dist_on = world > 1 and rehearse is None
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
                         "decode": {"kernel": dec_kernel, "achieved": round(dec_gbs, 1),
                                    "frac": round(dec_gbs / HBM_PEAK_GBS, 4),
                                    "bytes_per_launch": dec_bytes, "ms": round(dec_ms, 4)},
                         "encode": {"kernel": enc_kernel, "achieved": round(enc_gbs, 1),
                                    "frac": round(enc_gbs / HBM_PEAK_GBS, 4),
                                    "bytes_per_launch": enc_bytes, "ms": round(enc_ms, 4)}},
            "breakdown": {"encode_ms": round(enc_ms, 4), "plan_ms": round(plan_ms, 4), "decode_ms": round(dec_ms, 4),
                          "encode_GBps": round(enc_gbs, 1), "decode_GBps": round(dec_gbs, 1),
                          "encode_blob_GiBps": round(n * CS / GIB / (enc_ms * 1e-3), 1),
                          "repair_blob_GiBps": round(rep_len / GIB / ((plan_ms + dec_ms) * 1e-3), 1),
                          "ready_chunksets": n_ready, "not_ready_chunksets": n - n_ready},
            "rehearsal": None if rehearse is None else dict(rehearse, first_chunkset=lo, chunksets=n,
                                                             blob_bytes=blob_per_gpu * world, shard_bytes=blob_len_rank),
            "commitment": commit,
            "encode_batch_sweep": sweep,
        }
        if dist_on:
            line["world_size"] = dist.get_world_size()
            line["backend"] = "rccl" if backend == "nccl" else backend
            line["per_rank"] = per_rank
            devs = [r["device_uuid"] or "%s/%d" % (r["host"], r["local_rank"]) for r in per_rank]
            line["scaling_point"] = len(set(devs)) == world
            if not line["scaling_point"]:
                line["scaling_note"] = ("ranks share devices (%d ranks on %d devices): a rehearsal of the N-rank "
                                        "path, not a scaling measurement" % (world, len(set(devs))))
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.cpu_sample, 0xDEC05002)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""Multi-process (world_size 2, gloo, CPU) coverage of the N>1 bench path: chunkset-index sharding
with no data-path collective, each rank encoding/repairing its own shard, and the
max-over-ranks timing reduction bench.py uses. The per-rank compute here is the CPU restatement;
on the GPU node the same shard plan drives the HIP kernels."""
import hashlib
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import bench  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range_partitions():
    for n_total in (1, 2, 3, 103, 205, 1639, 13108):
        for world in (1, 2, 4, 8):
            spans = [bench.shard_range(n_total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n_total
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c and a <= b
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= -(-n_total // world)


def test_cfg5_shard_plan():
    # BASELINE cfg5: a 128 GiB blob over 8 GPUs = bench.py --config cfg3 at N = 8 (and the one-GPU
    # rehearsal --rehearse-shard R/8): 13108 chunksets, 1639 per rank, the last rank 1635 with a final
    # chunkset of 2 MiB of data
    blob_per_gpu, world, cs = bench.CONFIGS["cfg3"][0], 8, 10 << 20
    n_total = -(-(blob_per_gpu * world) // cs)
    assert n_total == 13108
    spans = [bench.shard_range(n_total, world, r) for r in range(world)]
    assert [b - a for a, b in spans] == [1639] * 7 + [1635]
    assert blob_per_gpu * world - (n_total - 1) * cs == 2 << 20


def _worker(rank, world, port, n_total, blob_len, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle as o
    lo, hi = bench.shard_range(n_total, world, rank)
    # each rank generates only its own slice of the global blob (counter-based stream)
    have = min(blob_len, hi * o.CS) - lo * o.CS
    blob = np.zeros((hi - lo) * o.CS, np.uint8)
    blob[:have] = o.fill_random(0xDEC05002, have, lo * o.CS)
    coeffs = o.fill_random(0xC0EF0002, (hi - lo) * o.N * o.K, lo * o.N * o.K)
    coded = o.blob_encode(blob, coeffs, nthreads=2)
    cand = np.stack([np.random.default_rng(c).permutation(o.N) for c in range(lo, hi)]).astype(np.uint8)
    out, status = o.blob_repair(coded, cand, blob.size, nthreads=2)
    assert (status == 0).all() and np.array_equal(out, blob)
    digests = [hashlib.sha256(coded[j].tobytes()).hexdigest() for j in range(coded.shape[0])]
    # bench.py's timing reduction: MAX over ranks
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    gathered = [None] * world
    dist.all_gather_object(gathered, digests)
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, float(t.item()), gathered))


def test_two_rank_sharded_encode_matches_single_process():
    import oracle as o
    n_total, blob_len = 3, 2 * o.CS + 12345      # 3 chunksets, partial last one
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, blob_len, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert all(r[1] == 2.0 for r in res)                       # max over ranks
    gathered = res[0][2]
    assert gathered == res[1][2]
    flat = [d for rank_digests in gathered for d in rank_digests]
    # single-process reference over the whole blob
    blob = o.fill_random(0xDEC05002, blob_len)
    coeffs = o.fill_random(0xC0EF0002, n_total * o.N * o.K)
    coded = o.blob_encode(blob, coeffs, nthreads=4)
    assert flat == [hashlib.sha256(coded[j].tobytes()).hexdigest() for j in range(coded.shape[0])]


def test_rehearse_shard_argument_checked_before_any_device_work():
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # argparse refuses a malformed or out-of-range R/W with a usage error, before torch is imported
    for bad, msg in (("8/8", "needs 0 <= R < W"), ("-1/8", "needs 0 <= R < W"), ("3", "expected R/W"),
                     ("x/8", "expected R/W"), ("1/2/3", "expected R/W")):
        r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--rehearse-shard=" + bad],
                           capture_output=True, text=True, timeout=120, env=dict(os.environ, WORLD_SIZE="1"))
        assert r.returncode == 2 and msg in r.stderr and "Traceback" not in r.stderr, (bad, r.stderr[-500:])
    assert bench.parse(["--rehearse-shard", "7/8"]).rehearse_shard == (7, 8)
    assert bench.parse([]).config == "cfg3"     # BASELINE's largest single-GPU configuration


def test_init_failure_exits_with_a_message_not_a_hang():
    # bench.init_group: a rendezvous that cannot complete (rank 0 of 2, rank 1 never starts) ends the
    # process within the timeout with exit status 3 and a one-line reason — the driver's N-GPU run
    # never hangs on a failed RCCL init (the same path; gloo here, no device)
    import subprocess
    code = ("import sys; sys.path.insert(0, %r); import bench, torch.distributed as dist; "
            "bench.init_group(dist, 'gloo', None, 0, 2, timeout_s=4); print('unreachable')" % ROOT)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE="2", RANK="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr[-1500:])
    assert "rank 0/2: gloo process group init failed" in r.stderr and "unreachable" not in r.stdout


def test_cpu_baseline_thread_counts(monkeypatch):
    # bench.cpu_threads: every usable CPU (the reference's rayon pool on all cores), rayon's default pool
    # (Rust's available_parallelism caps the usable CPUs by the cgroup quota: 16 of 256 on the GPU box,
    # BENCH r07a) and 16; the quota parsed from cgroup v2 cpu.max
    monkeypatch.setattr(bench, "usable_cpus", lambda: 256)
    monkeypatch.setattr(bench, "cgroup_cpus", lambda: 16.0)
    assert bench.cpu_threads() == {"all_cores": 256, "rayon_default": 16, "threads_16": 16}
    monkeypatch.setattr(bench, "cgroup_cpus", lambda: 2.5)
    assert bench.cpu_threads()["rayon_default"] == 3
    monkeypatch.setattr(bench, "cgroup_cpus", lambda: None)
    assert bench.cpu_threads() == {"all_cores": 256, "rayon_default": 256, "threads_16": 16}
    monkeypatch.setattr(bench, "usable_cpus", lambda: 8)
    assert bench.cpu_threads() == {"all_cores": 8, "rayon_default": 8, "threads_16": 8}


def test_cgroup_quota_parsing(monkeypatch, tmp_path):
    import builtins
    real_open = builtins.open
    for text, want in (("1600000 100000\n", 16.0), ("max 100000\n", None), ("garbage\n", None)):
        f = tmp_path / "cpu.max"
        f.write_text(text)
        monkeypatch.setattr(builtins, "open", lambda p, *a, **k: real_open(str(f) if p == "/sys/fs/cgroup/cpu.max" else p, *a, **k))
        assert bench.cgroup_cpus() == want
        monkeypatch.setattr(builtins, "open", real_open)

"""GPU tests of the host-memory paths: the blob pipelines over many batches (every slot reused,
an unready and a repair-failed chunkset in reused slots), registered vs staged caller memory, the
multi-context (multi-device) shard forms, the host registry's rules, and concurrent chunkset-mirror
callers (ChunkSet::new from rayon workers, blob.rs:256-264). Bit-exact against oracle/."""
import os
import threading

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import decds_amd  # noqa: E402
from decds_amd import codec  # noqa: E402
from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N, DecdsError, check, lib  # noqa: E402
import oracle as o  # noqa: E402

pytestmark = pytest.mark.gpu


def _as(buf, src):
    buf[:] = src
    return buf


def _cand_with_failures(coded, coeffs, n, rng, not_ready, broken, short):
    """random arrival orders; chunkset `not_ready` gets 9 candidates; chunksets `broken` and `short`
    get piece 9's boundary marker flipped in every row (row r's payload byte changes by c[r][9] * 0x81:
    linearity), so rlnc's get_decoded_data cuts at the last marker inside the data — none in
    `broken`'s data (the caller removed them): ChunksetRepairingFailed"""
    cand = np.full((n, N), 0xFF, np.uint8)
    for c in range(n):
        cand[c, :] = rng.permutation(N)
    cand[not_ready, 9:] = 0xFF
    coded = coded.copy()
    cv = np.asarray(coeffs, np.uint8).reshape(n, N, K)
    for c in (broken, short):
        for r in range(N):
            coded[c * N + r, F - K] ^= o.gf_mul(int(cv[c, r, 9]), o.MARKER)
    return cand, coded


@pytest.mark.parametrize("n,batch,pinned", [(7, 1, False), (7, 2, True), (7, 2, False), (7, 3, True), (48, 16, True),
                                             (48, 16, False)])
def test_blob_host_paths_reuse_every_slot(ctx, n, batch, pinned):
    # 7 chunksets in batches of 1-3: 3-7 batches over the 3 slots, so every slot is reused; the
    # unready chunkset (4) and the repair-failed one (5) sit in reused slots; last chunkset ragged.
    # 48 in batches of 16: the ramped sizes (blob.cpp batch_sizes: 2, 4, 8, 2, 16, 8, 4, 2, 2)
    blob_len = (n - 1) * CS + 12345
    blob = o.fill_random(0xA5A5 + batch, blob_len).copy()
    part = blob[5 * CS:6 * CS]
    part[part == o.MARKER] ^= 1  # chunkset 5 holds no marker byte
    coeffs = o.fill_random(0xC5C5 + batch, n * N * K)
    hb = []
    if pinned:  # registered caller memory: DMA'd directly
        hb = [decds_amd.HostBuffer(blob_len), decds_amd.HostBuffer(n * N * F), decds_amd.HostBuffer(blob_len)]
        blob_in, coded_out, rep_out = _as(hb[0].array, blob), hb[1].array.reshape(n * N, F), hb[2].array
    else:  # plain memory: staged through the context's page-locked rings
        blob_in, coded_out, rep_out = blob, None, None
    coded = codec.blob_encode_host(ctx, blob_in, coeffs, batch=batch, out=coded_out)
    assert np.array_equal(coded, o.blob_encode(blob, coeffs, nthreads=8))
    cand, coded_bad = _cand_with_failures(coded, coeffs, n, np.random.default_rng(batch), not_ready=4, broken=5,
                                          short=2)
    ref_out, ref_st = o.blob_repair(coded_bad, cand, blob_len, nthreads=8)
    if pinned:
        coded_bad = _as(coded_out, coded_bad)
    out, status = codec.blob_repair_host(ctx, coded_bad, cand, blob_len, batch=batch, out=rep_out)
    assert status.tolist() == [0, 0, 0, 0, 5, 6] + [0] * (n - 6)
    assert ref_st.tolist() == [o.OK, o.OK, o.OK, o.OK, o.NOT_ALL, o.INVALID_DATA] + [o.OK] * (n - 6)
    cut = int(np.nonzero(blob[2 * CS:3 * CS] == o.MARKER)[0][-1])
    for c in range(n):
        lo, hi = c * CS, min(blob_len, (c + 1) * CS)
        if status[c] == 0:
            assert np.array_equal(out[lo:hi], ref_out[lo:hi]), c
            want = blob[lo:hi].copy()
            if c == 2:
                want[cut:] = 0  # cut at the last marker of the data, zeros past it
            assert np.array_equal(out[lo:hi], want), c
        else:
            assert not out[lo:hi].any(), c  # no data for a chunkset that could not be repaired
    for b in hb:
        b.free()


def test_multi_context_shards_match_single(ctx):
    # two contexts on the one device stand in for two GPUs: chunkset shards [0, 3) and [3, 5)
    ctx2 = decds_amd.Context(0)
    n = 5
    blob_len = 4 * CS + 777
    blob = o.fill_random(0xB0B0, blob_len)
    coeffs = o.fill_random(0xB1B1, n * N * K)
    single = codec.blob_encode_host(ctx, blob, coeffs, batch=2)
    multi = codec.blob_encode_host_multi([ctx, ctx2], blob, coeffs, batch=2)
    assert np.array_equal(single, multi)
    cand = np.stack([np.random.default_rng(c).permutation(N) for c in range(n)]).astype(np.uint8)
    cand[1, 9:] = 0xFF
    o1, s1 = codec.blob_repair_host(ctx, single, cand, blob_len, batch=2)
    o2, s2 = codec.blob_repair_host_multi([ctx, ctx2], single, cand, blob_len, batch=2)
    assert s1.tolist() == s2.tolist() == [0, 5, 0, 0, 0]
    assert np.array_equal(o1, o2)
    ok = np.repeat(s1 == 0, CS)[:blob_len]
    assert np.array_equal(o2[ok], blob[ok])
    ctx2.close()


def test_host_registry_rules(ctx):
    L = lib()
    a = np.zeros(3 << 20, np.uint8)
    p = a.ctypes.data
    assert L.decds_host_is_registered(p, a.nbytes) == 0
    check(L.decds_host_register(p, a.nbytes))
    check(L.decds_host_register(p, a.nbytes))                     # same range again: refcounted
    assert L.decds_host_is_registered(p + 100, 1000) == 1
    assert L.decds_host_register(p + 4096, 4096) == -2            # partial overlap refused
    check(L.decds_host_unregister(p))
    assert L.decds_host_is_registered(p, a.nbytes) == 1           # one registration left
    check(L.decds_host_unregister(p))
    assert L.decds_host_is_registered(p, a.nbytes) == 0
    assert L.decds_host_unregister(p) == -2                       # not registered any more
    hb = decds_amd.HostBuffer(5000)
    assert L.decds_host_is_registered(hb.array.ctypes.data, 5000) == 1
    assert L.decds_host_unregister(hb.array.ctypes.data) == -2    # allocations are freed, not unregistered
    assert hb.free() is True
    # a registered caller buffer used by a host path, unregistered in between calls
    blob = o.fill_random(0xC0C0, CS + 5)
    coeffs = o.fill_random(0xC1C1, 2 * N * K)
    codec.host_register(blob)
    got = codec.blob_encode_host(ctx, blob, coeffs)
    codec.host_unregister(blob)
    assert np.array_equal(got, o.blob_encode(blob, coeffs, nthreads=8))


def test_chunkset_mirror_concurrent_callers(ctx):
    # ChunkSet::new / RepairingChunkSet::repair from 8 threads at once, each on its own chunkset:
    # every thread takes its own lane (stream, device buffers, staging)
    T = 8
    results, errors = [None] * T, []

    def worker(t):
        try:
            data = o.fill_random(0xD000 + t, CS)
            coeffs = o.fill_random(0xD100 + t, N * K)
            cs = decds_amd.ChunkSet(ctx, t, data.tobytes(), coeffs.tobytes())
            rcs = decds_amd.RepairingChunkSet(ctx, t, cs.get_root_commitment())
            for j in np.random.default_rng(t).permutation(N)[:K + 2]:
                if rcs.is_ready_to_repair():
                    break
                try:
                    rcs.add_chunk(cs.get_chunk(int(j)))
                except DecdsError as e:
                    assert e.kind == "ChunkDecodingFailed"
            results[t] = (cs, rcs.repair() == data.tobytes())
        except Exception as e:  # surfaced below
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    assert all(r[1] for r in results)
    for t in (0, T - 1):
        data = o.fill_random(0xD000 + t, CS)
        ref = o.chunkset_encode(data, o.fill_random(0xD100 + t, N * K), nthreads=8)
        cs = results[t][0]
        assert all(cs.get_chunk(j).erasure_coded_data == ref[j].tobytes() for j in range(N))


def test_pinned_block_cache_reuse_and_trim(ctx):
    # blocks >= 64 MiB go back to the library's page-locked cache on free and serve the next request
    # of 80-100 % of their size (a Blob's coded store: page-locking costs ~0.25 s per GiB); trim frees them
    import ctypes
    L = lib()
    L.decds_host_cache_trim()
    big = 96 << 20
    p1 = ctypes.c_void_p()
    check(L.decds_host_alloc(big, ctypes.byref(p1)))
    assert L.decds_host_is_registered(p1, big) == 1
    ctypes.memset(p1, 0x5A, big)
    check(L.decds_host_free(p1))
    assert L.decds_host_is_registered(p1, big) == 0
    p2 = ctypes.c_void_p()
    check(L.decds_host_alloc(big - (8 << 20), ctypes.byref(p2)))      # 92 % of the cached block
    assert p2.value == p1.value and L.decds_host_is_registered(p2, big - (8 << 20)) == 1
    check(L.decds_host_free(p2))
    p3 = ctypes.c_void_p()
    check(L.decds_host_alloc(64 << 20, ctypes.byref(p3)))             # 67 %: too small a request for it
    assert p3.value != p1.value
    check(L.decds_host_free(p3))                                       # 64 MiB: cached too
    assert L.decds_host_cache_trim() == big + (64 << 20)
    assert L.decds_host_cache_trim() == 0
    # the blob path into a cached block (holding the previous call's bytes) is still bit-exact
    n = 5
    blob = o.fill_random(0xCAC4E, n * CS - 99)
    coeffs = o.fill_random(0xCAC4F, n * N * K)
    want = o.blob_encode(blob, coeffs, nthreads=8)
    ptrs = []
    for fill in (0xA5, None):
        hb = decds_amd.HostBuffer(n * N * F)                            # 84 MiB: cached when freed
        ptrs.append(hb.array.ctypes.data)
        if fill is not None:
            hb.array[:] = fill
        coded = codec.blob_encode_host(ctx, blob, coeffs, batch=2, out=hb.array.reshape(n * N, F))
        assert np.array_equal(coded, want)
        del coded                       # the returned view would keep the block (HostBuffer.free refuses)
        assert hb.free() is True
    assert ptrs[0] == ptrs[1]
    L.decds_host_cache_trim()


def test_pinned_block_cache_evicts_the_longest_cached_for_a_new_block():
    # a freed block that does not fit beside the cached ones releases the longest-cached blocks instead
    # of being refused (a 4 GiB Blob's 6.4 GiB store behind smaller ones, r09e): a process with a
    # 256 MiB cap frees 96 MiB, then 200 MiB — the 200 MiB block is the one kept
    import subprocess
    import sys
    code = """
import ctypes, sys
sys.path.insert(0, %r)
from decds_amd._capi import lib, check
import decds_amd
ctx = decds_amd.Context(0)
L = lib()
a, b, c, d = (ctypes.c_void_p() for _ in range(4))
check(L.decds_host_alloc(96 << 20, ctypes.byref(a))); check(L.decds_host_free(a))
check(L.decds_host_alloc(200 << 20, ctypes.byref(b))); check(L.decds_host_free(b))
check(L.decds_host_alloc(200 << 20, ctypes.byref(c)))
assert c.value == b.value, "the newest block was not kept"
check(L.decds_host_alloc(96 << 20, ctypes.byref(d)))  # a fresh block: a was released to make room for b
check(L.decds_host_free(c)); check(L.decds_host_free(d))  # d does not fit beside c: c (cached first) goes
freed = L.decds_host_cache_trim()
assert freed == 96 << 20, freed
print("ok")
""" % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, DECDS_PINNED_CACHE_MB="256"))
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


@pytest.mark.parametrize("coalesce", ["0", "1"])
def test_chunkset_new_16_concurrent_callers(ctx, coalesce, monkeypatch):
    # ChunkSet::new from 16 threads at once (Blob::new's rayon loop, blob.rs:256-264). Coalesced, the
    # calls are gathered into shared fused encode + hashing launches with per-request chunkset ids, so
    # unrelated ids in one batch must each get their own digests (chunk.rs:40-46, id =
    # chunkset_id*16+j), root and proofs; every chunkset bit-exact against the oracle, several rounds
    # so batches mix callers
    # coalesce "0": per-call lanes (8 at most, the rest wait); "1": the opt-in coalesced launches
    monkeypatch.setenv("DECDS_CHUNKSET_COALESCE", coalesce)
    T, rounds = 16, 3
    ids = [7 + 1000 * t for t in range(T)]
    errors, results = [], {}

    def worker(t):
        try:
            for rd in range(rounds):
                data = o.fill_random(0xE000 + 97 * t + rd, CS)
                coeffs = o.fill_random(0xE100 + 97 * t + rd, N * K)
                results[(t, rd)] = decds_amd.ChunkSet(ctx, ids[t] + rd, data.tobytes(), coeffs.tobytes())
        except Exception as e:
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    for t in range(T):
        for rd in range(rounds):
            cid = ids[t] + rd
            data = o.fill_random(0xE000 + 97 * t + rd, CS)
            ref = o.chunkset_encode(data, o.fill_random(0xE100 + 97 * t + rd, N * K), nthreads=8)
            cs = results[(t, rd)]
            chunks = [cs.get_chunk(j) for j in range(N)]
            assert all(c.erasure_coded_data == ref[j].tobytes() for j, c in enumerate(chunks)), (t, rd)
            assert all(c.chunk_id == cid * N + j for j, c in enumerate(chunks))
            if (t + rd) % 5 == 0:  # commitment spot checks: root and every proof against the oracle
                leaves = [o.chunk_digest(cid, cid * N + j, ref[j]) for j in range(N)]
                root, proofs = o.merkle(leaves)
                assert cs.get_root_commitment() == root, (t, rd)
                assert [c.proof for c in chunks] == proofs, (t, rd)


def _loaded_hip_runtime():
    """the libamdhip64 this process already loaded (torch's; the library binds to the same one)"""
    import ctypes
    with open("/proc/self/maps") as f:
        paths = {ln.split()[-1] for ln in f if "libamdhip64.so" in ln}
    assert paths, "no HIP runtime mapped"
    return ctypes.CDLL(sorted(paths)[0])  # an already-loaded path: the same handle, no second runtime


def test_launch_reports_an_earlier_pending_hip_error_by_name(ctx):
    # HIP keeps the last error per thread (CUDA semantics): a failed call outside the library leaves
    # it pending, and the hipGetLastError() that reports a launch would return it. The launchers peek
    # before launching (hip_launch_begin, decds_amd/csrc/hip_status.h): the pending error is returned
    # once, named as an earlier call's — round 3's r05b failure read "fused encode + chunk hashing
    # launch: invalid device ordinal (101)" with nothing saying it was not the launch's — and the
    # next call is clean.
    import torch
    hip = _loaded_hip_runtime()
    n = 1
    src = torch.zeros(n * CS, dtype=torch.uint8, device="cuda")
    cv = torch.ones(n * N * K, dtype=torch.uint8, device="cuda")
    dst = torch.empty(n * N * F, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    assert hip.hipSetDevice(12345) == 101          # hipErrorInvalidDevice, left pending on this thread
    with pytest.raises(DecdsError) as e:
        codec.encode_batch(ctx, src, n, cv, dst)
    msg = str(e.value)
    assert e.value.kind == "HipError", msg
    assert "(101)" in msg and "earlier HIP call on this thread" in msg and "outside the library" in msg, msg
    codec.encode_batch(ctx, src, n, cv, dst)       # consumed: the next launch runs
    torch.cuda.synchronize()
    assert dst.view(n * N, F)[:, :K].cpu().numpy().tolist() == [[1] * K] * (n * N)



@pytest.mark.perf
def test_blob_host_rate_does_not_depend_on_caller_streams():
    # The host pipeline's H2D and D2H streams must never share a hardware queue: HIP backs the streams
    # of a priority level with at most 4 queues and puts a new stream on the least-used one, so with
    # equal priorities the two copy directions could land on one queue — and run one after the other —
    # depending on how many streams the process held (blob encode 49-50 ms instead of 38 at 1 GiB with
    # one caller stream alive, r07r). blob.cpp Pipe::init gives them different priority levels. Fresh
    # processes (tools/e2e_bench.py) holding 0, 1 and 2 caller streams when the context is created must
    # encode a 1 GiB blob at one rate. Each case runs twice, interleaved, and keeps its faster run: the
    # queue sharing is a property of the process's stream state (slow on every run), while the box's
    # link can be slow for one whole process now and then (60 ms once in r08e, 36-39 ms otherwise).
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    enc = {}
    for pre in (0, 1, 2, 0, 1, 2):
        r = subprocess.run([sys.executable, os.path.join(root, "tools", "e2e_bench.py"), "--gib", "1", "--batch", "16",
                            "--reps", "4", "--memory", "alloc", "--pre-streams", str(pre)], capture_output=True, text=True,
                           timeout=180, cwd=root)
        assert r.returncode == 0, r.stderr[-2000:]
        d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{"blob')][-1])
        assert d["ready"] == d["chunksets"] and d["spot_check_ok"]
        enc[pre] = min(enc.get(pre, 1e9), d["encode_median_s"])
    print("encode medians (s), faster of two processes, with 0, 1, 2 caller streams:", enc)
    assert max(enc.values()) < 1.15 * min(enc.values()), enc

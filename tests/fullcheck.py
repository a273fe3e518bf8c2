"""Every coded row of a full-size launch against the oracle (test infrastructure).

The oracle's coded rows of a synthetic blob — SplitMix64 bytes (seed, global byte offset) zero-padded to
whole chunksets (blob.rs:252-254), coding vectors from their own SplitMix64 stream — are produced in
batches of chunksets on a pool of host threads (the oracle's C calls release the GIL), with the
column-blocked GFNI restatement where the CPU has it (the same bytes as the scalar restatement,
tests/test_oracle.py) and the scalar one otherwise. Two ways to compare them with the device:

* compare_device_rows: the device rows themselves, copied back batch by batch (in-process tests);
* shard_oracle_digests: chunk.rs:40-46 digests of the oracle's rows, for a process that can only hand
  back the device rows' digests (bench.py --digest-out: decds_commit_batch over its coded rows). Equal
  digests of a collision-resistant hash mean equal rows.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

import oracle as o


def host_threads():
    """worker threads for the host side: the CPUs this process may use, at most 16 (the GPU box grants 16)"""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def oracle_rows(blob_seed, coeff_seed, blob_len, c0, c1):
    """the oracle's (16 * (c1 - c0), F) coded rows of chunksets [c0, c1) of the synthetic blob"""
    nb = c1 - c0
    have = max(0, min(blob_len, c1 * o.CS) - c0 * o.CS)
    src = np.zeros(nb * o.CS, np.uint8)
    if have:
        src[:have] = o.fill_random(blob_seed, have, c0 * o.CS)
    cv = o.fill_random(coeff_seed, nb * o.N * o.K, c0 * o.N * o.K)
    enc = o.fast_blob_encode if o.fast_supported() else o.blob_encode
    return enc(src, cv, nthreads=1)


def _batches(lo, hi, batch):
    return [(c, min(c + batch, hi)) for c in range(lo, hi, batch)]


def _pipelined(jobs, fn, consume, threads):
    """fn(job) on the pool, consume(job, result) in job order, at most 2 x threads results held at once"""
    with ThreadPoolExecutor(threads) as ex:
        pending = []
        it = iter(jobs)
        for job in it:
            pending.append((job, ex.submit(fn, job)))
            if len(pending) >= 2 * threads:
                j, f = pending.pop(0)
                consume(j, f.result())
        for j, f in pending:
            consume(j, f.result())


def compare_device_rows(rows_dev, lo, hi, blob_seed, coeff_seed, blob_len, batch=16, threads=None):
    """Every byte of the device's coded rows of chunksets [lo, hi) (rows_dev: a (16 * (hi - lo), F) view of
    any pitch, row 0 = chunkset lo's first row) equals the oracle's; returns the number of rows compared.
    Raises AssertionError naming the first differing chunkset."""
    threads = threads or host_threads()
    count = [0]

    def consume(job, ref):
        c0, c1 = job
        got = np.ascontiguousarray(rows_dev[(c0 - lo) * o.N:(c1 - lo) * o.N].cpu().numpy())
        assert got.shape == ref.shape, (got.shape, ref.shape)
        words = lambda a: a.reshape(-1).view(np.uint64)  # 16 rows x F bytes is a multiple of 8
        if not np.array_equal(words(got), words(ref)):
            for c in range(c0, c1):
                a, b = got[(c - c0) * o.N:(c - c0 + 1) * o.N], ref[(c - c0) * o.N:(c - c0 + 1) * o.N]
                if not np.array_equal(a, b):
                    rows = [j for j in range(o.N) if not np.array_equal(a[j], b[j])]
                    raise AssertionError("chunkset %d: coded rows %s differ from the oracle's" % (c, rows))
        count[0] += ref.shape[0]

    _pipelined(_batches(lo, hi, batch), lambda j: oracle_rows(blob_seed, coeff_seed, blob_len, *j), consume, threads)
    return count[0]


def shard_oracle_digests(lo, hi, blob_seed, coeff_seed, blob_len, batch=8, threads=None):
    """(16 * (hi - lo), 32) chunk digests (chunk.rs:40-46, global chunk ids) of the oracle's coded rows of
    chunksets [lo, hi)"""
    threads = threads or host_threads()
    out = np.empty(((hi - lo) * o.N, 32), np.uint8)

    def work(job):
        c0, c1 = job
        return o.chunk_digest_rows(oracle_rows(blob_seed, coeff_seed, blob_len, c0, c1), c0 * o.N)

    def consume(job, dig):
        out[(job[0] - lo) * o.N:(job[1] - lo) * o.N] = dig

    _pipelined(_batches(lo, hi, batch), work, consume, threads)
    return out

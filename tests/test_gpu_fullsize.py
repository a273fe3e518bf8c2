"""BASELINE config 3/4 at full size on one GPU: a 16 GiB blob (1639 chunksets, the last one holding
4 MiB of data) encoded in one batch, repaired from exactly 10 random survivors per chunkset, and
committed (separately and fused into the encode) + validated (rows f1, f2). Every coded row of the
1639-chunkset launches is compared byte for byte with the oracle's, and every chunk digest with the
BLAKE3 restatement's digest of the oracle's row (tests/fullcheck.py); the other
checks are size-independent properties (decode∘encode = id, rank-deficient sets reported
not-ready exactly where the oracle's rank test says so, every row's proof verifies, a flipped byte
does not)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from decds_amd import codec  # noqa: E402
from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N  # noqa: E402
import oracle as o  # noqa: E402
from fullcheck import compare_device_rows, shard_oracle_digests  # noqa: E402

pytestmark = pytest.mark.gpu


def _rank_of(cvs, cand):
    """the oracle decoder's rank after the candidates' coefficient prefixes (chunkset.rs:173-184)"""
    dec = o.Decoder(3, K)
    for r in cand:
        if r == 0xFF or dec.is_already_decoded():
            break
        dec.decode(np.concatenate([cvs[r], np.zeros(3, np.uint8)]))
    return dec.rank()


def test_cfg3_16gib_encode_repair_commit_validate(ctx):
    blob_len = 16 << 30
    n = -(-blob_len // CS)
    assert n == 1639
    src = torch.zeros(n * CS, dtype=torch.uint8, device="cuda")
    codec.fill_random_device(ctx, 0xDEC05003, src, nbytes=blob_len)
    coeffs = o.fill_random(0xC0EF0003, n * N * K)
    coded = torch.empty(n * N * F, dtype=torch.uint8, device="cuda")
    codec.encode_batch(ctx, src, n, torch.from_numpy(coeffs).cuda(), coded)
    torch.cuda.synchronize()
    # every one of the 26,224 coded rows (packed layout) against the oracle's, byte for byte
    assert compare_device_rows(coded.view(n * N, F), 0, n, 0xDEC05003, 0xC0EF0003, blob_len) == n * N
    # and one chunkset through the oracle's scalar chunkset path on the device's own source bytes
    c = 820
    ref = o.chunkset_encode(src[c * CS:(c + 1) * CS].cpu().numpy(), coeffs[c * 160:(c + 1) * 160], nthreads=8)
    assert np.array_equal(coded[c * N * F:(c + 1) * N * F].cpu().numpy().reshape(N, F), ref), c

    # repair from exactly 10 random survivors per chunkset (cfg4)
    rng = np.random.default_rng(0x5EED0003)
    cand = np.full((n, N), 0xFF, np.uint8)
    for c in range(n):
        cand[c, :K] = rng.permutation(N)[:K]
    plan = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(n * N, dtype=torch.int8, device="cuda")
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    out = torch.empty(n * CS, dtype=torch.uint8, device="cuda")
    codec.repair_batch(ctx, coded, n, torch.from_numpy(cand).cuda(), plan, verd, out, status)
    st = status.cpu().numpy()
    cv = coeffs.reshape(n, N, K)
    expect = np.array([0 if _rank_of(cv[c], cand[c]) == K else 5 for c in range(n)])
    assert np.array_equal(st, expect)
    assert 0 < int((st == 5).sum()) < 30     # ~0.39 % of 1639 are rank-deficient
    for c in np.nonzero(st == 0)[0].tolist():
        assert torch.equal(out[c * CS:(c + 1) * CS], src[c * CS:(c + 1) * CS]), c
    del out

    # commitment of every coded row, then the blob-level tree and validation of all 26,224 rows
    dig = torch.empty(n * N * 32, dtype=torch.uint8, device="cuda")
    roots = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    proofs = torch.empty(n * N * 128, dtype=torch.uint8, device="cuda")
    codec.commit_batch(ctx, coded, n, dig, roots, proofs)
    torch.cuda.synchronize()
    # the fused ChunkSet::new at full size (rows 16 bytes past a 128-byte boundary): the same coded
    # bytes, digests, roots and proofs as encode + commit
    from decds_amd._capi import CODED_PITCH_ALIGNED as P
    mbuf = torch.empty(n * N * P + 256, dtype=torch.uint8, device="cuda")
    off = (16 - mbuf.data_ptr()) % 128
    mcoded = mbuf[off:off + (n * N - 1) * P + F]
    fo = [torch.empty_like(t) for t in (dig, roots, proofs)]
    codec.encode_commit_batch(ctx, src, n, torch.from_numpy(coeffs).cuda(), mcoded, *fo, pitch=P)
    torch.cuda.synchronize()
    for a, b in zip(fo, (dig, roots, proofs)):
        assert torch.equal(a, b)
    assert torch.equal(mcoded.as_strided((n * N, F), (P, 1)), coded.view(n * N, F))
    del mbuf, mcoded, fo, src
    d = dig.cpu().numpy()
    for row in (0, 1, 13107, n * N - 1):
        piece = coded[row * F:(row + 1) * F].cpu().numpy()
        assert d[row * 32:(row + 1) * 32].tobytes() == o.chunk_digest(row // N, row, piece), row
    # every row's digest (chunk.rs:40-46; the fused and unfused paths gave the same, above) against the
    # BLAKE3 restatement's digest of the oracle's own coded row
    ref = shard_oracle_digests(0, n, 0xDEC05003, 0xC0EF0003, blob_len)
    bad = np.nonzero((d.reshape(n * N, 32) != ref).any(axis=1))[0]
    assert bad.size == 0, "digests differ from the oracle's: rows %s" % bad[:16].tolist()
    leaves = [d[((n - 1) * N + j) * 32:((n - 1) * N + j + 1) * 32].tobytes() for j in range(N)]
    r = roots.cpu().numpy()
    assert r[(n - 1) * 32:n * 32].tobytes() == o.merkle(leaves)[0]
    cs_roots = [r[c * 32:(c + 1) * 32].tobytes() for c in range(n)]
    blob_root, blob_proofs = o.merkle(cs_roots)
    depth = len(blob_proofs[0])
    assert depth == 11
    pr = proofs.cpu().numpy().reshape(n * N, 128)
    full = np.empty((n * N, 4 + depth, 32), np.uint8)
    full[:, :4] = pr.reshape(n * N, 4, 32)
    bp = np.frombuffer(b"".join(b"".join(p) for p in blob_proofs), np.uint8).reshape(n, depth, 32)
    full[:, 4:] = np.repeat(bp, N, axis=0)
    ids = torch.tensor([(row // N, row) for row in range(n * N)], dtype=torch.int64).cuda()
    fp = torch.from_numpy(full.reshape(-1)).cuda()
    vdig = torch.empty(n * N * 32, dtype=torch.uint8, device="cuda")
    valid = torch.empty(n * N, dtype=torch.uint8, device="cuda")
    broot = torch.from_numpy(np.frombuffer(blob_root, np.uint8).copy()).cuda()
    codec.validate_batch(ctx, coded, n * N, ids, fp, 4 + depth, roots, n, vdig, valid, blob_root=broot)
    torch.cuda.synchronize()
    assert int(valid.sum()) == n * N
    assert torch.equal(vdig, dig)
    # one flipped payload byte invalidates exactly its row
    coded[777 * F + 4321] ^= 1
    codec.validate_batch(ctx, coded, n * N, ids, fp, 4 + depth, roots, n, vdig, valid, blob_root=broot)
    v = valid.cpu().numpy()
    assert int(v.sum()) == n * N - 1 and v[777] == 0


def test_payload_aligned_layout_at_the_bench_batches(ctx):
    # the layout bench.py and the encode sweep time (pitch 1,048,704, payloads 128-byte aligned) at the
    # north-star batches: launches of 256 (first / middle / last chunkset) and of all 1639 chunksets
    # (every coded row) of a 16 GiB blob bit-exact against the oracle; then every chunkset of the 1639 repaired
    # from 10 survivors equals its source
    blob_len = 16 << 30
    n = -(-blob_len // CS)
    src = torch.zeros(n * CS, dtype=torch.uint8, device="cuda")
    codec.fill_random_device(ctx, 0xDEC05004, src, nbytes=blob_len)
    coeffs = o.fill_random(0xC0EF0004, n * N * K)
    dco = torch.from_numpy(coeffs).cuda()
    coded, pitch = codec.coded_buffer(n)
    assert pitch == codec.CODED_PITCH_ALIGNED and (coded.data_ptr() + K) % 128 == 0
    rows = coded.as_strided((n * N, F), (pitch, 1))
    for nb in (256, n):
        coded.fill_(0xA5)
        codec.encode_batch(ctx, src, nb, dco, coded, pitch)
        torch.cuda.synchronize()
        if nb == n:  # the whole launch: every coded row against the oracle's
            assert compare_device_rows(rows, 0, n, 0xDEC05004, 0xC0EF0004, blob_len) == n * N
        else:
            for c in sorted({0, nb // 2, nb - 1}):
                ref = o.chunkset_encode(src[c * CS:(c + 1) * CS].cpu().numpy(), coeffs[c * 160:(c + 1) * 160], nthreads=8)
                assert np.array_equal(rows[c * N:(c + 1) * N].cpu().numpy(), ref), (nb, c)
        if nb < n:  # nothing past the batch was written
            assert int(rows[nb * N].cpu()[0]) == 0xA5 and int(rows[n * N - 1].cpu()[-1]) == 0xA5
    rng = np.random.default_rng(0x5EED0004)
    cand = np.full((n, N), 0xFF, np.uint8)
    for c in range(n):
        cand[c, :K] = rng.permutation(N)[:K]
    plan = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(n * N, dtype=torch.int8, device="cuda")
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    out = torch.empty(n * CS, dtype=torch.uint8, device="cuda")
    codec.repair_batch(ctx, coded, n, torch.from_numpy(cand).cuda(), plan, verd, out, status, pitch=pitch)
    st = status.cpu().numpy()
    assert set(np.unique(st).tolist()) <= {0, 5} and int((st == 0).sum()) > n - 30
    for c in np.nonzero(st == 0)[0].tolist():
        assert torch.equal(out[c * CS:(c + 1) * CS], src[c * CS:(c + 1) * CS]), c

"""GPU parity of the commitment kernels against the CPU restatement: BLAKE3 chunk
digests of every coded row (chunk.rs:40-46), chunkset Merkle roots (chunkset.rs:54-57) and the
16 inclusion proofs (chunkset.rs:59-63), bit-exact."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from decds_amd import codec  # noqa: E402
from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N  # noqa: E402
import oracle as o  # noqa: E402

pytestmark = pytest.mark.gpu


def test_commit_batch_matches_oracle(ctx):
    n, first = 3, 41
    data = o.fill_random(0xC0117, n * CS)
    coeffs = o.fill_random(0xC0118, n * N * K)
    coded = torch.empty(n * N * F, dtype=torch.uint8, device="cuda")
    codec.encode_batch(ctx, torch.from_numpy(data).cuda(), n, torch.from_numpy(coeffs).cuda(), coded)
    dig = torch.empty(n * N * 32, dtype=torch.uint8, device="cuda")
    roots = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    proofs = torch.empty(n * N * 4 * 32, dtype=torch.uint8, device="cuda")
    codec.commit_batch(ctx, coded, n, dig, roots, proofs, first_chunkset_id=first)
    torch.cuda.synchronize()
    rows = coded.cpu().numpy().reshape(n * N, F)
    d, r, p = dig.cpu().numpy(), roots.cpu().numpy(), proofs.cpu().numpy()
    for c in range(n):
        cs_id = first + c
        leaves = [o.chunk_digest(cs_id, cs_id * N + j, rows[c * N + j]) for j in range(N)]
        for j in range(N):
            assert d[(c * N + j) * 32:(c * N + j + 1) * 32].tobytes() == leaves[j], (c, j)
        root, pr = o.merkle(leaves)
        assert r[c * 32:(c + 1) * 32].tobytes() == root
        for j in range(N):
            got = [p[((c * N + j) * 4 + k) * 32:((c * N + j) * 4 + k + 1) * 32].tobytes() for k in range(4)]
            assert got == pr[j]
            assert o.merkle_verify(j, leaves[j], got, root)


def test_commit_batch_pitch(ctx):
    n, pitch = 1, F + 301
    data = o.fill_random(0xC0119, CS)
    coeffs = o.fill_random(0xC011A, N * K)
    coded = torch.empty((N - 1) * pitch + F, dtype=torch.uint8, device="cuda")
    codec.encode_batch(ctx, torch.from_numpy(data).cuda(), n, torch.from_numpy(coeffs).cuda(), coded, pitch)
    dig = torch.empty(N * 32, dtype=torch.uint8, device="cuda")
    roots = torch.empty(32, dtype=torch.uint8, device="cuda")
    proofs = torch.empty(N * 4 * 32, dtype=torch.uint8, device="cuda")
    codec.commit_batch(ctx, coded, n, dig, roots, proofs, pitch=pitch)
    torch.cuda.synchronize()
    h = coded.cpu().numpy()
    leaves = [o.chunk_digest(0, j, h[j * pitch:j * pitch + F]) for j in range(N)]
    assert dig.cpu().numpy().tobytes() == b"".join(leaves)
    assert roots.cpu().numpy().tobytes() == o.merkle(leaves)[0]


def _aligned_rows(n, row_offset):
    """n*16 coded rows at the aligned pitch, the first row starting row_offset bytes past a 128-byte
    boundary"""
    from decds_amd._capi import CODED_PITCH_ALIGNED as P
    buf = torch.empty(n * N * P + 256, dtype=torch.uint8, device="cuda")
    off = (row_offset - buf.data_ptr()) % 128
    return buf[off:off + (n * N - 1) * P + F], P


@pytest.mark.parametrize("row_offset,first", [(16, 1000), (48, 1000), (0, (1 << 33) + 5), (118, 1000)])
def test_encode_commit_fused_matches_oracle(ctx, row_offset, first):
    # ChunkSet::new (chunkset.rs:37-63) in one call: rows at 16 mod 16 take the fused kernel (chunk
    # hashing from LDS right behind the encode + commit_fold_kernel), 118 the unfused fallback; both
    # must give the oracle's coded rows, digests, roots and proofs (ids above 2^32: both id words)
    n = 3
    data = o.fill_random(0xC011B + row_offset, n * CS)
    coeffs = o.fill_random(0xC011C + row_offset, n * N * K)
    coded, pitch = _aligned_rows(n, row_offset)
    dig = torch.empty(n * N * 32, dtype=torch.uint8, device="cuda")
    roots = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    proofs = torch.empty(n * N * 4 * 32, dtype=torch.uint8, device="cuda")
    codec.encode_commit_batch(ctx, torch.from_numpy(data).cuda(), n, torch.from_numpy(coeffs).cuda(), coded, dig, roots,
                              proofs, first_chunkset_id=first, pitch=pitch)
    torch.cuda.synchronize()
    h = coded.cpu().numpy()
    d, r, p = dig.cpu().numpy(), roots.cpu().numpy(), proofs.cpu().numpy()
    for c in range(n):
        ref = o.chunkset_encode(data[c * CS:(c + 1) * CS], coeffs[c * N * K:(c + 1) * N * K], nthreads=8)
        rows = [h[(c * N + j) * pitch:(c * N + j) * pitch + F] for j in range(N)]
        for j in range(N):
            assert np.array_equal(rows[j], ref[j]), (c, j)
        cs_id = first + c
        leaves = [o.chunk_digest(cs_id, cs_id * N + j, rows[j]) for j in range(N)]
        assert d[c * N * 32:(c + 1) * N * 32].tobytes() == b"".join(leaves), c
        root, pr = o.merkle(leaves)
        assert r[c * 32:(c + 1) * 32].tobytes() == root
        for j in range(N):
            got = [p[((c * N + j) * 4 + k) * 32:((c * N + j) * 4 + k + 1) * 32].tobytes() for k in range(4)]
            assert got == pr[j]


def test_encode_commit_fused_large_batch_matches_unfused(ctx):
    # 103 chunksets (cfg2): every XCD eighth of the fused launch; the fused commitment must equal the
    # separate commit kernels over the same rows, and the rows the plain encode's
    n, first = 103, 7
    src = torch.empty(n * CS, dtype=torch.uint8, device="cuda")
    codec.fill_random_device(ctx, 0xC011D, src)
    cv = torch.from_numpy(codec.fill_random_host(0xC011E, n * N * K)).cuda()
    coded, pitch = _aligned_rows(n, 16)
    out = [torch.empty(s, dtype=torch.uint8, device="cuda") for s in (n * N * 32, n * 32, n * N * 128)]
    codec.encode_commit_batch(ctx, src, n, cv, coded, *out, first_chunkset_id=first, pitch=pitch)
    ref = [torch.empty_like(t) for t in out]
    codec.commit_batch(ctx, coded, n, *ref, first_chunkset_id=first, pitch=pitch)
    plain, ppitch = _aligned_rows(n, 118)
    codec.encode_batch(ctx, src, n, cv, plain, ppitch)
    torch.cuda.synchronize()
    for a, b in zip(out, ref):
        assert torch.equal(a, b)
    a = coded.as_strided((n * N, F), (pitch, 1))
    b = plain.as_strided((n * N, F), (ppitch, 1))
    assert torch.equal(a, b)

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

"""GPU parity of the commitment-carrying chunkset mirror (chunkset.rs:37-105, 129-157) and of the
batched repair-side validation (BlobHeader::validate_chunk, blob.rs:211-215;
chunk.rs:88-110; merkle_tree.rs:131-146) against the BLAKE3/Merkle restatement in oracle/."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import decds_amd  # noqa: E402
from decds_amd import codec  # noqa: E402
from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N, DecdsError  # noqa: E402
import oracle as o  # noqa: E402

pytestmark = pytest.mark.gpu


def _chunkset(ctx, cs_id, seed):
    data = o.fill_random(seed, CS)
    coeffs = o.fill_random(seed + 1, N * K)
    return data, decds_amd.ChunkSet(ctx, cs_id, data.tobytes(), coeffs.tobytes())


def test_chunkset_new_commitment_matches_oracle(ctx):
    cs_id = 7
    data, cs = _chunkset(ctx, cs_id, 0xA11)
    chunks = [cs.get_chunk(j) for j in range(N)]
    leaves = [o.chunk_digest(cs_id, cs_id * N + j, np.frombuffer(c.erasure_coded_data, np.uint8))
              for j, c in enumerate(chunks)]
    root, proofs = o.merkle(leaves)
    assert cs.get_root_commitment() == root
    for j, c in enumerate(chunks):
        assert c.get_global_chunk_id() == cs_id * N + j and c.get_local_chunk_id() == j
        assert c.digest() == leaves[j]
        assert c.get_proof() == proofs[j]
        assert c.validate_inclusion_in_chunkset(root)
        assert not c.validate_inclusion_in_chunkset(bytes(32))
    # chunkset.rs:98-102: an empty blob proof is a no-op, a non-empty one is appended to every chunk
    cs.append_blob_inclusion_proof([])
    assert len(cs.get_chunk(3).get_proof()) == 4
    extra = [bytes([i]) * 32 for i in range(3)]
    cs.append_blob_inclusion_proof(extra)
    assert cs.get_chunk(3).get_proof() == proofs[3] + extra


def test_repairing_chunkset_add_chunk_validates_proofs(ctx):
    """chunkset.rs:151-157 and the reference's own test shape (chunkset.rs:300-436): valid chunks are
    accepted, a tampered chunk or proof is InvalidProofInChunk, a chunk of another chunkset fails
    its proof against this commitment, and the repaired bytes equal the original."""
    data, cs = _chunkset(ctx, 3, 0xB22)
    _, other = _chunkset(ctx, 4, 0xC33)
    root = cs.get_root_commitment()
    rcs = decds_amd.RepairingChunkSet(ctx, 3, root)

    bad = cs.get_chunk(0)
    flipped = bytearray(bad.erasure_coded_data)
    flipped[12345] ^= 1
    bad.erasure_coded_data = bytes(flipped)
    with pytest.raises(DecdsError) as e:
        rcs.add_chunk(bad)
    assert e.value.kind == "InvalidProofInChunk"

    bad = cs.get_chunk(1)
    bad.proof[2] = bytes(32)
    with pytest.raises(DecdsError) as e:
        rcs.add_chunk(bad)
    assert e.value.kind == "InvalidProofInChunk"

    bad = cs.get_chunk(2)
    bad.proof = bad.proof[:3]  # shorter than PROOF_SIZE
    with pytest.raises(DecdsError) as e:
        rcs.add_chunk(bad)
    assert e.value.kind == "InvalidProofInChunk"

    with pytest.raises(DecdsError) as e:
        rcs.add_chunk(other.get_chunk(0))
    assert e.value.kind == "InvalidProofInChunk"

    order = np.random.default_rng(5).permutation(N)
    added = 0
    for j in order:
        if rcs.is_ready_to_repair():
            with pytest.raises(DecdsError) as e:
                rcs.add_chunk(cs.get_chunk(int(j)))
            assert e.value.kind == "ChunksetReadyToRepair"
            break
        try:
            rcs.add_chunk(cs.get_chunk(int(j)))
            added += 1
        except DecdsError as err:  # a dependent chunk (about 0.4 % per chunkset)
            assert err.kind == "ChunkDecodingFailed"
    assert rcs.is_ready_to_repair() and added == K
    assert rcs.repair() == data.tobytes()


def test_repairing_chunkset_without_commitment_refuses_add_chunk(ctx):
    _, cs = _chunkset(ctx, 0, 0xD44)
    rcs = decds_amd.RepairingChunkSet(ctx, 0)
    with pytest.raises(DecdsError) as e:
        rcs.add_chunk(cs.get_chunk(0))
    assert e.value.kind == "InvalidArgument"
    rcs.add_chunk_unvalidated(cs.get_chunk(0))  # the unvalidated path needs no commitment


def _blob_setup(ctx, n):
    data = o.fill_random(0xE55, n * CS)
    coeffs = o.fill_random(0xE56, n * N * K)
    coded = torch.empty(n * N * F, dtype=torch.uint8, device="cuda")
    codec.encode_batch(ctx, torch.from_numpy(data).cuda(), n, torch.from_numpy(coeffs).cuda(), coded)
    dig = torch.empty(n * N * 32, dtype=torch.uint8, device="cuda")
    roots = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    proofs = torch.empty(n * N * 128, dtype=torch.uint8, device="cuda")
    codec.commit_batch(ctx, coded, n, dig, roots, proofs)
    torch.cuda.synchronize()
    r = roots.cpu().numpy()
    cs_roots = [r[c * 32:(c + 1) * 32].tobytes() for c in range(n)]
    blob_root, blob_proofs = o.merkle(cs_roots)  # blob.rs:266-273
    p = proofs.cpu().numpy()
    full = []  # per row: 4 chunkset-level hashes + the chunkset's blob-level path (chunkset.rs:98-102)
    for row in range(n * N):
        cp = [p[(row * 4 + k) * 32:(row * 4 + k + 1) * 32].tobytes() for k in range(4)]
        full.append(cp + blob_proofs[row // N])
    return coded, roots, cs_roots, blob_root, full


def test_validate_batch_matches_reference_semantics(ctx):
    n = 3
    coded, roots, cs_roots, blob_root, full = _blob_setup(ctx, n)
    plen = len(full[0])
    assert plen == 4 + 2
    host = coded.cpu().numpy().reshape(n * N, F)
    # received rows: a shuffled subset, plus tampered copies
    rng = np.random.default_rng(9)
    rows = rng.permutation(n * N)[:20].tolist()
    recv, ids, prf, expect = [], [], [], []
    for r in rows:
        recv.append(host[r]); ids.append((r // N, r)); prf.append(full[r]); expect.append(1)
    t = host[rows[0]].copy(); t[777] ^= 0x40                       # flipped payload byte
    recv.append(t); ids.append((rows[0] // N, rows[0])); prf.append(full[rows[0]]); expect.append(0)
    r1 = rows[1]                                                   # wrong claimed chunk id
    recv.append(host[r1]); ids.append((r1 // N, r1 ^ 1)); prf.append(full[r1]); expect.append(0)
    r2 = rows[2]                                                   # chunkset id out of range
    recv.append(host[r2]); ids.append((n + 5, r2)); prf.append(full[r2]); expect.append(0)
    r3 = rows[3]                                                   # corrupted blob-level hash
    recv.append(host[r3]); ids.append((r3 // N, r3)); prf.append(full[r3][:5] + [bytes(32)]); expect.append(0)
    m = len(recv)
    dev_rows = torch.from_numpy(np.stack(recv)).cuda().reshape(-1)
    dev_ids = torch.tensor(ids, dtype=torch.int64).cuda()
    dev_prf = torch.from_numpy(np.frombuffer(b"".join(b"".join(p) for p in prf), np.uint8).copy()).cuda()
    dig = torch.empty(m * 32, dtype=torch.uint8, device="cuda")
    valid = torch.empty(m, dtype=torch.uint8, device="cuda")
    broot = torch.from_numpy(np.frombuffer(blob_root, np.uint8).copy()).cuda()
    codec.validate_batch(ctx, dev_rows, m, dev_ids, dev_prf, plen, roots, n, dig, valid, blob_root=broot)
    torch.cuda.synchronize()
    v = valid.cpu().numpy().tolist()
    assert v == expect
    d = dig.cpu().numpy()
    for i in (0, m - 4, m - 3):  # digest under the claimed ids, as Chunk::digest would compute it
        assert d[i * 32:(i + 1) * 32].tobytes() == o.chunk_digest(ids[i][0], ids[i][1], recv[i])
    # the reference's own checks, row by row (chunk.rs:88-110, blob.rs:211-215)
    for i in range(m):
        leaf = o.chunk_digest(ids[i][0], ids[i][1], recv[i])
        ref = (o.merkle_verify(ids[i][1], leaf, prf[i], blob_root) and ids[i][0] < n
               and o.merkle_verify(ids[i][1] % N, leaf, prf[i][:4], cs_roots[ids[i][0]]))
        assert v[i] == int(ref), i
    # without the blob root only the chunkset-level proof is checked: the blob-hash corruption passes
    codec.validate_batch(ctx, dev_rows, m, dev_ids, dev_prf, plen, roots, n, dig, valid, blob_root=None)
    torch.cuda.synchronize()
    assert valid.cpu().numpy().tolist() == expect[:-1] + [1]
    # a wrong blob root rejects everything
    codec.validate_batch(ctx, dev_rows, m, dev_ids, dev_prf, plen, roots, n, dig, valid,
                         blob_root=torch.zeros(32, dtype=torch.uint8, device="cuda"))
    torch.cuda.synchronize()
    assert valid.cpu().numpy().sum() == 0


def test_validate_batch_short_proof_is_invalid(ctx):
    n = 1
    coded, roots, _, _, full = _blob_setup(ctx, n)
    m = 4
    ids = torch.tensor([(0, j) for j in range(m)], dtype=torch.int64).cuda()
    prf = torch.from_numpy(np.frombuffer(b"".join(b"".join(full[j][:3]) for j in range(m)), np.uint8).copy()).cuda()
    dig = torch.empty(m * 32, dtype=torch.uint8, device="cuda")
    valid = torch.full((m,), 7, dtype=torch.uint8, device="cuda")
    codec.validate_batch(ctx, coded, m, ids, prf, 3, roots, n, dig, valid)
    torch.cuda.synchronize()
    assert valid.cpu().numpy().tolist() == [0] * m
    # the same rows with their 4-hash proofs (1 chunkset: empty blob-level path) are valid
    prf4 = torch.from_numpy(np.frombuffer(b"".join(b"".join(full[j]) for j in range(m)), np.uint8).copy()).cuda()
    codec.validate_batch(ctx, coded, m, ids, prf4, 4, roots, n, dig, valid)
    torch.cuda.synchronize()
    assert valid.cpu().numpy().tolist() == [1] * m

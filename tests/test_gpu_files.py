"""decds-bin's break / repair file flow over the device path: layout, wire format,
proofs against the BLAKE3/Merkle restatement, repair from a lossy and partly corrupted share set
(handle_break.rs, handle_repair.rs), and the not-enough-shares failure."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from decds_amd import files, wire  # noqa: E402
from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N, DecdsError  # noqa: E402
import oracle as o  # noqa: E402

pytestmark = pytest.mark.gpu


def _broken(ctx, tmp_path, size, seed, **kw):
    blob = o.fill_random(seed, size)
    coeffs = o.fill_random(seed + 1, -(-size // CS) * N * K)
    src = tmp_path / "blob.data"
    blob.tofile(src)
    d = tmp_path / "shares"
    header = files.break_blob(ctx, str(src), str(d), batch=2, coeffs=coeffs, **kw)
    return blob, header, d


@pytest.mark.parametrize("device_store", [None, False])  # coded rows kept in HBM / in a page-locked host store
def test_break_layout_header_and_proofs(ctx, tmp_path, device_store):
    size = 2 * CS + 12345
    blob, header, d = _broken(ctx, tmp_path, size, 0xF11E, device_store=device_store)
    n = 3
    h2 = files.read_blob_metadata(str(d))
    assert h2 == header and h2.get_blob_size() == size and h2.get_num_chunksets() == n
    assert h2.get_blob_digest() == o.blake3(blob.tobytes())            # blob.rs:249
    leaves_by_cs = []
    for c in range(n):
        leaves = []
        for j in range(N):
            raw = open(os.path.join(d, "chunkset.%d" % c, "share%02d.data" % j), "rb").read()
            ch, used = wire.pcc_from_bytes(raw)
            assert used == len(raw) and len(ch.erasure_coded_data) == F
            assert (ch.chunkset_id, ch.chunk_id) == (c, c * N + j)
            leaves.append(o.chunk_digest(c, c * N + j, np.frombuffer(ch.erasure_coded_data, np.uint8)))
            assert ch.validate_inclusion_in_blob(h2.get_root_commitment())
            assert ch.validate_inclusion_in_chunkset(h2.chunkset_root_commitments[c])
            assert len(ch.proof) == 4 + 2                               # 3 chunksets -> depth 2
        root, _ = o.merkle(leaves)
        assert h2.chunkset_root_commitments[c] == root
        leaves_by_cs.append(root)
    assert h2.get_root_commitment() == o.merkle(leaves_by_cs)[0]      # blob.rs:266-268


def test_repair_from_lossy_corrupted_shares(ctx, tmp_path):
    size = 2 * CS + 777
    blob, header, d = _broken(ctx, tmp_path, size, 0xF22E)
    rng = np.random.default_rng(4)
    for c in range(3):
        for j in rng.permutation(N)[:5]:                               # lose 5 of 16 shares
            os.remove(os.path.join(d, "chunkset.%d" % c, "share%02d.data" % j))
    # corrupt one surviving share of chunkset 0 (its proof stops verifying: skipped, as the
    # reference skips InvalidProofInChunk), and truncate one of chunkset 1 (unparsable: skipped)
    left0 = sorted(os.listdir(os.path.join(d, "chunkset.0")))
    p = os.path.join(d, "chunkset.0", left0[0])
    b = bytearray(open(p, "rb").read())
    b[5000] ^= 0x10
    open(p, "wb").write(bytes(b))
    left1 = sorted(os.listdir(os.path.join(d, "chunkset.1")))
    p = os.path.join(d, "chunkset.1", left1[0])
    open(p, "wb").write(open(p, "rb").read()[:1000])
    out_dir = tmp_path / "repaired"
    t = {}
    path = files.repair_blob(ctx, str(d), str(out_dir), batch=2, timings=t)
    assert open(path, "rb").read() == blob.tobytes()
    assert os.path.getsize(os.path.join(out_dir, "chunkset.2.data")) == size - 2 * CS
    assert os.path.getsize(os.path.join(out_dir, "chunkset.0.data")) == CS


def test_repair_not_enough_shares_fails(ctx, tmp_path):
    blob, header, d = _broken(ctx, tmp_path, CS, 0xF33E)
    for j in range(7):                                                 # 9 left: rank < 10
        os.remove(os.path.join(d, "chunkset.0", "share%02d.data" % j))
    with pytest.raises(DecdsError) as e:
        files.repair_blob(ctx, str(d), str(tmp_path / "r"))
    assert e.value.kind == "ChunksetNotYetReadyToRepair"


def test_metadata_with_trailing_bytes_is_rejected(ctx, tmp_path):
    blob, header, d = _broken(ctx, tmp_path, 1000, 0xF44E)
    with open(os.path.join(d, "metadata.commit"), "ab") as f:
        f.write(b"\x00")
    with pytest.raises(DecdsError) as e:
        files.read_blob_metadata(str(d))
    assert e.value.kind == "BlobHeaderDeserializationFailed"


def test_repair_foreign_shares_follow_the_reference(ctx, tmp_path):
    # handle_repair.rs:41-92 + blob.rs:373-394: a chunk is routed by its OWN chunkset id. A share of
    # chunkset 2 found in chunkset 0's directory goes to chunkset 2 (its own copy later is then not
    # useful: ignored) and the repair succeeds; the same result as the batched pass, by the
    # sequential loop the batched pass falls back to.
    size = 2 * CS + 4321
    blob, header, d = _broken(ctx, tmp_path, size, 0xF55E)
    share = lambda c, j: os.path.join(d, "chunkset.%d" % c, "share%02d.data" % j)
    open(share(0, 0), "wb").write(open(share(2, 5), "rb").read())
    for j in range(1, 4):
        os.remove(share(2, j))                                         # chunkset 2 needs the foreign copy less
    t = {}
    path = files.repair_blob(ctx, str(d), str(tmp_path / "r1"), batch=2, timings=t)
    assert t.get("sequential") and open(path, "rb").read() == blob.tobytes()
    # a share of chunkset 0 in chunkset 1's directory: chunkset 0 is repaired by then, so the
    # reference stops with ChunksetAlreadyRepaired (not one of the errors it ignores)
    open(share(1, 3), "wb").write(open(share(0, 7), "rb").read())
    with pytest.raises(DecdsError) as e:
        files.repair_blob(ctx, str(d), str(tmp_path / "r2"), batch=2)
    assert e.value.kind == "ChunksetAlreadyRepaired"

"""GPU parity of the Blob / RepairingBlob mirror (decds-lib/src/blob.rs:227-473) against oracle/:
Blob::new's coded bytes, commitments, blob-level tree and get_share; RepairingBlob's incremental
add_chunk / get_repaired_chunkset with every error branch, the reference's own tests
(blob.rs:700-837) and the all-chunks shuffle round trip (tests.rs:4-57), and the batched add_chunks
against sequential add_chunk calls."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import decds_amd  # noqa: E402
from decds_amd import BlobHeader, DecdsError  # noqa: E402
from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N  # noqa: E402
import oracle as o  # noqa: E402

pytestmark = pytest.mark.gpu


def _blob(ctx, blob_len, seed):
    data = o.fill_random(seed, blob_len)
    n = -(-blob_len // CS)
    coeffs = o.fill_random(seed + 1, n * N * K)
    return data, coeffs, decds_amd.Blob(ctx, data, coeffs)


def _all_chunks(blob):
    return [c for j in range(N) for c in blob.get_share(j)]  # the reference's order (blob.rs:710-712)


def _raises(kind, fn, *a):
    with pytest.raises(DecdsError) as e:
        fn(*a)
    assert e.value.kind == kind, e.value
    return e.value


def test_blob_new_matches_oracle(ctx):
    blob_len = 2 * CS + CS // 2
    data, coeffs, blob = _blob(ctx, blob_len, 0x1B10)
    n = 3
    coded = o.blob_encode(data, coeffs, nthreads=8)
    h = blob.get_blob_header()
    assert (h.get_blob_size(), h.get_num_chunksets()) == (blob_len, n)
    assert h.get_blob_digest() == o.blake3(data)                                     # blob.rs:249
    leaves = [[o.chunk_digest(c, c * N + j, coded[c * N + j]) for j in range(N)] for c in range(n)]
    roots = [o.merkle(lv)[0] for lv in leaves]
    assert h.chunkset_root_commitments == roots                                    # chunkset.rs:54-57
    broot, bproofs = o.merkle(roots)                                                # blob.rs:266-273
    assert h.get_root_commitment() == broot
    assert blob.proof_len() == 4 + 2
    for j in range(N):
        share = blob.get_share(j)                                                   # blob.rs:306-317
        assert len(share) == n
        for c, ch in enumerate(share):
            assert ch.get_chunkset_id() == c and ch.get_global_chunk_id() == c * N + j
            assert ch.get_erasure_coded_data() == coded[c * N + j].tobytes()
            cproof = o.merkle(leaves[c])[1][j]
            assert ch.get_proof() == cproof + bproofs[c]                            # chunkset.rs:98-102
            assert o.merkle_verify(c * N + j, leaves[c][j], ch.get_proof(), broot)  # chunk.rs:88-90
            assert h.validate_chunk(ch)                                              # blob.rs:211-215
    # a flipped byte, or a chunk presented under another chunkset's id, fails validation
    ch = blob.get_share(3)[1]
    bad = bytearray(ch.get_erasure_coded_data())
    bad[777] ^= 1
    assert not h.validate_chunk(decds_amd.Chunk(1, N + 3, bytes(bad), ch.get_proof()))
    assert not h.validate_chunk(decds_amd.Chunk(2, N + 3, ch.get_erasure_coded_data(), ch.get_proof()))
    _raises("InvalidErasureCodedShareId", blob.get_share, N)
    _raises("EmptyDataForBlob", decds_amd.Blob, ctx, b"")
    # a multi-context Blob (shards over two contexts of the one device) is identical
    ctx2 = decds_amd.Context(0)
    b2 = decds_amd.Blob([ctx, ctx2], data, coeffs)
    assert b2.get_blob_header() == h
    assert [c.get_erasure_coded_data() for c in b2.get_share(7)] == [c.get_erasure_coded_data() for c in blob.get_share(7)]
    del b2
    ctx2.close()


@pytest.mark.parametrize("blob_len", [1, 1023, 1024, 1025, (1 << 20) - 1, 1 << 20, (1 << 20) + 1, 2 << 20,
                                      (3 << 20) + 777, CS - 1, CS, CS + 1, 2 * CS + 12345, 4 * CS + (1 << 20) + 5])
def test_blob_digest_every_group_shape(ctx, blob_len):
    """Blob::new's whole-blob digest (blake3::hash(&data), blob.rs:249) at every shape of its split: up to
    1 MiB on the host; above, full 1 MiB groups on the device (blob_group_kernel) plus the last partial
    group on the host, folded on the host — against the oracle's BLAKE3, one and three contexts."""
    data = o.fill_random(0xD16E57 + blob_len, blob_len)
    n = -(-blob_len // CS)
    coeffs = o.fill_random(0xC0DE + blob_len, n * N * K)
    want = o.blake3(data)
    assert decds_amd.Blob(ctx, data, coeffs).get_blob_header().get_blob_digest() == want
    if n >= 3:
        ctxs = [decds_amd.Context(0) for _ in range(2)]
        try:
            assert decds_amd.Blob([ctx] + ctxs, data, coeffs).get_blob_header().get_blob_digest() == want
        finally:
            for c in ctxs:
                c.close()


def test_repairing_blob_add_chunk_like_reference(ctx):
    # blob.rs:700-762
    _, _, blob = _blob(ctx, 2 * CS, 0x2B20)
    header = blob.get_blob_header()
    chunks = _all_chunks(blob)
    rep = decds_amd.RepairingBlob(ctx, header)
    rep.add_chunk(chunks[0])
    bad_header = BlobHeader(header.byte_length, header.num_chunksets, header.digest, o.blake3(b"fake_root_commitment"),
                            header.chunkset_root_commitments)
    _raises("InvalidProofInChunk", decds_amd.RepairingBlob(ctx, bad_header).add_chunk, chunks[0])
    ready = decds_amd.RepairingBlob(ctx, header)
    cs0 = chunks[0].get_chunkset_id()
    for c in chunks:
        if c.get_chunkset_id() == cs0:
            ready.add_chunk(c)
            if ready.is_chunkset_ready_to_repair(cs0):
                break
    assert ready.is_chunkset_ready_to_repair(cs0)
    extra = next(c for c in chunks if c.get_chunkset_id() == cs0 and c.get_global_chunk_id() != chunks[0].get_global_chunk_id())
    _raises("ChunksetReadyToRepair", ready.add_chunk, extra)
    ready.get_repaired_chunkset(cs0)
    assert not ready.is_chunkset_ready_to_repair(cs0)
    assert ready.is_chunkset_already_repaired(cs0)
    _raises("ChunksetAlreadyRepaired", ready.add_chunk, chunks[0])


@pytest.mark.usefixtures("decode_form")
def test_repairing_blob_get_repaired_chunkset_like_reference(ctx):
    # blob.rs:765-837: 2.5 chunksets, the partial last one truncated
    blob_len = 2 * CS + CS // 2
    data, _, blob = _blob(ctx, blob_len, 0x3B30)
    header = blob.get_blob_header()
    chunks = _all_chunks(blob)
    rep = decds_amd.RepairingBlob(ctx, header)
    _raises("ChunksetNotYetReadyToRepair", rep.get_repaired_chunkset, 0)
    for cid in (0, 2):
        for c in chunks:
            if c.get_chunkset_id() == cid:
                rep.add_chunk(c)
                if rep.is_chunkset_ready_to_repair(cid):
                    break
        assert rep.is_chunkset_ready_to_repair(cid)
        got = rep.get_repaired_chunkset(cid)
        assert got == data[cid * CS:min(blob_len, (cid + 1) * CS)].tobytes()
        assert rep.is_chunkset_already_repaired(cid)
        _raises("ChunksetAlreadyRepaired", rep.get_repaired_chunkset, cid)
    _raises("InvalidChunksetId", rep.get_repaired_chunkset, 3)
    _raises("InvalidChunksetId", rep.is_chunkset_ready_to_repair, 3)
    _raises("InvalidChunksetId", rep.is_chunkset_already_repaired, 3)


def test_repairing_blob_error_branches(ctx):
    data, _, blob = _blob(ctx, CS + 99, 0x4B40)
    header = blob.get_blob_header()
    rep = decds_amd.RepairingBlob(ctx, header)
    c0 = blob.get_chunk(0, 3)
    moved = decds_amd.Chunk(5, c0.chunk_id, c0.erasure_coded_data, c0.proof)
    _raises("InvalidChunksetId", rep.add_chunk, moved)                            # blob.rs:376-379
    t = bytearray(c0.erasure_coded_data)
    t[4321] ^= 1
    _raises("InvalidProofInChunk", rep.add_chunk, decds_amd.Chunk(0, c0.chunk_id, bytes(t), c0.proof))
    _raises("InvalidProofInChunk", rep.add_chunk, decds_amd.Chunk(0, c0.chunk_id, c0.erasure_coded_data, c0.proof[:3]))
    wrong = blob.get_chunk(1, 3)                                                   # a valid chunk of chunkset 1
    _raises("InvalidProofInChunk", rep.add_chunk, decds_amd.Chunk(0, c0.chunk_id, wrong.erasure_coded_data, wrong.proof))
    rep.add_chunk(c0)
    _raises("ChunkDecodingFailed", rep.add_chunk, c0)                              # not useful (chunkset.rs:181-183)
    for j in range(N):
        if rep.is_chunkset_ready_to_repair(0):
            break
        try:
            rep.add_chunk(blob.get_chunk(0, j))
        except DecdsError as e:
            assert e.kind == "ChunkDecodingFailed"
    _raises("ChunksetNotYetReadyToRepair", rep.get_repaired_chunkset, 1)
    assert rep.get_repaired_chunkset(0) == data[:CS].tobytes()
    _raises("ChunksetAlreadyRepaired", rep.add_chunk, c0)


@pytest.mark.usefixtures("decode_form")
def test_repairing_blob_all_chunks_shuffled_batch_vs_sequential(ctx):
    # tests.rs:4-57 through RepairingBlob: every chunk of every chunkset in one shuffled order, some
    # tampered; the batched add_chunks must return exactly the sequential add_chunk results, and
    # every chunkset repairs (several decoded in one device batch)
    blob_len = 5 * CS + 4321
    data, _, blob = _blob(ctx, blob_len, 0x5B50)
    header = blob.get_blob_header()
    n = header.get_num_chunksets()
    chunks = _all_chunks(blob)
    order = np.random.default_rng(3).permutation(len(chunks))
    arrivals = []
    for i, k in enumerate(order):
        c = chunks[int(k)]
        if i % 17 == 5:  # tamper with a few on the way
            t = bytearray(c.erasure_coded_data)
            t[i * 97 % F] ^= 0x10
            c = decds_amd.Chunk(c.chunkset_id, c.chunk_id, bytes(t), c.proof)
        arrivals.append(c)
    seq = decds_amd.RepairingBlob(ctx, header)
    want = []
    for c in arrivals:
        try:
            seq.add_chunk(c)
            want.append(0)
        except DecdsError as e:
            want.append(e.status)
    bat = decds_amd.RepairingBlob(ctx, header)
    got = bat.add_chunks(arrivals)
    assert got.tolist() == want
    assert 11 in want and 3 in want  # InvalidProofInChunk and ChunksetReadyToRepair both occurred
    for rep in (bat, seq):
        for c in range(n):
            assert rep.is_chunkset_ready_to_repair(c)
        for c in (3, 0, 5, 1, 2, 4):
            assert rep.get_repaired_chunkset(c) == data[c * CS:min(blob_len, (c + 1) * CS)].tobytes(), c
    # after everything is repaired, every further chunk is rejected as already repaired
    assert set(bat.add_chunks(arrivals[:20]).tolist()) == {10}


@pytest.mark.parametrize("budget", [None, "2 slabs"])
def test_repairing_blob_cfg2_slots_span_4gib_windows(ctx, budget):
    # cfg2 through RepairingBlob: 103 chunksets, 10 random survivors each, validated in device batches
    # and decoded from per-chunkset device slots (gather form). The 103 slots span > 2 GiB of slabs, so
    # some slot addresses have bit 31 of their low word set: r02i's fault (a sign-extended
    # readfirstlane in the gather addressing) is hit deterministically here.
    blob_len = 1 << 30
    data, _, blob = _blob(ctx, blob_len, 0x6B60)
    header = blob.get_blob_header()
    n = header.get_num_chunksets()
    assert n == 103
    rng = np.random.default_rng(0x6B61)
    plen = blob.proof_len()
    rows = np.empty((n * K, F), np.uint8)
    ids = np.empty((n * K, 2), np.uint64)
    proofs = np.empty((n * K, plen * 32), np.uint8)
    for c in range(n):
        for a, j in enumerate(rng.permutation(N)[:K].tolist()):
            ch = blob.get_chunk(c, j)
            r = c * K + a
            rows[r] = np.frombuffer(ch.erasure_coded_data, np.uint8)
            ids[r] = (c, ch.chunk_id)
            proofs[r] = np.frombuffer(b"".join(ch.proof), np.uint8)
    # "2 slabs": a device budget of two decode areas (a quarter of the budget goes to areas) + 16
    # chunksets' rows; the other 87 chunksets' rows spill to page-locked host memory and are staged
    # into the decode areas at their decode
    rep = decds_amd.RepairingBlob(ctx, header, device_budget=None if budget is None else 2 * _AREA + 2 * _SLAB)
    st = rep.add_rows(rows, ids, proofs, plen)
    del rows
    assert set(st.tolist()) <= {0, 4}  # accepted, or not useful (a dependent survivor)
    mem = rep.memory()
    assert mem["spilled_chunksets"] == (0 if budget is None else n - 16), mem
    out = decds_amd.HostBuffer(CS)
    for c in range(n):
        if not rep.is_chunkset_ready_to_repair(c):
            continue
        got = rep.get_repaired_chunkset(c, out=out.array)
        assert np.array_equal(got, data[c * CS:min(blob_len, (c + 1) * CS)]), c
    del got
    left = rep.memory()                       # only chunksets that never became ready keep their rows
    not_ready = sum(not rep.is_chunkset_ready_to_repair(c) and not rep.is_chunkset_already_repaired(c) for c in range(n))
    assert left["device_chunksets"] + left["spilled_chunksets"] == not_ready, left


# the decode-area + one-slab budget of decds_repairing_blob_set_device_budget (blob.cpp RbShard)
_ROWS = -(-K * F // 256) * 256
_AREA = _ROWS + CS
_SLAB = 8 * _ROWS


def _arrivals(blob, seed, tamper_every=13):
    chunks = _all_chunks(blob)
    out = []
    for i, k in enumerate(np.random.default_rng(seed).permutation(len(chunks))):
        c = chunks[int(k)]
        if i % tamper_every == 4:
            t = bytearray(c.erasure_coded_data)
            t[i * 131 % F] ^= 0x40
            c = decds_amd.Chunk(c.chunkset_id, c.chunk_id, bytes(t), c.proof)
        out.append(c)
    return out


def _sequential(rep, arrivals):
    st = []
    for c in arrivals:
        try:
            rep.add_chunk(c)
            st.append(0)
        except DecdsError as e:
            st.append(e.status)
    return st


@pytest.mark.usefixtures("decode_form")
def test_repairing_blob_sharded_and_spilled_match_one_context(ctx):
    # blob.rs:321-473 over two contexts (chunksets [0, 5) and [5, 9) of the one device stand in for
    # two GPUs) and under device budgets that spill accepted rows to page-locked host memory: statuses
    # of every shuffled arrival (tampered ones included) and every repaired chunkset are identical to
    # the one-context object with everything resident
    blob_len = 8 * CS + 54321
    data, _, blob = _blob(ctx, blob_len, 0x7B70)
    header = blob.get_blob_header()
    n = header.get_num_chunksets()
    assert n == 9
    arrivals = _arrivals(blob, 0x7B71)
    ref = decds_amd.RepairingBlob(ctx, header)
    want = _sequential(ref, arrivals)
    assert 11 in want and 3 in want
    ctx2 = decds_amd.Context(0)
    cases = {
        "2 contexts, batch": (decds_amd.RepairingBlob([ctx, ctx2], header), True),
        "2 contexts, all spilled": (decds_amd.RepairingBlob([ctx, ctx2], header, device_budget=0), False),
        "1 context, 1 slab + 1 area": (decds_amd.RepairingBlob(ctx, header, device_budget=_AREA + _SLAB), True),
        "2 contexts, 1 slab + 1 area, sequential": (decds_amd.RepairingBlob([ctx, ctx2], header,
                                                                            device_budget=_AREA + _SLAB), False),
    }
    fetch = [4, 8, 0, 5, 2, 7, 1, 3, 6]
    for name, (rep, batched) in cases.items():
        got = rep.add_chunks(arrivals).tolist() if batched else _sequential(rep, arrivals)
        assert got == want, name
        mem = rep.memory()
        assert mem["contexts"] == (2 if name.startswith("2") else 1), name
        # rows on the device / spilled: one slab holds 8 chunksets' rows per context
        expect = {"2 contexts, batch": (n, 0), "2 contexts, all spilled": (0, n), "1 context, 1 slab + 1 area": (8, 1),
                  "2 contexts, 1 slab + 1 area, sequential": (n, 0)}[name]
        assert (mem["device_chunksets"], mem["spilled_chunksets"]) == expect, (name, mem)
        if "slab" in name or "spilled" in name:
            batch_area = 256 * (F + 16 + 32 * blob.proof_len() + 32) if batched else 0
            assert mem["device_bytes"] <= mem["contexts"] * (_AREA + _SLAB + batch_area + (1 << 20)), (name, mem)
        for c in fetch:
            assert rep.get_repaired_chunkset(c) == data[c * CS:min(blob_len, (c + 1) * CS)].tobytes(), (name, c)
        assert rep.memory()["device_chunksets"] == 0 and rep.memory()["spilled_chunksets"] == 0
        _raises("ChunksetAlreadyRepaired", rep.add_chunk, arrivals[0])
    del cases, ref, rep
    ctx2.close()


def test_host_buffer_views_keep_the_block_alive(ctx):
    # a view of HostBuffer.array must not outlive the page-locked block it points into
    hb = decds_amd.HostBuffer(3 << 20)
    view = hb.array[1000:2000]
    view[:] = 7
    assert hb.free() is False                   # a view is alive: refused
    del hb
    assert int(view.sum()) == 7 * 1000          # still readable: the view holds the block
    other = decds_amd.HostBuffer(3 << 20)
    other.array[:] = 1
    assert int(view.sum()) == 7 * 1000          # and no later allocation aliases it
    assert other.free() is True
    del view


def test_context_close_releases_its_objects_first(ctx):
    # a RepairingBlob / Blob built on a context that is closed while they are alive is released
    # first (Context.close): no destructor touches freed device state afterwards
    data, _, blob = _blob(ctx, CS + 5, 0x8B80)
    header = blob.get_blob_header()
    ctx2 = decds_amd.Context(0)
    rep = decds_amd.RepairingBlob([ctx, ctx2], header)
    b2 = decds_amd.Blob([ctx2], data)
    rep.add_chunk(blob.get_chunk(0, 1))
    ctx2.close()
    assert rep._h is None and b2._h is None
    del rep, b2



@pytest.mark.usefixtures("decode_form")
def test_repairing_blob_two_decode_areas_any_fetch_order(ctx):
    # RbShard's decode-area pool (blob.cpp) at its smallest useful size, two areas: each fetch decodes
    # the chunkset asked for plus the next ready one into the other area when that is free, and frees
    # the asked-for one's area, so a later fetch always finds a free area (take_area's eviction branch
    # is a guard that this API order never reaches). Out-of-order fetches must return
    # every chunkset's bytes, whether it was decoded as the asked-for one or ahead of time.
    blob_len = 5 * CS + 777
    data, _, blob = _blob(ctx, blob_len, 0x8B80)
    header = blob.get_blob_header()
    n = header.get_num_chunksets()
    rep = decds_amd.RepairingBlob(ctx, header, device_budget=8 * _AREA + 1)  # a quarter: 2 areas; 1 slab for rows
    for c in _all_chunks(blob):
        if not rep.is_chunkset_ready_to_repair(c.get_chunkset_id()):
            rep.add_chunk(c)
    assert all(rep.is_chunkset_ready_to_repair(c) for c in range(n))
    want = lambda c: data[c * CS:min(blob_len, (c + 1) * CS)].tobytes()  # noqa: E731
    for c in (0, 3, 4, 1, 5, 2):  # c1 is decoded ahead with c0 and c2 with c5, the others on demand
        assert rep.get_repaired_chunkset(c) == want(c), c
        assert rep.memory()["decode_areas"] == 2
    assert all(rep.is_chunkset_already_repaired(c) for c in range(n))


def test_objects_built_on_temporary_contexts_stay_usable():
    # Blob, RepairingBlob and RepairingChunkSet keep the contexts they were built on alive:
    # built on contexts nobody else holds, they still work after a garbage collection
    import gc
    blob_len = CS + 12345
    data = o.fill_random(0x7E4D, blob_len)
    coeffs = o.fill_random(0x7E4E, 2 * N * K)
    blob = decds_amd.Blob(decds_amd.Context(0), data, coeffs)
    gc.collect()
    header = blob.get_blob_header()
    chunks = _all_chunks(blob)
    rep = decds_amd.RepairingBlob([decds_amd.Context(0), decds_amd.Context(0)], header)
    rcs = decds_amd.RepairingChunkSet(decds_amd.Context(0), 1)
    gc.collect()
    for ch in chunks:
        if ch.get_chunkset_id() == 1 and not rcs.is_ready_to_repair():
            rcs.add_chunk_unvalidated(ch)
        for cid in (0, 1):
            if ch.get_chunkset_id() == cid and not rep.is_chunkset_ready_to_repair(cid):
                rep.add_chunk(ch)
    gc.collect()
    assert rep.get_repaired_chunkset(0) == data[:CS].tobytes()
    assert rep.get_repaired_chunkset(1) == data[CS:].tobytes()
    assert rcs.repair()[:blob_len - CS] == data[CS:].tobytes()

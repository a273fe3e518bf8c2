"""GPU parity tests: the gfx950 kernels (through the C-ABI) against the CPU restatement (oracle/)
and the committed known-answer vectors, on the same seeded inputs. Bit-exact everywhere — the
path is integer / byte GF(2^8) work. Reference tests mirrored: chunkset.rs:257-298, 419-480,
blob.rs:767-837, tests.rs:4-57."""
import hashlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import decds_amd  # noqa: E402
from decds_amd import codec  # noqa: E402
from decds_amd._capi import CHUNKSET_BYTES as CS, CODED_PIECE_BYTES as F, K, N, PIECE_BYTES as L  # noqa: E402
import oracle as o  # noqa: E402

pytestmark = pytest.mark.gpu

OKV, NOT_USEFUL, AFTER_READY, NONE = 0, 4, 3, -1


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def dev(a):
    # a writable copy: torch.from_numpy warns on read-only arrays (np.frombuffer over bytes, golden fixtures)
    return torch.from_numpy(np.array(a, copy=True)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def gpu_encode(ctx, data, coeffs, n, pitch=F, off=0):
    # off: the coded rows start `off` bytes into the allocation (another column phase, edge_col)
    src, cv = dev(data), dev(coeffs)
    dst = torch.zeros(off + (n * N - 1) * pitch + F, dtype=torch.uint8, device="cuda")
    codec.encode_batch(ctx, src, n, cv, dst[off:], pitch)
    out = host(dst)[off:]
    return np.stack([out[r * pitch: r * pitch + F] for r in range(n * N)])


@pytest.mark.usefixtures("encode_form")
def test_encode_cfg1_matches_golden_and_oracle(ctx, kat):
    c = kat["cfg1"]
    data = o.fill_random(c["data_seed"], CS)
    coeffs = np.frombuffer(bytes.fromhex(c["coeffs"]), dtype=np.uint8)
    coded = gpu_encode(ctx, data, coeffs, 1)
    assert [sha(coded[j]) for j in range(N)] == c["coded_sha256"]
    assert np.array_equal(coded, o.chunkset_encode(data, coeffs, nthreads=8))


@pytest.mark.usefixtures("encode_form")
def test_encode_batch_bitexact_and_pitch(ctx):
    n = 5
    data = o.fill_random(0xDEC05002, n * CS)
    coeffs = o.fill_random(0xC0EF0002, n * N * K)
    refs = {c: o.chunkset_encode(data[c * CS:(c + 1) * CS], coeffs[c * 160:(c + 1) * 160], nthreads=8)
            for c in (0, 2, 4)}
    # 16-byte-aligned pitches run the blocks at column phase (6 - off) mod 16: head columns too
    for pitch, off in ((F, 0), (F + 53, 0), (1 << 21, 0), (F + 5, 0), (F + 5, 3), (F + 5, 6), (F + 117, 15)):
        coded = gpu_encode(ctx, data, coeffs, n, pitch, off)
        for c in (0, 2, 4):
            assert np.array_equal(coded[c * N:(c + 1) * N], refs[c]), (pitch, off, c)


@pytest.mark.usefixtures("encode_form")
def test_encode_every_column_phase(ctx):
    # a 16-byte-aligned pitch at each of the 16 base offsets runs the encode blocks at each column
    # phase; above phase 7 the last block becomes edge columns (piece 9 must not read past the
    # chunkset into its marker / padding), so 2 chunksets, the first one's neighbour readable
    n, pitch = 2, F + 5
    data = o.fill_random(0xDEC05005, n * CS)
    coeffs = o.fill_random(0xC0EF0005, n * N * K)
    refs = [o.chunkset_encode(data[c * CS:(c + 1) * CS], coeffs[c * 160:(c + 1) * 160], nthreads=8) for c in range(n)]
    for off in range(16):
        coded = gpu_encode(ctx, data, coeffs, n, pitch, off)
        for c in range(n):
            assert np.array_equal(coded[c * N:(c + 1) * N], refs[c]), (off, c)


@pytest.mark.usefixtures("encode_form")
@pytest.mark.parametrize("n", [1, 16])
def test_encode_small_batches_match_oracle(ctx, n):
    # the small-batch sizes of the bench's sweep through every encode form, in the
    # bench's payload-aligned layout: first, middle and last chunkset against the oracle
    data = o.fill_random(0xDEC05016 + n, n * CS)
    coeffs = o.fill_random(0xC0EF0016 + n, n * N * K)
    src, cv = dev(data), dev(coeffs)
    dst, pitch = codec.coded_buffer(n)
    codec.encode_batch(ctx, src, n, cv, dst, pitch)
    out = host(dst)
    for c in sorted({0, n // 2, n - 1}):
        ref = o.chunkset_encode(data[c * CS:(c + 1) * CS], coeffs[c * 160:(c + 1) * 160], nthreads=8)
        rows = np.stack([out[(c * N + j) * pitch:(c * N + j) * pitch + F] for j in range(N)])
        assert np.array_equal(rows, ref), c


@pytest.mark.usefixtures("decode_form")
def test_encode_decode_at_the_largest_pitch(ctx):
    # a chunkset's 16 rows must fit one 2 GiB buffer descriptor (include/decds_rlnc.h): the largest
    # pitch is bit-exact through encode and repair (lanes past the last block use out-of-range
    # offsets, which must stay out of range there too); one byte more is refused
    pmax = ((1 << 31) - 1 - F) // (N - 1)
    data = o.fill_random(0xDEC05003, CS)
    coeffs = o.fill_random(0xC0EF0003, N * K)
    dst = torch.zeros((N - 1) * (pmax + 1) + F, dtype=torch.uint8, device="cuda")
    codec.encode_batch(ctx, dev(data), 1, dev(coeffs), dst, pmax)
    rows = host(dst.as_strided((N, F), (pmax, 1)))
    assert np.array_equal(rows, o.chunkset_encode(data, coeffs, nthreads=8))
    cand = np.array([15, 3, 8, 0, 12, 5, 9, 1, 14, 6, 2, 4, 7, 10, 11, 13], np.uint8)
    plan = torch.empty(128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(N, dtype=torch.int8, device="cuda")
    status = torch.empty(1, dtype=torch.int32, device="cuda")
    out = torch.zeros(CS, dtype=torch.uint8, device="cuda")
    codec.repair_batch(ctx, dst, 1, dev(cand), plan, verd, out, status, pitch=pmax)
    assert host(status)[0] == 0 and np.array_equal(host(out), data)
    with pytest.raises(decds_amd.DecdsError) as e:
        codec.encode_batch(ctx, dev(data), 1, dev(coeffs), dst, pmax + 1)
    assert e.value.kind == "InvalidArgument"


@pytest.mark.usefixtures("encode_form")
def test_encode_zero_and_edge_coefficients(ctx):
    # zero coding vectors, identity rows (systematic pieces) and 0xFF everywhere
    data = o.fill_random(31, CS)
    coeffs = np.zeros((N, K), np.uint8)
    for j in range(K):
        coeffs[j, j] = 1
    coeffs[10] = 0xFF
    coeffs[11, 9] = 0x80
    coeffs[12] = np.arange(1, 11)
    coded = gpu_encode(ctx, data, coeffs, 1)
    assert np.array_equal(coded, o.chunkset_encode(data, coeffs))
    padded = o.encoder_pad(data)
    for j in range(K):  # identity rows reproduce the padded pieces (marker included)
        assert np.array_equal(coded[j, K:], padded[j * L:(j + 1) * L])
    assert not coded[13:, K:].any()


def test_field_parameter_other_polynomial(ctx, kat):
    c = kat["cfg1"]
    data = o.fill_random(c["data_seed"], CS)
    coeffs = np.frombuffer(bytes.fromhex(c["coeffs"]), dtype=np.uint8)
    ctx.set_field(0x11B, 0x81)
    try:
        coded = gpu_encode(ctx, data, coeffs, 1)
        # repair under 0x11B too: 2 is not a generator there, so the plan kernel's log/exp tables
        # run on the host-found generator 3
        cand = np.array([15, 3, 8, 0, 12, 5, 9, 1, 14, 6, 2, 4, 7, 10, 11, 13], np.uint8)
        plan = torch.empty(128, dtype=torch.uint8, device="cuda")
        verd = torch.empty(N, dtype=torch.int8, device="cuda")
        status = torch.empty(1, dtype=torch.int32, device="cuda")
        out = torch.zeros(CS, dtype=torch.uint8, device="cuda")
        codec.repair_batch(ctx, dev(coded.reshape(-1)), 1, dev(cand), plan, verd, out, status)
        assert host(status)[0] == 0 and np.array_equal(host(out), data)
    finally:
        ctx.set_field(0x11D, 0x81)
    assert [sha(coded[j]) for j in range(N)] == kat["cfg1_poly_0x11b_coded_sha256"]
    # a reducible polynomial is no field (x^8 + 1 = (x + 1)^8): refused, the field is unchanged
    with pytest.raises(decds_amd.DecdsError) as e:
        ctx.set_field(0x101, 0x81)
    assert e.value.kind == "InvalidArgument"


def _oracle_verdicts(coded, cand):
    """replay chunkset.rs:173-184 on the oracle decoder over the coefficient prefix only"""
    dec = o.Decoder(3, K)
    out = []
    for r in cand:
        if r == 0xFF:
            out.append(NONE)
            continue
        if dec.is_already_decoded():
            out.append(AFTER_READY)
            continue
        st = dec.decode(np.concatenate([coded[r, :K], np.zeros(3, np.uint8)]))
        out.append(OKV if st == o.OK else NOT_USEFUL)
    return out, dec.rank()


@pytest.mark.usefixtures("decode_form")
def test_repair_batch_roundtrip_dependent_and_not_ready(ctx):
    n = 6
    data = o.fill_random(0xDEC05003, n * CS)
    coeffs = o.fill_random(0xC0EF0003, n * N * K).reshape(n, N, K).copy()
    coeffs[1, 5] = coeffs[1, 2]                                   # duplicate row -> not useful
    coeffs[2, 7] = [o.gf_mul(9, int(x)) for x in coeffs[2, 3]]   # scalar multiple -> not useful
    coeffs[3, 4] = 0                                              # zero coding vector
    src, cv = dev(data), dev(coeffs)
    coded_d = torch.empty(n * N * F, dtype=torch.uint8, device="cuda")
    codec.encode_batch(ctx, src, n, cv, coded_d)
    rng = np.random.default_rng(4)
    cand = np.full((n, N), 0xFF, np.uint8)
    for c in range(n):
        perm = rng.permutation(N).astype(np.uint8)
        if c == 1:
            perm = np.array([2, 5] + [x for x in perm if x not in (2, 5)], np.uint8)
        if c == 2:
            perm = np.array([3, 7] + [x for x in perm if x not in (3, 7)], np.uint8)
        if c == 4:
            perm = perm[:9]                                       # only 9 chunks -> not ready
        if c == 5:
            perm = perm[:10]                                      # exactly 10 survivors
        cand[c, :perm.size] = perm
    plan = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(n * N, dtype=torch.int8, device="cuda")
    status = torch.full((n,), -7, dtype=torch.int32, device="cuda")
    out = torch.zeros(n * CS, dtype=torch.uint8, device="cuda")
    codec.repair_batch(ctx, coded_d, n, dev(cand), plan, verd, out, status)
    coded = host(coded_d).reshape(n * N, F)
    st, v, res = host(status), host(verd).reshape(n, N), host(out)
    for c in range(n):
        ov, rank = _oracle_verdicts(coded[c * N:(c + 1) * N], cand[c])
        assert list(v[c]) == ov, c
        if rank == K:
            assert st[c] == 0
            assert np.array_equal(res[c * CS:(c + 1) * CS], data[c * CS:(c + 1) * CS]), c
        else:
            assert st[c] == 5 and c == 4
            assert not res[c * CS:(c + 1) * CS].any()            # untouched
    assert NOT_USEFUL in list(v[1]) and NOT_USEFUL in list(v[2])


@pytest.mark.usefixtures("decode_form")
def test_repair_batch_nothing_ready_leaves_every_output(ctx):
    # every chunkset one chunk short (chunkset.rs:206: not yet ready): the decode's tiles all run with
    # out-of-range columns (the sweep's whole grid, incl. its tile counter) and write nothing
    n = 5
    data = o.fill_random(0xDEC05009, n * CS)
    coeffs = o.fill_random(0xC0EF0009, n * N * K)
    coded_d = torch.empty(n * N * F, dtype=torch.uint8, device="cuda")
    codec.encode_batch(ctx, dev(data), n, dev(coeffs), coded_d)
    cand = np.full((n, N), 0xFF, np.uint8)
    rng = np.random.default_rng(9)
    for c in range(n):
        cand[c, :K - 1] = rng.permutation(N)[:K - 1]
    plan = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(n * N, dtype=torch.int8, device="cuda")
    status = torch.full((n,), -7, dtype=torch.int32, device="cuda")
    out = torch.full((n * CS,), 0x5A, dtype=torch.uint8, device="cuda")
    codec.repair_batch(ctx, coded_d, n, dev(cand), plan, verd, out, status)
    assert list(host(status)) == [5] * n
    assert (host(out) == 0x5A).all()

def _fuzz_plan_inputs(n=96):
    """coding vectors of rank-deficient chunksets (rows from random subspaces of rank 1..10, zero and
    repeated rows) and candidate lists of every length with repeated ids"""
    rng = np.random.default_rng(0x91A7)
    coded = torch.zeros(n * N * F, dtype=torch.uint8, device="cuda")
    vecs = np.zeros((n, N, K), np.uint8)
    cand = np.full((n, N), 0xFF, np.uint8)
    for c in range(n):
        r = 10 if c % 4 == 0 else int(rng.integers(1, K + 1))
        basis = rng.integers(0, 256, (r, K), dtype=np.uint8)
        for j in range(N):
            w = rng.integers(0, 256, r)
            v = np.zeros(K, np.uint8)
            for i in range(r):
                v ^= np.array([o.gf_mul(int(w[i]), int(x)) for x in basis[i]], np.uint8)
            vecs[c, j] = v
        if c % 7 == 3:
            vecs[c, 5] = 0
        length = int(rng.integers(0, N + 1)) if c % 3 else N
        ids = rng.integers(0, N, length) if c % 2 else rng.permutation(N)[:length]
        cand[c, :length] = ids
    host_rows = np.zeros((n * N, 16), np.uint8)
    host_rows[:, :K] = vecs.reshape(n * N, K)
    coded.view(n * N, F)[:, :16].copy_(dev(host_rows))
    return coded, vecs, cand


def _check_plans_against_oracle(n, vecs, cand, st, v, pl):
    ranks = set()
    for c in range(n):
        ov, rank = _oracle_verdicts(vecs[c], cand[c])
        assert list(v[c]) == ov, (c, list(v[c]), ov)
        assert pl[c, 10] == rank, c
        ranks.add(rank)
        if rank < K:
            assert st[c] == 5, c
            continue
        assert st[c] == 0, c
        acc = [int(cand[c, a]) for a in range(N) if ov[a] == OKV]
        assert list(pl[c, :K]) == acc, c
        inv = pl[c, 16:16 + K * K].reshape(K, K).T  # stored input-major (rlnc_layout.h RepairPlan)
        m = vecs[c, acc]
        for i in range(K):
            for j in range(K):
                s = 0
                for k in range(K):
                    s ^= o.gf_mul(int(inv[i, k]), int(m[k, j]))
                assert s == (1 if i == j else 0), (c, i, j)
    return ranks


def test_repair_plan_fuzz_low_rank_and_repeats(ctx):
    """The plan kernel alone (chunkset.rs:173-184 replayed per candidate) on 96 chunksets of
    rank-deficient coding vectors: rows drawn from random subspaces of rank 1..10, zero and repeated
    rows, candidate lists of every length with repeated ids. Verdicts, rank and status must equal the
    oracle decoder's; at rank 10 sel must be the accepted rows in order and inv their inverse."""
    n = 96
    coded, vecs, cand = _fuzz_plan_inputs(n)
    plan = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(n * N, dtype=torch.int8, device="cuda")
    status = torch.full((n,), -7, dtype=torch.int32, device="cuda")
    codec.repair_plan_batch(ctx, coded, n, dev(cand), plan, verd, status)
    ranks = _check_plans_against_oracle(n, vecs, cand, host(status), host(verd).reshape(n, N), host(plan).reshape(n, 128))
    assert len(ranks) >= 8  # the draws cover most ranks


def _fast_path_inputs(n=128):
    """chunksets whose first ten candidates are valid (the plan's Gauss-Jordan fast path, plan_fast):
    permuted scaled unit vectors and sparse rows (zero pivots: row swaps at most columns), dense random
    rows, rows over {0..3}, and a dependent or repeated row among the ten (the fast path gives up and
    the incremental form decides); candidate lists of 10..16 ids whose tail ends at every position"""
    rng = np.random.default_rng(0xFA57)
    coded = torch.zeros(n * N * F, dtype=torch.uint8, device="cuda")
    vecs = np.zeros((n, N, K), np.uint8)
    cand = np.full((n, N), 0xFF, np.uint8)
    for c in range(n):
        kind = c % 6
        if kind == 0:
            v = np.zeros((N, K), np.uint8)
            perm = rng.permutation(K)
            v[np.arange(K), perm] = rng.integers(1, 256, K)
            v[K:] = rng.integers(0, 256, (N - K, K))
        elif kind == 1:
            v = (rng.integers(1, 256, (N, K)) * (rng.random((N, K)) < 0.3)).astype(np.uint8)
        elif kind == 2:
            v = rng.integers(0, 256, (N, K), dtype=np.uint8)
        elif kind == 3:
            v = rng.integers(0, 4, (N, K), dtype=np.uint8)
        else:
            v = rng.integers(0, 256, (N, K), dtype=np.uint8)
        order = rng.permutation(N)
        if kind == 4:  # a row among the first ten = a combination of two earlier ones
            i, j, t = sorted(rng.choice(K, 3, replace=False))
            a, b = int(rng.integers(1, 256)), int(rng.integers(1, 256))
            v[order[t]] = [o.gf_mul(a, int(x)) ^ o.gf_mul(b, int(y)) for x, y in zip(v[order[i]], v[order[j]])]
        if kind == 5 and c % 12 == 5:  # a repeated id among the first ten
            order[int(rng.integers(1, K))] = order[0]
        vecs[c] = v
        length = K + (c // 6) % (N - K + 1)
        cand[c, :length] = order[:length]
    host_rows = np.zeros((n * N, 16), np.uint8)
    host_rows[:, :K] = vecs.reshape(n * N, K)
    coded.view(n * N, F)[:, :16].copy_(dev(host_rows))
    return coded, vecs, cand


@pytest.mark.parametrize("form", ["plan_kernel", "fused", "fused_pairs"])
def test_repair_plan_fast_path_matches_oracle(ctx, form):
    """The plan's Gauss-Jordan fast path (first ten candidates valid; rlnc_kernels.hip plan_fast) in the plan
    kernel and in the fused plan + decode — one 128-chunkset launch (16-column tiles) or 64 launches of two
    (the default repair of small batches, 8-column tiles): verdicts, rank, sel and the inverse equal the oracle
    decoder's on row swaps, sparse and small-valued rows, lists of every length from 10, and first tens that
    are dependent (handed to the incremental form)."""
    from decds_amd._capi import lib
    n = 128
    coded, vecs, cand = _fast_path_inputs(n)
    plan = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(n * N, dtype=torch.int8, device="cuda")
    status = torch.full((n,), -7, dtype=torch.int32, device="cuda")
    if form == "plan_kernel":
        codec.repair_plan_batch(ctx, coded, n, dev(cand), plan, verd, status)
        st = host(status)
    elif form == "fused_pairs":
        assert lib().decds_repair_kernel_name(2) == b"rlnc_plan_decode_kernel"
        out = torch.empty(2 * CS, dtype=torch.uint8, device="cuda")
        cand_d = dev(cand)
        for c in range(0, n, 2):  # rows of chunksets c, c + 1: the coded buffer's view from row 16c
            codec.repair_batch(ctx, coded[c * N * F:], 2, cand_d[c:c + 2], plan[c * 128:], verd[c * N:], out, status[c:])
        st = host(status)
        ready = st != 5
        assert set(np.unique(st[ready]).tolist()) <= {6}
        st = np.where(ready, 0, st)
    else:
        lib().decds_tuning(b"DECDS_PLAN_DECODE_MAX_N", 1 << 62, 1)
        try:
            assert lib().decds_repair_kernel_name(n) == b"rlnc_plan_decode_kernel"
            out = torch.empty(n * CS, dtype=torch.uint8, device="cuda")
            codec.repair_batch(ctx, coded, n, dev(cand), plan, verd, out, status)
        finally:
            lib().decds_tuning(b"DECDS_PLAN_DECODE_MAX_N", (1 << 64) - 1, 1)
        st = host(status)
        ready = st != 5
        assert set(np.unique(st[ready]).tolist()) <= {6}  # zero payloads: no marker anywhere
        st = np.where(ready, 0, st)
    ranks = _check_plans_against_oracle(n, vecs, cand, st, host(verd).reshape(n, N), host(plan).reshape(n, 128))
    assert K in ranks and len(ranks) >= 2  # ready chunksets, and dependent tens that stay below rank 10


@pytest.fixture
def plan_decode_fused():
    """decds_repair_batch with plan + decode as one launch (rlnc_plan_decode_kernel) at any batch size"""
    from decds_amd._capi import lib
    lib().decds_tuning(b"DECDS_PLAN_DECODE_MAX_N", 1 << 62, 1)
    yield
    lib().decds_tuning(b"DECDS_PLAN_DECODE_MAX_N", (1 << 64) - 1, 1)


def test_fused_repair_plans_match_oracle_on_the_fuzz(ctx, plan_decode_fused):
    """The fused kernel's plans (each decode workgroup runs its chunkset's plan on one wave; the tile-0
    workgroup writes plan, verdicts and status) on the same 96 rank-deficient chunksets: identical to
    the oracle decoder's, as the plan kernel's. (Payloads are zero: every ready chunkset decodes to
    zeros, has no boundary marker anywhere, and ends ChunksetRepairingFailed.)"""
    from decds_amd._capi import lib
    assert lib().decds_repair_kernel_name(96) == b"rlnc_plan_decode_kernel"
    n = 96
    coded, vecs, cand = _fuzz_plan_inputs(n)
    plan = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(n * N, dtype=torch.int8, device="cuda")
    status = torch.full((n,), -7, dtype=torch.int32, device="cuda")
    out = torch.empty(n * CS, dtype=torch.uint8, device="cuda")
    codec.repair_batch(ctx, coded, n, dev(cand), plan, verd, out, status)
    st = host(status)
    ready = st != 5
    assert set(np.unique(st[ready]).tolist()) == {6}  # zero payloads: no marker anywhere
    st = np.where(ready, 0, st)
    ranks = _check_plans_against_oracle(n, vecs, cand, st, host(verd).reshape(n, N), host(plan).reshape(n, 128))
    assert len(ranks) >= 8


@pytest.mark.parametrize("n", [1, 2, 5, 16])
def test_fused_repair_equals_plan_then_decode(ctx, n):
    """decds_repair_batch in one launch (rlnc_plan_decode_kernel, forced at every n) against the plan kernel then
    the decode (the form above the threshold), each with 16- and 8-column lane blocks: plan bytes, verdicts,
    statuses, repair infos and every repaired byte identical, and the repaired chunksets equal their sources. Candidates: shuffled full
    lists, exactly 10, 9 (not ready), a repeated id, and a dependent row among the first 10."""
    from decds_amd._capi import lib
    rng = np.random.default_rng(0xF05E + n)
    data = o.fill_random(0xF05E0 + n, n * CS)
    coeffs = o.fill_random(0xF05E1 + n, n * N * K).reshape(n, N, K)
    if n >= 5:
        coeffs[4, 3] = coeffs[4, 1]           # chunkset 4: row 3 repeats row 1 (not useful when it arrives)
    cand = np.full((n, N), 0xFF, np.uint8)
    for c in range(n):
        kind = c % 5
        if kind == 0:
            cand[c] = rng.permutation(N)
        elif kind == 1:
            cand[c, :K] = rng.permutation(N)[:K]
        elif kind == 2:
            cand[c, :K - 1] = rng.permutation(N)[:K - 1]     # rank 9: not ready
        elif kind == 3:
            p = rng.permutation(N)
            cand[c, :12] = np.concatenate([p[:3], p[:1], p[3:11]])  # a repeated id
        else:
            cand[c, :13] = np.concatenate([[1, 3], rng.permutation([x for x in range(N) if x not in (1, 3)])[:11]])
    coded = torch.empty(n * N * F, dtype=torch.uint8, device="cuda")
    codec.encode_batch(ctx, dev(data), n, dev(coeffs.reshape(-1)), coded)
    res = {}
    # every form: fused / split, each with 16- and 8-column lane blocks (DECDS_DEC_NARROW_MAX_N)
    for form, limit in (("fused", 1 << 62), ("split", 0)):
        for cols, narrow in ((16, 0), (8, 1 << 62)):
            lib().decds_tuning(b"DECDS_PLAN_DECODE_MAX_N", limit, 1)
            lib().decds_tuning(b"DECDS_DEC_NARROW_MAX_N", narrow, 1)
            try:
                assert lib().decds_repair_kernel_name(n) == (b"rlnc_plan_decode_kernel" if form == "fused" else b"rlnc_plan_kernel")
                plan = torch.full((n * 128,), 0xEE, dtype=torch.uint8, device="cuda")
                verd = torch.full((n * N,), 99, dtype=torch.int8, device="cuda")
                status = torch.full((n,), -7, dtype=torch.int32, device="cuda")
                out = torch.zeros(n * CS, dtype=torch.uint8, device="cuda")
                info = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
                codec.repair_batch(ctx, coded, n, dev(cand), plan, verd, out, status, info=info)
                res[form, cols] = [host(t) for t in (plan, verd, status, out, info)]
            finally:
                lib().decds_tuning(b"DECDS_PLAN_DECODE_MAX_N", (1 << 64) - 1, 1)
                lib().decds_tuning(b"DECDS_DEC_NARROW_MAX_N", (1 << 64) - 1, 1)
    sp = res["split", 16]
    st = sp[2]
    ps = sp[0].reshape(n, 128)
    for key in (("fused", 16), ("fused", 8), ("split", 8)):
        f = res[key]
        assert np.array_equal(f[2], st) and np.array_equal(f[1], sp[1]), key
        pf = f[0].reshape(n, 128)
        for c in range(n):
            assert pf[c, 10] == ps[c, 10], (key, c)                       # rank
            if st[c] == 0:
                assert np.array_equal(pf[c, :K], ps[c, :K]) and np.array_equal(pf[c, 16:116], ps[c, 16:116]), (key, c)
                assert np.array_equal(f[3][c * CS:(c + 1) * CS], data[c * CS:(c + 1) * CS]), (key, c)
                assert np.array_equal(f[4][c * 16:c * 16 + 14], sp[4][c * 16:c * 16 + 14]), (key, c)
    for c in range(n):
        if st[c] == 0:
            assert np.array_equal(sp[3][c * CS:(c + 1) * CS], data[c * CS:(c + 1) * CS]), c
    assert set(st.tolist()) <= {0, 5} and (st == 5).sum() == sum(1 for c in range(n) if c % 5 == 2)


MARKER = 0x81


def _tail_cases():
    """Chunksets whose decoded data (the 10 pieces concatenated, CS + 10 bytes) ends other than in
    marker || 9 zeros — reachable through the public add_chunk_unvalidated (lib.rs:138,
    chunkset.rs:173-184). rlnc's get_decoded_data cuts at the LAST marker (oracle/rlnc_oracle.c
    orc_decoder_get_decoded_data). Each case: (name, data, {tail position: xor value})."""
    rng = np.random.default_rng(0x7A11)
    cases = []
    d = o.fill_random(41, CS)
    cases.append(("padding byte flipped", d, {3: 0x5A}))             # cut stays at CS
    cases.append(("padding byte set to the marker", o.fill_random(42, CS), {6: MARKER}))  # cut at CS + 6
    cases.append(("marker flipped", o.fill_random(43, CS), {0: MARKER}))  # cut at the data's last marker
    d = o.fill_random(44, CS).copy()
    p0 = CS - 3 * 4096 - 77                                          # marker moved earlier
    d[p0 + 1:][d[p0 + 1:] == MARKER] ^= 1
    d[p0] = MARKER
    cases.append(("marker moved earlier", d, {0: MARKER, 1: 0x33}))
    d = o.fill_random(45, CS).copy()
    d[d == MARKER] ^= 1                                              # no marker anywhere: an error
    cases.append(("no marker anywhere", d, {0: MARKER}))
    d = np.zeros(CS, np.uint8)
    d[:4 << 20] = o.fill_random(46, 4 << 20)                         # a blob's zero-padded last chunkset
    cases.append(("zero-padded chunkset, marker flipped", d, {0: MARKER}))
    cases.append(("intact", o.fill_random(47, CS), {}))
    cases.append(("several tail markers", o.fill_random(48, CS), {2: MARKER, 9: MARKER, 4: 7}))
    return cases, rng


def _corrupt_tail(coded, coeffs, flips):
    """coded rows of the padded pieces with piece 9's tail byte j (decoded position CS + j) xor'ed
    by v: multiplication by a coefficient is linear, so row r's payload byte changes by c[r][9] * v"""
    coded = coded.copy()
    for j, v in flips.items():
        col = K + L - K + j
        for r in range(N):
            coded[r, col] ^= o.gf_mul(int(coeffs[r, 9]), v)
    return coded


@pytest.mark.usefixtures("decode_form")
def test_decoded_data_cut_at_last_marker_matches_oracle(ctx):
    """get_decoded_data (chunkset.rs:200-208) on corrupted tails: the device batch decode (status,
    repair info, bytes), the chunkset mirror (add_chunk_unvalidated + repair), the host blob path and
    both CPU restatements (scalar decoder, blocked GFNI) give the same status and the same bytes."""
    cases, rng = _tail_cases()
    n = len(cases)
    data = np.concatenate([c[1] for c in cases])
    coeffs = o.fill_random(0xC0EF7A11, n * N * K).reshape(n, N, K)
    coded_d = torch.empty(n * N * F, dtype=torch.uint8, device="cuda")
    codec.encode_batch(ctx, dev(data), n, dev(coeffs), coded_d)
    coded = host(coded_d).reshape(n, N, F)
    coded = np.stack([_corrupt_tail(coded[c], coeffs[c], cases[c][2]) for c in range(n)])
    cand = np.full((n, N), 0xFF, np.uint8)
    for c in range(n):
        m = 10 if c % 2 else N
        cand[c, :m] = rng.permutation(N)[:m]
    plan = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(n * N, dtype=torch.int8, device="cuda")
    status = torch.full((n,), -7, dtype=torch.int32, device="cuda")
    info = torch.zeros(n * codec.REPAIR_INFO_BYTES, dtype=torch.uint8, device="cuda")
    out = torch.zeros(n * CS, dtype=torch.uint8, device="cuda")
    codec.repair_batch(ctx, dev(coded.reshape(-1)), n, dev(cand), plan, verd, out, status, info=info)
    st, res = host(status), host(out)
    lens, tails = codec.repair_info(info, n)
    fast_out, fast_st = (o.fast_blob_repair(coded.reshape(n * N, F), cand, n * CS, nthreads=8)
                         if o.fast_supported() else (None, None))
    blob_out, blob_st = o.blob_repair(coded.reshape(n * N, F), cand, n * CS, nthreads=8)
    host_out, host_st = codec.blob_repair_host(ctx, coded.reshape(n * N, F), cand, n * CS)
    seen = set()
    for c, (name, d, flips) in enumerate(cases):
        dec = o.Decoder()
        for r in cand[c]:
            if r == 0xFF or dec.is_already_decoded():
                break
            dec.decode(coded[c, r])
        assert dec.is_already_decoded(), name
        ost, obytes = dec.get_decoded_data()
        # the mirror: add_chunk_unvalidated in arrival order, then repair()
        rcs = decds_amd.RepairingChunkSet(ctx, c)
        for r in cand[c]:
            if r == 0xFF or rcs.is_ready_to_repair():
                break
            try:
                rcs.add_chunk_unvalidated(decds_amd.Chunk(c, c * N + int(r), coded[c, r].tobytes()))
            except decds_amd.DecdsError as e:
                assert e.kind == "ChunkDecodingFailed"
        sl = slice(c * CS, (c + 1) * CS)
        if ost == o.INVALID_DATA:
            seen.add("error")
            assert st[c] == 6, name
            with pytest.raises(decds_amd.DecdsError) as e:
                rcs.repair()
            assert e.value.kind == "ChunksetRepairingFailed", name
            assert blob_st[c] == o.INVALID_DATA and host_st[c] == 6, name
            assert fast_st is None or fast_st[c] == o.INVALID_DATA, name
            continue
        assert ost == o.OK and st[c] == 0, (name, ost, st[c])
        ln = len(obytes)
        seen.add("short" if ln < CS else "long" if ln > CS else "cs")
        assert lens[c] == ln, (name, lens[c], ln)
        assert codec.decoded_bytes(res[sl], lens[c], tails[c]) == obytes.tobytes(), name
        assert rcs.repair() == obytes.tobytes(), name
        # blob layout: the vector truncated to the chunkset (blob.rs:464), zeros past a short cut
        want = np.zeros(CS, np.uint8)
        want[:min(ln, CS)] = obytes[:CS]
        assert blob_st[c] == o.OK and np.array_equal(blob_out[sl], want), name
        assert host_st[c] == 0 and np.array_equal(host_out[sl], want), name
        if fast_st is not None:
            assert fast_st[c] == o.OK and np.array_equal(fast_out[sl], want), name
        if not flips:
            assert ln == CS and np.array_equal(res[sl], d), name
    assert seen == {"error", "short", "long", "cs"}


@pytest.mark.parametrize("n", [1, 256])
def test_no_marker_anywhere_worst_case_cost(ctx, n):
    from decds_amd._capi import lib
    lib().decds_tuning(b"DECDS_DEC_SWEEP_MIN_N", 256, 1)  # n = 256: the sweep (its default threshold is higher)
    try:
        _no_marker_worst_case(ctx, n)
    finally:
        lib().decds_tuning(b"DECDS_DEC_SWEEP_MIN_N", (1 << 64) - 1, 1)


def _no_marker_worst_case(ctx, n):
    """a chunkset whose decoded data holds no boundary marker at all (only rows accepted
    unvalidated get there) is decoded once more in full by its edge workgroup (tail_scan_decoded) before
    it is ChunksetRepairingFailed. Its cost, at n = 1 (one-tile decode) and inside a 256-chunkset batch
    (the sweep), against the same launch with every chunkset intact: status 6 for it, 0 and intact bytes
    for the others, the extra time recorded and bounded (print: `pytest -s`)."""
    import time
    d = o.fill_random(0xBAD0, CS).copy()
    d[d == MARKER] ^= 1
    data = np.concatenate([d] + [o.fill_random(0xB000 + c, CS) for c in range(1, n)])
    coeffs = o.fill_random(0xC0EFBAD0, n * N * K).reshape(n, N, K)
    coded_d = torch.empty(n * N * F, dtype=torch.uint8, device="cuda")
    codec.encode_batch(ctx, dev(data), n, dev(coeffs), coded_d)
    bad = coded_d.clone()
    bad[:N * F] = dev(_corrupt_tail(host(coded_d[:N * F]).reshape(N, F), coeffs[0], {0: MARKER}).reshape(-1))
    cand = dev(np.tile(np.arange(N, dtype=np.uint8), (n, 1)))
    plan = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(n * N, dtype=torch.int8, device="cuda")
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    out = torch.empty(n * CS, dtype=torch.uint8, device="cuda")
    ms = {}
    for name, rows in (("intact", coded_d), ("no_marker", bad)):
        codec.repair_plan_batch(ctx, rows, n, cand, plan, verd, status)
        codec.decode_batch(ctx, rows, n, plan, out, status)  # warm
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
        ev[0].record()
        for r in range(5):
            codec.decode_batch(ctx, rows, n, plan, out, status)
            ev[r + 1].record()
        torch.cuda.synchronize()
        ms[name] = float(np.median([ev[r].elapsed_time(ev[r + 1]) for r in range(5)]))
        st = host(status)
        assert st[0] == (6 if name == "no_marker" else 0), (name, st[:4])
        assert (st[1:] == 0).all(), name
        assert torch.equal(out[CS:], dev(data[CS:])), name
    extra = ms["no_marker"] - ms["intact"]
    print("no-marker worst case n=%d (%s): intact %.3f ms, no marker %.3f ms, extra %.3f ms"
          % (n, _lib_decode_name(n), ms["intact"], ms["no_marker"], extra))
    assert extra < 50.0, ms


def _lib_decode_name(n):
    from decds_amd._capi import lib
    return lib().decds_decode_kernel_name(n).decode()


@pytest.mark.usefixtures("decode_form")
def test_chunkset_mirror_roundtrip_like_reference(ctx):
    # chunkset.rs:257-283 (fixed seeds instead of rand::rng())
    for it in range(3):
        data = o.fill_random(500 + it, CS).tobytes()
        cs = decds_amd.ChunkSet(ctx, 0, data)
        rcs = decds_amd.RepairingChunkSet(ctx, 0)
        chunks = [cs.get_chunk(i) for i in range(N)]
        assert [c.chunk_id for c in chunks] == list(range(N))
        for j in np.random.default_rng(it).permutation(N):
            if rcs.is_ready_to_repair():
                break
            try:
                rcs.add_chunk_unvalidated(chunks[j])
            except decds_amd.DecdsError as e:
                assert e.kind == "ChunkDecodingFailed"
        assert rcs.repair() == data


def test_chunkset_mirror_errors(ctx):
    data = o.fill_random(600, CS).tobytes()
    coeffs = o.fill_random(601, N * K)
    cs = decds_amd.ChunkSet(ctx, 3, data, coeffs)
    # coded bytes equal the oracle at the pinned coding vectors
    ref = o.chunkset_encode(np.frombuffer(data, np.uint8), coeffs)
    assert all(cs.get_chunk(i).erasure_coded_data == ref[i].tobytes() for i in range(N))
    assert cs.get_chunk(5).chunk_id == 3 * N + 5                     # chunkset.rs:47
    for bad in (N, N + 100):                                         # chunkset.rs:300-315
        with pytest.raises(decds_amd.DecdsError) as e:
            cs.get_chunk(bad)
        assert e.value.kind == "InvalidErasureCodedShareId"
    for n in (CS - 1, CS + 1):                                       # chunkset.rs:285-298
        with pytest.raises(decds_amd.DecdsError) as e:
            decds_amd.ChunkSet(ctx, 0, bytes(n))
        assert e.value.kind == "InvalidChunksetSize"
    # chunkset.rs:419-436 invalid metadata
    with pytest.raises(decds_amd.DecdsError) as e:
        decds_amd.RepairingChunkSet(ctx, 1).add_chunk_unvalidated(cs.get_chunk(0))
    assert e.value.kind == "InvalidChunkMetadata"
    # chunkset.rs:438-453 not ready with 9
    rcs = decds_amd.RepairingChunkSet(ctx, 3)
    for i in range(K - 1):
        rcs.add_chunk_unvalidated(cs.get_chunk(i))
    assert not rcs.is_ready_to_repair()
    with pytest.raises(decds_amd.DecdsError) as e:
        rcs.repair()
    assert e.value.kind == "ChunksetNotYetReadyToRepair"
    # chunkset.rs:455-480 ready, then every further chunk is rejected, repair still succeeds
    rcs.add_chunk_unvalidated(cs.get_chunk(K - 1))
    assert rcs.is_ready_to_repair()
    for i in range(K, N):
        with pytest.raises(decds_amd.DecdsError) as e:
            rcs.add_chunk_unvalidated(cs.get_chunk(i))
        assert e.value.kind == "ChunksetReadyToRepair"
    assert rcs.repair() == data
    with pytest.raises(decds_amd.DecdsError) as e:
        rcs.repair()
    assert e.value.kind == "ChunksetAlreadyRepaired"
    # a duplicate chunk is not useful (rlnc decode error -> ChunkDecodingFailed)
    rcs2 = decds_amd.RepairingChunkSet(ctx, 3)
    rcs2.add_chunk_unvalidated(cs.get_chunk(0))
    with pytest.raises(decds_amd.DecdsError) as e:
        rcs2.add_chunk_unvalidated(cs.get_chunk(0))
    assert e.value.kind == "ChunkDecodingFailed"
    # a repair into a too-small buffer reports the decoded length and keeps the decoder (and its
    # result: the retry only copies); the repair that delivers the bytes consumes it
    import ctypes
    from decds_amd._capi import lib
    rcs3 = decds_amd.RepairingChunkSet(ctx, 3)
    for i in range(N - K, N):
        rcs3.add_chunk_unvalidated(cs.get_chunk(i))
    small, n_out = ctypes.create_string_buffer(64), ctypes.c_size_t()
    assert lib().decds_repairing_chunkset_repair(rcs3._h, small, 64, ctypes.byref(n_out)) == -2  # invalid argument
    assert n_out.value == CS and rcs3.is_ready_to_repair()
    assert rcs3.repair() == data
    assert not rcs3.is_ready_to_repair()


def test_blob_host_roundtrip_partial_last_chunkset(ctx):
    # blob.rs:767-837: 2.5 chunksets, pinned-staged host path, two batches
    blob_len = 2 * CS + CS // 2
    blob = o.fill_random(0xB10B, blob_len)
    n = 3
    coeffs = o.fill_random(0xC0EF, n * N * K)
    coded = codec.blob_encode_host(ctx, blob, coeffs, batch=2)
    assert np.array_equal(coded, o.blob_encode(blob, coeffs, nthreads=8))
    cand = np.stack([np.random.default_rng(c).permutation(N) for c in range(n)]).astype(np.uint8)
    out, status = codec.blob_repair_host(ctx, coded, cand, blob_len, batch=2)
    assert (status == 0).all() and np.array_equal(out, blob)
    with pytest.raises(decds_amd.DecdsError) as e:
        codec.blob_encode_host(ctx, np.zeros(0, np.uint8), np.zeros(0, np.uint8))
    assert e.value.kind == "EmptyDataForBlob"


def test_device_fill_random_matches_host(ctx):
    t = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
    codec.fill_random_device(ctx, 0xDEC05001, t)
    assert np.array_equal(host(t), o.fill_random(0xDEC05001, 1 << 20))
    t2 = torch.empty(1001, dtype=torch.uint8, device="cuda")
    codec.fill_random_device(ctx, 9, t2, byte_offset=13)
    assert np.array_equal(host(t2), o.fill_random(9, 1001, 13))


def test_cfg2_one_gib_encode_repair_device_resident(ctx):
    """BASELINE config 2: 1 GiB blob (103 chunksets, last one 4 MiB of data) encoded in one batch and
    repaired from exactly 10 random survivors per chunkset; spot chunksets bit-exact vs the oracle,
    every repaired chunkset equal to the source, rank-deficient ones reported not-ready."""
    blob_len = 1 << 30
    n = -(-blob_len // CS)
    assert n == 103
    src = torch.zeros(n * CS, dtype=torch.uint8, device="cuda")
    codec.fill_random_device(ctx, 0xDEC05002, src, nbytes=blob_len)
    coeffs = o.fill_random(0xC0EF0002, n * N * K)
    coded = torch.empty(n * N * F, dtype=torch.uint8, device="cuda")
    codec.encode_batch(ctx, src, n, dev(coeffs), coded)
    torch.cuda.synchronize()
    for c in (0, 57, n - 1):
        data_c = src[c * CS:(c + 1) * CS].cpu().numpy()
        ref = o.chunkset_encode(data_c, coeffs[c * 160:(c + 1) * 160], nthreads=8)
        assert np.array_equal(coded[c * N * F:(c + 1) * N * F].cpu().numpy().reshape(N, F), ref), c
    rng = np.random.default_rng(0x5EED0002)
    cand = np.full((n, N), 0xFF, np.uint8)
    for c in range(n):
        cand[c, :K] = rng.permutation(N)[:K]
    plan = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(n * N, dtype=torch.int8, device="cuda")
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    out = torch.zeros(n * CS, dtype=torch.uint8, device="cuda")
    codec.repair_batch(ctx, coded, n, dev(cand), plan, verd, out, status)
    st = host(status)
    cv = coeffs.reshape(n, N, K)
    for c in range(n):
        _, rank = _oracle_verdicts(np.concatenate([cv[c], np.zeros((N, 3), np.uint8)], axis=1), cand[c])
        assert st[c] == (0 if rank == K else 5)
    ok = torch.from_numpy(st == 0).cuda().repeat_interleave(CS)
    assert torch.equal(out[ok], src[ok])


@pytest.mark.parametrize("pitch,off", [(F + 4093, 0), (F + 5, 0), (F + 5, 9)])
@pytest.mark.usefixtures("decode_form")
def test_repair_pitch_and_repeated_candidates(ctx, pitch, off):
    # decode from a padded coded layout (16-byte-aligned pitches: block loads at a column phase);
    # a candidate row repeated in the arrival order is not useful
    n = 2
    data = o.fill_random(0xDEC05004, n * CS)
    coeffs = o.fill_random(0xC0EF0004, n * N * K)
    coded = torch.empty(off + (n * N - 1) * pitch + F, dtype=torch.uint8, device="cuda")[off:]
    codec.encode_batch(ctx, dev(data), n, dev(coeffs), coded, pitch)
    cand = np.full((n, N), 0xFF, np.uint8)
    cand[0, :12] = [3, 3, 7, 1, 0, 15, 2, 9, 11, 4, 5, 6]
    cand[1, :16] = np.random.default_rng(8).permutation(N)
    plan = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(n * N, dtype=torch.int8, device="cuda")
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    out = torch.zeros(n * CS, dtype=torch.uint8, device="cuda")
    codec.repair_batch(ctx, coded, n, dev(cand), plan, verd, out, status, pitch)
    v = host(verd).reshape(n, N)
    assert v[0, 1] == NOT_USEFUL
    ch = host(coded)
    for c in range(n):
        rows = np.stack([ch[(c * N + r) * pitch:(c * N + r) * pitch + F] for r in range(N)])
        assert list(v[c]) == _oracle_verdicts(rows, cand[c])[0]
    st = host(status)
    res = host(out)
    for c in range(n):
        if st[c] == 0:
            assert np.array_equal(res[c * CS:(c + 1) * CS], data[c * CS:(c + 1) * CS])
    assert st[0] == 0


@pytest.mark.parametrize("blob_len", [1, 4093, CS - 1, CS, CS + 1, 3 * CS + 12345])
@pytest.mark.usefixtures("decode_form")
def test_blob_all_chunks_shuffled_roundtrip(ctx, blob_len):
    """tests.rs:4-57: build a blob, shuffle ALL 16*n chunks of all chunksets together, feed them to
    the repairing blob in that order (each chunkset sees its own chunks in their global order), and
    get the blob back; coded bytes equal the oracle's. Sizes: 1 B, odd, either side of one
    chunkset, and a ragged multi-chunkset blob (the reference draws 1 B ... 256 MiB)."""
    blob = o.fill_random(0xB10D + blob_len, blob_len)
    n = -(-blob_len // CS)
    coeffs = o.fill_random(0xC0F1 + blob_len, n * N * K)
    coded = codec.blob_encode_host(ctx, blob, coeffs, batch=2)
    assert np.array_equal(coded, o.blob_encode(blob, coeffs, nthreads=8))
    order = np.random.default_rng(blob_len).permutation(n * N)   # global chunk ids c*16 + j
    cand = np.full((n, N), 0xFF, np.uint8)
    fill = np.zeros(n, np.int64)
    for gid in order:
        c, j = divmod(int(gid), N)
        cand[c, fill[c]] = j
        fill[c] += 1
    out, status = codec.blob_repair_host(ctx, coded, cand, blob_len, batch=2)
    assert (status == 0).all() and np.array_equal(out, blob)


@pytest.mark.usefixtures("decode_form")
def test_blob_host_not_ready_chunkset(ctx):
    blob_len = CS + 777
    blob = o.fill_random(0xB10C, blob_len)
    coeffs = o.fill_random(0xC0F0, 2 * N * K)
    coded = codec.blob_encode_host(ctx, blob, coeffs)
    cand = np.stack([np.random.default_rng(c).permutation(N) for c in range(2)]).astype(np.uint8)
    cand[1, 9:] = 0xFF                                   # only 9 chunks of chunkset 1 arrive
    out, status = codec.blob_repair_host(ctx, coded, cand, blob_len)
    assert status[0] == 0 and status[1] == 5
    assert np.array_equal(out[:CS], blob[:CS]) and not out[CS:].any()


def test_encode_large_n_last_chunkset_bounds(ctx):
    # the last chunkset of a large batch sits at the very end of its allocations
    n = 40
    src = torch.empty(n * CS, dtype=torch.uint8, device="cuda")
    codec.fill_random_device(ctx, 0xABCD, src)
    coeffs = o.fill_random(0xC0EF0005, n * N * K)
    coded = torch.empty(n * N * F, dtype=torch.uint8, device="cuda")
    codec.encode_batch(ctx, src, n, dev(coeffs), coded)
    torch.cuda.synchronize()
    c = n - 1
    ref = o.chunkset_encode(src[c * CS:].cpu().numpy(), coeffs[c * 160:], nthreads=8)
    assert np.array_equal(coded[c * N * F:].cpu().numpy().reshape(N, F), ref)


def test_encode_batch_above_512_bitexact(ctx):
    # a batch past the old units-of-8 threshold (512 chunksets): XCD eighths of 65 chunksets, last
    # eighth shorter; first, middle and last chunksets bit-exact against the oracle
    n = 520
    src = torch.empty(n * CS, dtype=torch.uint8, device="cuda")
    codec.fill_random_device(ctx, 0xABCE, src)
    coeffs = o.fill_random(0xC0EF0006, n * N * K)
    coded = torch.empty(n * N * F, dtype=torch.uint8, device="cuda")
    codec.encode_batch(ctx, src, n, dev(coeffs), coded)
    torch.cuda.synchronize()
    for c in (0, 64, 65, 259, n - 1):
        ref = o.chunkset_encode(src[c * CS:(c + 1) * CS].cpu().numpy(), coeffs[c * 160:(c + 1) * 160], nthreads=8)
        assert np.array_equal(coded[c * N * F:(c + 1) * N * F].cpu().numpy().reshape(N, F), ref), c
    del src, coded


@pytest.mark.parametrize("trial", range(6))
@pytest.mark.usefixtures("decode_form")
def test_randomized_layouts_encode_repair(ctx, trial):
    # seeded random batch shapes through both kernels: batch sizes that pick every unit size
    # (encode 4 / decode 2 / 4 / 8 tiles), rlnc-pitch and 16-byte-aligned pitches at any base offset
    # (column phases 0..15), survivor subsets of 10..16 rows in random arrival order
    rng = np.random.default_rng(0x7A1A1 + trial)
    n = int(rng.choice([1, 2, 3, 4, 5, 9, 17]))
    pitch = int(rng.choice([F, F + 1, F + 5, F + 13, F + 117, F + 4096, 1 << 21]))
    off = int(rng.integers(0, 16))
    data = o.fill_random(0xDEC06000 + trial, n * CS)
    coeffs = o.fill_random(0xC0EF6000 + trial, n * N * K)
    coded = torch.zeros(off + (n * N - 1) * pitch + F, dtype=torch.uint8, device="cuda")[off:]
    codec.encode_batch(ctx, dev(data), n, dev(coeffs), coded, pitch)
    rows = host(coded.as_strided((n * N, F), (pitch, 1)))
    for c in sorted({0, n - 1, int(rng.integers(0, n))}):
        ref = o.chunkset_encode(data[c * CS:(c + 1) * CS], coeffs[c * 160:(c + 1) * 160], nthreads=8)
        assert np.array_equal(rows[c * N:(c + 1) * N], ref), (trial, n, pitch, off, c)
    cand = np.full((n, N), 0xFF, np.uint8)
    for c in range(n):
        m = int(rng.integers(K, N + 1))
        cand[c, :m] = rng.permutation(N)[:m]
    plan = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(n * N, dtype=torch.int8, device="cuda")
    status = torch.full((n,), -7, dtype=torch.int32, device="cuda")
    out = torch.zeros(n * CS, dtype=torch.uint8, device="cuda")
    codec.repair_batch(ctx, coded, n, dev(cand), plan, verd, out, status, pitch=pitch)
    st, v, res = host(status), host(verd).reshape(n, N), host(out)
    for c in range(n):
        ov, rank = _oracle_verdicts(rows[c * N:(c + 1) * N], cand[c])
        assert list(v[c]) == ov, (trial, c)
        assert st[c] == (0 if rank == K else 5), (trial, c)
        if rank == K:
            assert np.array_equal(res[c * CS:(c + 1) * CS], data[c * CS:(c + 1) * CS]), (trial, n, pitch, off, c)


@pytest.mark.parametrize("n", [3, 20])
@pytest.mark.usefixtures("decode_form")
def test_aligned_device_layout_roundtrip(ctx, n):
    # the recommended device layout (include/decds_rlnc.h): pitch 1,048,704, payloads 128-byte aligned;
    # n = 3 runs the small-batch encode (units of 1 tile), n = 20 the units of 4 with XCD eighths
    data = o.fill_random(0xA11A + n, n * CS)
    coeffs = o.fill_random(0xA11B + n, n * N * K)
    coded, pitch = codec.coded_buffer(n)
    assert pitch == 1048704 and (coded.data_ptr() + K) % 128 == 0
    codec.encode_batch(ctx, dev(data), n, dev(coeffs), coded, pitch)
    rows = host(coded.as_strided((n * N, F), (pitch, 1)))
    for c in sorted({0, n // 2, n - 1}):
        ref = o.chunkset_encode(data[c * CS:(c + 1) * CS], coeffs[c * 160:(c + 1) * 160], nthreads=8)
        assert np.array_equal(rows[c * N:(c + 1) * N], ref), c
    cand = np.stack([np.random.default_rng(c).permutation(N) for c in range(n)]).astype(np.uint8)
    plan = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    verd = torch.empty(n * N, dtype=torch.int8, device="cuda")
    status = torch.full((n,), -7, dtype=torch.int32, device="cuda")
    out = torch.zeros(n * CS, dtype=torch.uint8, device="cuda")
    codec.repair_batch(ctx, coded, n, dev(cand), plan, verd, out, status, pitch=pitch)
    assert (host(status) == 0).all() and np.array_equal(host(out), data)

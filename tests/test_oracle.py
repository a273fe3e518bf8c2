"""CPU tests of the restatement (oracle/) against the committed known-answer vectors and the
reference's own round-trip properties (chunkset.rs:257-283, 438-480; tests.rs:4-57)."""
import hashlib

import numpy as np
import pytest

import oracle as o


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_field_known_answers(kat):
    t = o.mul_table()
    assert sha(t) == kat["mul_table_sha256"]
    assert sha(o.mul_table(0x11B)) == kat["mul_table_sha256_poly_0x11b"]
    for a, b, p in kat["products"]:
        assert t[a, b] == p
    for a, inv in kat["inverses"]:
        assert o.gf_inv(a) == inv and t[a, inv] == 1


def test_field_axioms():
    t = o.mul_table().astype(np.int64)
    rng = np.random.default_rng(1)
    a, b, c = rng.integers(0, 256, (3, 2000))
    assert np.array_equal(t[a, b], t[b, a])
    assert np.array_equal(t[t[a, b], c], t[a, t[b, c]])
    assert np.array_equal(t[a, b ^ c], t[a, b] ^ t[a, c])          # distributive over XOR (add)
    assert all(t[x, o.gf_inv(x)] == 1 for x in range(1, 256))
    assert len(set(t[2 ** 0 if False else 2, :].tolist())) == 256  # 2 is a unit; the map is a bijection


def test_small_encode_vectors(kat):
    for v in kat["small_encode"]:
        data = np.frombuffer(bytes.fromhex(v["data"]), dtype=np.uint8)
        cv = np.frombuffer(bytes.fromhex(v["coding_vector"]), dtype=np.uint8)
        piece = o.code_with_coding_vector(data, cv)
        assert piece.tobytes().hex() == v["full_coded_piece"]
        # structure: cv prefix, then L = ceil((len+1)/k) payload bytes (chunkset.rs:117)
        assert piece[:10].tobytes() == cv.tobytes()
        assert piece.size == 10 + (data.size + 1 + 9) // 10


def test_encoder_padding_layout():
    data = o.fill_random(5, o.CS)
    padded = o.encoder_pad(data)
    assert padded.size == o.K * o.L
    assert np.array_equal(padded[: o.CS], data)
    assert padded[o.CS] == o.MARKER and not padded[o.CS + 1:].any()


def test_cfg1_full_chunkset_golden(kat):
    c = kat["cfg1"]
    data = o.fill_random(c["data_seed"], o.CS)
    assert sha(data) == c["data_sha256"]
    coeffs = np.frombuffer(bytes.fromhex(c["coeffs"]), dtype=np.uint8)
    coded = o.chunkset_encode(data, coeffs, nthreads=8)
    assert [sha(coded[j]) for j in range(16)] == c["coded_sha256"]


def test_chunkset_encode_invalid_size():
    # chunkset.rs:285-298: InvalidChunksetSize for CS-1 and CS+1
    for n in (o.CS - 1, o.CS + 1):
        with pytest.raises(ValueError):
            o.chunkset_encode(np.zeros(n, np.uint8), np.ones(160, np.uint8))


def _roundtrip(data_len, seed, k=10):
    data = o.fill_random(seed, data_len)
    L = o.piece_len(data_len, k)
    rng = np.random.default_rng(seed)
    dec = o.Decoder(L, k)
    pieces = 0
    while not dec.is_already_decoded():
        cv = rng.integers(0, 256, k, dtype=np.uint8)
        st = dec.decode(o.code_with_coding_vector(data, cv, k))
        assert st in (o.OK, o.NOT_USEFUL)
        pieces += 1
    st, out = dec.get_decoded_data()
    assert st == o.OK
    assert np.array_equal(out, data)
    assert dec.decode(o.code_with_coding_vector(data, np.ones(k, np.uint8), k)) == o.RECEIVED_ALL


@pytest.mark.parametrize("n", [1, 9, 10, 11, 1000, 4097])
def test_decoder_roundtrip_small(n):
    _roundtrip(n, 100 + n)


def test_decoder_not_useful_and_state_unchanged():
    data = o.fill_random(9, 500)
    dec = o.Decoder(o.piece_len(500), 10)
    cv1 = np.arange(1, 11, dtype=np.uint8)
    assert dec.decode(o.code_with_coding_vector(data, cv1)) == o.OK
    # a multiple of an accepted vector does not raise the rank (rlnc: piece not useful)
    cv2 = np.array([o.gf_mul(7, int(x)) for x in cv1], dtype=np.uint8)
    assert dec.decode(o.code_with_coding_vector(data, cv2)) == o.NOT_USEFUL
    assert dec.rank() == 1
    assert dec.decode(np.zeros(10 + o.piece_len(500), np.uint8)) == o.NOT_USEFUL
    assert dec.decode(np.zeros(5, np.uint8)) == o.INVALID_LEN
    assert dec.get_decoded_data()[0] == o.NOT_ALL


def test_full_chunkset_roundtrip_shuffled():
    # chunkset.rs:257-283 with a fixed seed: encode, shuffle the 16 chunks, add until ready
    data = o.fill_random(77, o.CS)
    coeffs = o.fill_random(78, 160)
    coded = o.chunkset_encode(data, coeffs, nthreads=8)
    order = np.random.default_rng(3).permutation(16)
    dec = o.Decoder()
    for j in order:
        if dec.is_already_decoded():
            break
        assert dec.decode(coded[j]) in (o.OK, o.NOT_USEFUL)
    st, out = dec.get_decoded_data()
    assert st == o.OK and out.size == o.CS and np.array_equal(out, data)


def test_rank_push_matches_decoder():
    rng = np.random.default_rng(5)
    for trial in range(200):
        basis = np.zeros(100, np.uint8)
        piv = np.zeros(10, np.uint8)
        import ctypes
        rank = ctypes.c_size_t(0)
        dec = o.Decoder(3, 10)
        for _ in range(14):
            # low-entropy vectors so dependent ones actually occur
            cv = (rng.integers(0, 3, 10) * rng.integers(0, 2, 10)).astype(np.uint8)
            useful = o.lib().orc_rank_push(o._p(basis), o._p(piv), ctypes.byref(rank), o._p(cv), 10, o.POLY)
            if dec.is_already_decoded():
                assert not useful
                continue
            st = dec.decode(np.concatenate([cv, np.zeros(3, np.uint8)]))
            assert (st == o.OK) == bool(useful)
        assert rank.value == dec.rank()


def test_matrix_inverse():
    rng = np.random.default_rng(6)
    t = o.mul_table()
    for _ in range(20):
        m = rng.integers(0, 256, (10, 10), dtype=np.uint8)
        inv = o.matrix_inverse(m)
        if inv is None:
            continue
        prod = np.zeros((10, 10), np.uint8)
        for i in range(10):
            for j in range(10):
                acc = 0
                for kk in range(10):
                    acc ^= int(t[m[i, kk], inv[kk, j]])
                prod[i, j] = acc
        assert np.array_equal(prod, np.eye(10, dtype=np.uint8))


def test_blob_encode_repair_partial_last_chunkset():
    # blob.rs:767-837: a blob of 2.5 chunksets; the last one is zero-padded and truncated on repair
    blob_len = 2 * o.CS + o.CS // 2
    blob = o.fill_random(21, blob_len)
    n = 3
    coeffs = o.fill_random(22, n * 160)
    coded = o.blob_encode(blob, coeffs, nthreads=4)
    cand = np.array([np.random.default_rng(c).permutation(16) for c in range(n)], np.uint8)
    out, status = o.blob_repair(coded, cand, blob_len, nthreads=4)
    assert (status == 0).all() and np.array_equal(out, blob)


def test_simd_row_kernels_match_scalar():
    # the AVX2 nibble-table row kernels (bench.py's stronger CPU baseline) produce the scalar
    # restatement's bytes: encode of two chunksets (one partial) and the repair of both
    blob = o.fill_random(0x51D0, o.CS + 12345)
    coeffs = o.fill_random(0x51D1, 2 * o.N * o.K)
    cand = np.full((2, o.N), 0xFF, np.uint8)
    rng = np.random.default_rng(5)
    for c in range(2):
        cand[c, :o.K + 2] = rng.permutation(o.N)[:o.K + 2]
    o.set_simd(0)
    ref = o.blob_encode(blob, coeffs, nthreads=4)
    ref_out, ref_st = o.blob_repair(ref, cand, blob.size, nthreads=4)
    try:
        if not o.set_simd(1):
            pytest.skip("no AVX2 on this host")
        got = o.blob_encode(blob, coeffs, nthreads=4)
        out, st = o.blob_repair(got, cand, blob.size, nthreads=4)
    finally:
        o.set_simd(0)
    assert np.array_equal(got, ref)
    assert np.array_equal(st, ref_st) and np.array_equal(out, ref_out)
    assert np.array_equal(out[:blob.size], blob)


@pytest.mark.parametrize("poly", [0x11D, 0x11B])
def test_fast_gfni_codec_matches_scalar(poly):
    # bench.py's headline CPU baseline (rlnc_cpu_fast.c: column-blocked, GFNI affine multiplies,
    # coefficient-only rank + inverse for the repair) gives the scalar restatement's bytes and
    # verdicts: full, partial (piece 9 cut mid-block) and 1-byte last chunksets; rank-deficient,
    # repeated and short candidate lists
    if not o.fast_supported():
        pytest.skip("no AVX-512 + GFNI on this host")
    for blob_len in (2 * o.CS + 9 * o.L + 5, o.CS + 1):
        n = -(-blob_len // o.CS)
        blob = o.fill_random(0xFA57 + blob_len, blob_len)
        coeffs = o.fill_random(0xFA58, n * o.N * o.K)
        ref = o.blob_encode(blob, coeffs, poly=poly, nthreads=4)
        got = o.fast_blob_encode(blob, coeffs, poly=poly, nthreads=4)
        assert np.array_equal(got, ref)
        cand = np.full((n, o.N), 0xFF, np.uint8)
        rng = np.random.default_rng(blob_len)
        cand[0, :o.K + 3] = rng.permutation(o.N)[:o.K + 3]
        cand[1, :9] = rng.permutation(o.N)[:9]                      # not enough
        if n > 2:
            cand[2, :o.N] = np.concatenate([[3, 3, 5, 3], rng.permutation(o.N)[:12]])  # repeats
        ref_out, ref_st = o.blob_repair(ref, cand, blob_len, poly=poly, nthreads=4)
        out, st = o.fast_blob_repair(got, cand, blob_len, poly=poly, nthreads=4)
        assert np.array_equal(st, ref_st), (st, ref_st)
        assert np.array_equal(out, ref_out)
        assert ref_st[0] == 0 and ref_st[1] == o.NOT_ALL


def test_gf_affine_matrix_is_multiplication():
    if not o.fast_supported():
        pytest.skip("no AVX-512 + GFNI on this host")
    t = o.mul_table()
    for c in (0, 1, 2, 0x53, 0x81, 0xFF):
        a = int(o.lib().orc_gf_affine_matrix(c, o.POLY))
        for x in range(256):
            y = 0
            for i in range(8):
                row = (a >> (8 * (7 - i))) & 0xFF
                y |= (bin(row & x).count("1") & 1) << i
            assert y == t[c, x]


def test_decoded_data_cut_at_last_marker_restatements_agree():
    # rlnc get_decoded_data (chunkset.rs:200-208) cuts the decoded pieces at the LAST boundary marker:
    # the scalar decoder, the scalar blob driver and the blocked GFNI codec agree on corrupted tails
    # (rows accepted unvalidated): padding flipped (cut stays at CS), padding turned into the marker
    # (cut past CS, truncated to the chunkset), marker flipped (cut inside the data; in a blob's last,
    # zero-padded chunkset below its real size: zeros past the cut) and no marker at all (an error)
    K, N, CS, L, M = o.K, o.N, o.CS, o.L, o.MARKER
    d_nomark = o.fill_random(0x7A13, CS).copy()
    d_nomark[d_nomark == M] ^= 1
    d_last = np.zeros(CS, np.uint8)
    d_last[:3 << 20] = o.fill_random(0x7A14, 3 << 20)
    cases = [(o.fill_random(0x7A10, CS), {}), (o.fill_random(0x7A11, CS), {4: 0x5A}),
             (o.fill_random(0x7A12, CS), {6: M}), (o.fill_random(0x7A15, CS), {0: M}),
             (d_nomark, {0: M}), (d_last, {0: M})]
    n = len(cases)
    blob_len = (n - 1) * CS + (4 << 20)                   # the last chunkset holds 4 MiB of the blob
    data = np.concatenate([c[0] for c in cases])
    coeffs = o.fill_random(0x7A16, n * N * K).reshape(n, N, K)
    coded = o.blob_encode(data, coeffs, nthreads=8).reshape(n, N, o.F)
    for c, (_, flips) in enumerate(cases):               # piece 9's tail byte j changes by v (linearity)
        for j, v in flips.items():
            for r in range(N):
                coded[c, r, K + L - K + j] ^= o.gf_mul(int(coeffs[c, r, 9]), v)
    cand = np.tile(np.arange(N, dtype=np.uint8), (n, 1))
    ref_out, ref_st = o.blob_repair(coded.reshape(n * N, o.F), cand, blob_len, nthreads=8)
    if o.fast_supported():
        out, st = o.fast_blob_repair(coded.reshape(n * N, o.F), cand, blob_len, nthreads=8)
        assert np.array_equal(st, ref_st) and np.array_equal(out, ref_out)
    lens = []
    for c in range(n):
        dec = o.Decoder()
        for r in range(K):
            assert dec.decode(coded[c, r]) == o.OK
        st, got = dec.get_decoded_data()
        assert st == ref_st[c]
        if st != o.OK:
            lens.append(None)
            continue
        lens.append(len(got))
        keep = min(CS, blob_len - c * CS)
        want = np.zeros(keep, np.uint8)
        want[:min(len(got), keep)] = got[:keep]
        assert np.array_equal(ref_out[c * CS:c * CS + keep], want), c
    last = int(np.nonzero(cases[3][0] == M)[0][-1])
    last5 = int(np.nonzero(d_last == M)[0][-1])
    assert lens == [CS, CS, CS + 6, last, None, last5]
    assert list(ref_st) == [o.OK] * 4 + [o.INVALID_DATA, o.OK]

"""ctypes wrapper of the CPU restatement in oracle/ (liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, always as the checker / CPU baseline, never by the decds_amd product path. Parity status and
the reference lines restated: see rlnc_oracle.h.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")

K, N = 10, 16
CS = 10 * (1 << 20)
L = (CS + 1 + K - 1) // K
F = L + K
POLY = 0x11D
MARKER = 0x81

OK, NOT_USEFUL, RECEIVED_ALL, INVALID_LEN, NOT_ALL, INVALID_DATA, INVALID_CS_SIZE = 0, 1, 2, 3, 4, 5, 6

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        c = ctypes
        L_ = c.CDLL(LIB)
        vp, sz, u8, u32, u64 = c.c_void_p, c.c_size_t, c.c_uint8, c.c_uint32, c.c_uint64
        for name, res, args in [
            ("orc_gf256_mul", u8, [u8, u8, u32]),
            ("orc_gf256_inv", u8, [u8, u32]),
            ("orc_set_simd", c.c_int, [c.c_int]),
            ("orc_gf256_mul_table", None, [u32, vp]),
            ("orc_splitmix64_word", u64, [u64, u64]),
            ("orc_fill_random", None, [u64, u64, vp, sz]),
            ("orc_piece_len", sz, [sz, sz]),
            ("orc_encoder_pad", c.c_int, [vp, sz, sz, u8, vp]),
            ("orc_code_with_coding_vector", None, [vp, sz, sz, vp, vp, u32]),
            ("orc_chunkset_encode", c.c_int, [vp, sz, vp, vp, u32, u8, c.c_int]),
            ("orc_decoder_new", vp, [sz, sz, u32, u8]),
            ("orc_decoder_free", None, [vp]),
            ("orc_decoder_decode", c.c_int, [vp, vp, sz]),
            ("orc_decoder_is_decoded", c.c_int, [vp]),
            ("orc_decoder_rank", sz, [vp]),
            ("orc_decoder_get_decoded_data", c.c_int, [vp, vp, sz, c.POINTER(sz)]),
            ("orc_rank_push", c.c_int, [vp, vp, c.POINTER(sz), vp, sz, u32]),
            ("orc_matrix_inverse", c.c_int, [vp, vp, sz, u32]),
            ("orc_blob_encode", c.c_int, [vp, sz, vp, vp, u32, u8, c.c_int]),
            ("orc_blob_repair", c.c_int, [vp, sz, vp, sz, vp, vp, u32, u8, c.c_int]),
            ("orc_fast_supported", c.c_int, []),
            ("orc_gf_affine_matrix", u64, [u8, u32]),
            ("orc_fast_blob_encode", c.c_int, [vp, sz, vp, vp, u32, u8, c.c_int]),
            ("orc_fast_blob_repair", c.c_int, [vp, sz, vp, sz, vp, vp, u32, u8, c.c_int]),
            ("orc_blake3", None, [vp, sz, vp]),
            ("orc_chunk_digest", None, [u64, u64, vp, sz, vp]),
            ("orc_chunk_digest_rows", None, [vp, sz, sz, u64, vp]),
            ("orc_merkle", c.c_int, [vp, sz, vp, vp]),
            ("orc_merkle_verify", c.c_int, [sz, vp, vp, sz, vp]),
        ]:
            f = getattr(L_, name)
            f.restype, f.argtypes = res, args
        _lib = L_
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def set_simd(on):
    """AVX2 nibble-table row kernels (same bytes as the scalar restatement); returns the mode in effect"""
    return lib().orc_set_simd(int(bool(on)))


def gf_mul(a, b, poly=POLY):
    return lib().orc_gf256_mul(a, b, poly)


def gf_inv(a, poly=POLY):
    return lib().orc_gf256_inv(a, poly)


def mul_table(poly=POLY):
    t = np.empty(256 * 256, dtype=np.uint8)
    lib().orc_gf256_mul_table(poly, _p(t))
    return t.reshape(256, 256)


def fill_random(seed, nbytes, byte_offset=0):
    out = np.empty(nbytes, dtype=np.uint8)
    lib().orc_fill_random(seed, byte_offset, _p(out), nbytes)
    return out


def piece_len(data_len, k=K):
    return lib().orc_piece_len(data_len, k)


def encoder_pad(data, k=K, marker=MARKER):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    out = np.empty(k * piece_len(data.size, k), dtype=np.uint8)
    st = lib().orc_encoder_pad(_p(data), data.size, k, marker, _p(out))
    assert st == OK
    return out


def code_with_coding_vector(data, cv, k=K, poly=POLY, marker=MARKER):
    """rlnc Encoder::new(data, k) + code() with an explicit coding vector -> full coded piece."""
    padded = encoder_pad(data, k, marker)
    L_ = padded.size // k
    cv = np.ascontiguousarray(cv, dtype=np.uint8)
    out = np.empty(k + L_, dtype=np.uint8)
    lib().orc_code_with_coding_vector(_p(padded), L_, k, _p(cv), _p(out), poly)
    return out


def chunkset_encode(data, coeffs, poly=POLY, marker=MARKER, nthreads=1):
    """ChunkSet::new's RLNC part: (16, F) full coded pieces."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    coeffs = np.ascontiguousarray(coeffs, dtype=np.uint8).reshape(N * K)
    out = np.empty((N, F), dtype=np.uint8)
    st = lib().orc_chunkset_encode(_p(data), data.size, _p(coeffs), _p(out), poly, marker, nthreads)
    if st != OK:
        raise ValueError("orc_chunkset_encode status %d" % st)
    return out


class Decoder:
    """rlnc Decoder restatement (incremental RREF)."""

    def __init__(self, piece_len=L, k=K, poly=POLY, marker=MARKER):
        self.k, self.piece_len = k, piece_len
        self._h = lib().orc_decoder_new(piece_len, k, poly, marker)

    def decode(self, piece):
        piece = np.ascontiguousarray(np.frombuffer(piece, dtype=np.uint8) if isinstance(piece, bytes) else piece,
                                     dtype=np.uint8)
        return lib().orc_decoder_decode(self._h, _p(piece), piece.size)

    def is_already_decoded(self):
        return bool(lib().orc_decoder_is_decoded(self._h))

    def rank(self):
        return lib().orc_decoder_rank(self._h)

    def get_decoded_data(self):
        out = np.empty(self.k * self.piece_len, dtype=np.uint8)
        n = ctypes.c_size_t()
        st = lib().orc_decoder_get_decoded_data(self._h, _p(out), out.size, ctypes.byref(n))
        return st, out[: n.value] if st == OK else None

    def __del__(self):
        try:
            lib().orc_decoder_free(self._h)
        except Exception:
            pass


def matrix_inverse(m, k=K, poly=POLY):
    m = np.ascontiguousarray(m, dtype=np.uint8).reshape(k * k)
    inv = np.empty(k * k, dtype=np.uint8)
    st = lib().orc_matrix_inverse(_p(m), _p(inv), k, poly)
    return None if st else inv.reshape(k, k)


def blob_encode(blob, coeffs, poly=POLY, marker=MARKER, nthreads=1):
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    n = -(-blob.size // CS)
    coeffs = np.ascontiguousarray(coeffs, dtype=np.uint8)
    out = np.empty((n * N, F), dtype=np.uint8)
    st = lib().orc_blob_encode(_p(blob), blob.size, _p(coeffs), _p(out), poly, marker, nthreads)
    assert st == OK
    return out


def blob_repair(coded, cand, blob_len, poly=POLY, marker=MARKER, nthreads=1):
    coded = np.ascontiguousarray(coded, dtype=np.uint8)
    n = coded.shape[0] // N
    cand = np.ascontiguousarray(cand, dtype=np.uint8)
    out = np.zeros(blob_len, dtype=np.uint8)
    status = np.empty(n, dtype=np.int32)
    lib().orc_blob_repair(_p(coded), n, _p(cand), blob_len, _p(out), _p(status), poly, marker, nthreads)
    return out, status


def fast_supported():
    """the blocked GFNI / AVX-512 codec (rlnc_cpu_fast.c) runs on this CPU"""
    return bool(lib().orc_fast_supported())


def fast_blob_encode(blob, coeffs, poly=POLY, marker=MARKER, nthreads=1):
    """blob_encode's bytes from the column-blocked GFNI codec (cpu_baseline's headline variant)"""
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    n = -(-blob.size // CS)
    coeffs = np.ascontiguousarray(coeffs, dtype=np.uint8)
    out = np.empty((n * N, F), dtype=np.uint8)
    st = lib().orc_fast_blob_encode(_p(blob), blob.size, _p(coeffs), _p(out), poly, marker, nthreads)
    if st != OK:
        raise RuntimeError("orc_fast_blob_encode status %d" % st)
    return out


def fast_blob_repair(coded, cand, blob_len, poly=POLY, marker=MARKER, nthreads=1):
    """blob_repair's output and statuses from coefficient-only rank + inverse + one blocked GFNI pass"""
    coded = np.ascontiguousarray(coded, dtype=np.uint8)
    n = coded.shape[0] // N
    cand = np.ascontiguousarray(cand, dtype=np.uint8)
    out = np.zeros(blob_len, dtype=np.uint8)
    status = np.empty(n, dtype=np.int32)
    st = lib().orc_fast_blob_repair(_p(coded), n, _p(cand), blob_len, _p(out), _p(status), poly, marker, nthreads)
    if st != OK:
        raise RuntimeError("orc_fast_blob_repair status %d" % st)
    return out, status


# ---- commitment layer (blake3_oracle.c) ----------------------------------------------------------
def blake3(data):
    data = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8) if isinstance(data, (bytes, bytearray)) else data,
                                dtype=np.uint8)
    out = np.empty(32, np.uint8)
    lib().orc_blake3(_p(data) if data.size else None, data.size, _p(out))
    return out.tobytes()


def chunk_digest(chunkset_id, chunk_id, data):
    """chunk.rs:40-46"""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    out = np.empty(32, np.uint8)
    lib().orc_chunk_digest(chunkset_id, chunk_id, _p(data), data.size, _p(out))
    return out.tobytes()


def chunk_digest_rows(rows, first_row):
    """chunk.rs:40-46 for every row of a (m, F) array of coded rows, rows first_row .. first_row + m - 1
    of the blob (chunk id = chunkset_id * 16 + i, chunkset.rs:47) -> (m, 32) digests"""
    rows = np.ascontiguousarray(rows, dtype=np.uint8)
    m = rows.shape[0]
    out = np.empty((m, 32), np.uint8)
    lib().orc_chunk_digest_rows(_p(rows), m, rows.shape[1] if rows.ndim == 2 else F, first_row, _p(out))
    return out


def merkle(leaves):
    """merkle_tree.rs:23-116 -> (root, proofs[n][depth] of 32-byte hashes)"""
    lv = np.ascontiguousarray(np.frombuffer(b"".join(leaves), np.uint8))
    n = len(leaves)
    depth = max(0, (n - 1).bit_length())
    root = np.empty(32, np.uint8)
    proofs = np.empty(max(1, n * depth * 32), np.uint8)
    d = lib().orc_merkle(_p(lv), n, _p(root), _p(proofs))
    assert d == depth
    pr = [[proofs[(i * depth + k) * 32:(i * depth + k + 1) * 32].tobytes() for k in range(depth)] for i in range(n)]
    return root.tobytes(), pr


def merkle_verify(leaf_index, leaf, proof, root):
    """merkle_tree.rs:131-146"""
    pf = np.ascontiguousarray(np.frombuffer(b"".join(proof) or b"\0", np.uint8))
    lf = np.frombuffer(leaf, np.uint8).copy()
    rt = np.frombuffer(root, np.uint8).copy()
    return bool(lib().orc_merkle_verify(leaf_index, _p(lf), _p(pf), len(proof), _p(rt)))

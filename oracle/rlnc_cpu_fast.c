/*
 * rlnc_cpu_fast.c — the strongest CPU restatement of the chunkset codec, for bench.py's
 * cpu_baseline leg ("kind": "port"). TEST INFRASTRUCTURE ONLY, like the rest of oracle/: never
 * linked into or called by the product library.
 *
 * Same bytes as the scalar restatement in rlnc_oracle.c (tests/test_oracle.py checks every variant
 * against it), organised the way a tuned CPU erasure coder is:
 *   - column-blocked: one pass over the chunkset; every 64-byte column block loads the 10 pieces
 *     once and produces all 16 coded payloads (rlnc's Encoder::code re-streams the 10 pieces once
 *     per coded piece, chunkset.rs:45-52);
 *   - multiply by a constant with one GFNI vgf2p8affineqb per 64 bytes: multiplication by c in
 *     GF(2^8) is GF(2)-linear, i.e. an 8x8 bit matrix, for any field polynomial (the GF2P8MULB
 *     instruction is fixed to 0x11B, the affine form is not);
 *   - repair as rlnc's outcome, computed directly: the incremental rank test over the candidates'
 *     coding vectors in arrival order (chunkset.rs:173-184), the inverse of the accepted 10x10
 *     block, then one blocked pass piece_i = sum_k inv[i][k] * payload_k over the accepted rows,
 *     cut at the last boundary marker as get_decoded_data (chunkset.rs:200-208);
 *   - chunkset-parallel over POSIX threads, as Blob::new's rayon loop (blob.rs:256-264).
 */
#include <immintrin.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

#include "rlnc_oracle.h"

#define BLK 64u

int orc_fast_supported(void) {
    return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
           __builtin_cpu_supports("gfni");
}

/* the 8x8 GF(2) matrix of x -> c*x in vgf2p8affineqb's layout: result bit i = parity(A.byte[7-i] & x) */
uint64_t orc_gf_affine_matrix(uint8_t c, uint32_t poly) {
    uint8_t col[8];
    for (int k = 0; k < 8; k++) col[k] = orc_gf256_mul(c, (uint8_t)(1u << k), poly);
    uint64_t a = 0;
    for (int i = 0; i < 8; i++) {
        uint8_t row = 0;
        for (int k = 0; k < 8; k++) row |= (uint8_t)(((col[k] >> i) & 1u) << k);
        a |= (uint64_t)row << (8 * (7 - i));
    }
    return a;
}

/* out[j][0..64) = sum_i A[j][i] * in[i][0..64), NOUT outputs of 10 inputs */
/* A: the matrices pre-broadcast to 64 bytes (memory operands of the affine instructions, L1-resident) */
typedef struct {
    uint64_t q[8];
} __attribute__((aligned(64))) mat512;

static void broadcast_matrices(mat512 *A, const uint8_t *c, unsigned count, uint32_t poly) {
    for (unsigned t = 0; t < count; t++) {
        const uint64_t a = orc_gf_affine_matrix(c[t], poly);
        for (int w = 0; w < 8; w++) A[t].q[w] = a;
    }
}

__attribute__((target("avx512f,avx512bw,gfni"))) static inline void combine64(const uint8_t *const in[ORC_K],
                                                                              uint8_t *const out[], int nout,
                                                                              const mat512 *A) {
    __m512i x[ORC_K];
    for (unsigned i = 0; i < ORC_K; i++) x[i] = _mm512_loadu_si512((const void *)in[i]);
    for (int j = 0; j < nout; j++) {
        const mat512 *a = A + j * ORC_K;
#define MAT(i) _mm512_load_si512((const void *)&a[i])
        __m512i acc = _mm512_gf2p8affine_epi64_epi8(x[0], MAT(0), 0);
        for (unsigned i = 1; i + 1 < ORC_K; i += 2) {
            const __m512i p = _mm512_gf2p8affine_epi64_epi8(x[i], MAT(i), 0);
            const __m512i q = _mm512_gf2p8affine_epi64_epi8(x[i + 1], MAT(i + 1), 0);
            acc = _mm512_ternarylogic_epi64(acc, p, q, 0x96);
        }
        acc = _mm512_xor_si512(acc, _mm512_gf2p8affine_epi64_epi8(x[ORC_K - 1], MAT(ORC_K - 1), 0));
#undef MAT
        _mm512_storeu_si512((void *)out[j], acc);
    }
}

/* padded piece byte (rlnc Encoder::new, chunkset.rs:43): data (zero past `have`), marker at CS, zeros */
static inline uint8_t padded_byte(const uint8_t *data, size_t have, uint8_t marker, size_t p) {
    return p < have ? data[p] : (p == ORC_CS ? marker : 0u);
}

/* ChunkSet::new's RLNC part for one chunkset: `have` real bytes (blob.rs:252-254 pads the rest) */
static void fast_encode_chunkset(const uint8_t *data, size_t have, const uint8_t *cv, uint8_t *out, const mat512 *A,
                                 uint8_t marker) {
    for (unsigned j = 0; j < ORC_N; j++) memcpy(out + (size_t)j * ORC_F, cv + j * ORC_K, ORC_K);
    uint8_t tin[ORC_K][BLK], tout[ORC_N][BLK];
    const uint8_t *in[ORC_K];
    uint8_t *o[ORC_N];
    for (size_t c = 0; c < ORC_L; c += BLK) {
        const int direct_in = (ORC_K - 1) * (size_t)ORC_L + c + BLK <= have;
        const int direct_out = c + BLK <= ORC_L;
        for (unsigned i = 0; i < ORC_K; i++) {
            if (direct_in) {
                in[i] = data + (size_t)i * ORC_L + c;
            } else {
                for (unsigned b = 0; b < BLK; b++)
                    tin[i][b] = padded_byte(data, have, marker, (size_t)i * ORC_L + c + b);
                in[i] = tin[i];
            }
        }
        for (unsigned j = 0; j < ORC_N; j++) o[j] = direct_out ? out + (size_t)j * ORC_F + ORC_K + c : tout[j];
        combine64(in, o, ORC_N, A);
        if (!direct_out)
            for (unsigned j = 0; j < ORC_N; j++) memcpy(out + (size_t)j * ORC_F + ORC_K + c, tout[j], ORC_L - c);
    }
}

/* the blocked pass piece_i = sum_k inv[i][k] * payload_k over the accepted rows: decoded bytes below
 * `keep` into out, the 10 bytes past the chunkset ([CS, CS + 10): marker || zeros when intact) into tail */
static void fast_decode_pass(const uint8_t *coded, const uint8_t *sel, const mat512 *A, uint8_t *out, size_t keep,
                             uint8_t tail[ORC_K]) {
    const uint8_t *in[ORC_K];
    uint8_t *o[ORC_K];
    uint8_t tin[ORC_K][BLK], tout[ORC_K][BLK];
    for (size_t c = 0; c < ORC_L; c += BLK) {
        const int full = c + BLK <= ORC_L;
        for (unsigned k = 0; k < ORC_K; k++) {
            const uint8_t *row = coded + (size_t)sel[k] * ORC_F + ORC_K + c;
            if (full) {
                in[k] = row;
            } else {
                memset(tin[k], 0, BLK);
                memcpy(tin[k], row, ORC_L - c);
                in[k] = tin[k];
            }
        }
        const int direct = (ORC_K - 1) * (size_t)ORC_L + c + BLK <= keep && full;
        for (unsigned i = 0; i < ORC_K; i++) o[i] = direct ? out + (size_t)i * ORC_L + c : tout[i];
        combine64(in, o, ORC_K, A);
        if (direct) continue;
        for (unsigned i = 0; i < ORC_K; i++)
            for (size_t b = 0; b < BLK && c + b < ORC_L; b++) {
                const size_t p = (size_t)i * ORC_L + c + b;
                if (p < keep)
                    out[p] = tout[i][b];
                else if (p >= ORC_CS)
                    tail[p - ORC_CS] = tout[i][b];
            }
    }
}

/* RepairingChunkSet add_chunk_unvalidated x candidates + repair (chunkset.rs:173-208), keep = real size.
 * get_decoded_data's cut at the last boundary marker as orc_decoder_get_decoded_data: *cut = decoded
 * length; out holds its first min(cut, keep) bytes and zeros up to keep (the blob paths' layout). */
static int fast_repair_chunkset(const uint8_t *coded, const uint8_t *cand, uint8_t *out, size_t keep, uint32_t poly,
                                uint8_t marker, size_t *cut) {
    uint8_t basis[ORC_K * ORC_K], piv[ORC_K], sel[ORC_K], m[ORC_K * ORC_K], inv[ORC_K * ORC_K], tail[ORC_K];
    size_t rank = 0;
    for (unsigned a = 0; a < ORC_N && rank < ORC_K; a++) {
        const uint8_t r = cand[a];
        if (r >= ORC_N) break;
        const size_t before = rank;
        if (orc_rank_push(basis, piv, &rank, coded + (size_t)r * ORC_F, ORC_K, poly) && rank > before)
            sel[before] = r;
    }
    if (rank < ORC_K) return ORC_ERR_NOT_ALL_PIECES_RECEIVED;
    for (unsigned k = 0; k < ORC_K; k++) memcpy(m + k * ORC_K, coded + (size_t)sel[k] * ORC_F, ORC_K);
    if (orc_matrix_inverse(m, inv, ORC_K, poly)) return ORC_ERR_NOT_ALL_PIECES_RECEIVED;
    mat512 A[ORC_K * ORC_K];
    broadcast_matrices(A, inv, ORC_K * ORC_K, poly);
    fast_decode_pass(coded, sel, A, out, keep, tail);
    size_t len = 0;
    for (unsigned j = ORC_K; j-- > 0;)
        if (tail[j] == marker) {
            len = ORC_CS + j;
            break;
        }
    if (!len) { /* no marker past the chunkset (corrupted rows only): search the decoded chunkset */
        uint8_t *full = (uint8_t *)malloc(ORC_CS);
        if (!full) return ORC_ERR_ARGS;
        fast_decode_pass(coded, sel, A, full, ORC_CS, tail);
        size_t p = ORC_CS;
        while (p > 0 && full[p - 1] != marker) p--;
        free(full);
        if (p == 0) { /* an error gets no data (as the blob drivers leave it) */
            memset(out, 0, keep);
            return ORC_ERR_INVALID_DECODED_DATA;
        }
        len = p - 1;
    }
    if (len < keep) memset(out + len, 0, keep - len);
    if (cut) *cut = len;
    return ORC_OK;
}

struct fast_job {
    const uint8_t *blob, *coeffs, *coded, *cand;
    uint8_t *out;
    int32_t *status;
    size_t blob_len, n;
    uint32_t poly;
    uint8_t marker;
    atomic_size_t next;
};

static void *fast_encode_worker(void *arg) {
    struct fast_job *j = (struct fast_job *)arg;
    mat512 A[ORC_N * ORC_K];
    for (;;) {
        const size_t c = atomic_fetch_add(&j->next, 1);
        if (c >= j->n) break;
        const uint8_t *cv = j->coeffs + c * ORC_N * ORC_K;
        broadcast_matrices(A, cv, ORC_N * ORC_K, j->poly);
        const size_t off = c * (size_t)ORC_CS;
        const size_t have = j->blob_len - off < ORC_CS ? j->blob_len - off : ORC_CS;
        fast_encode_chunkset(j->blob + off, have, cv, j->out + c * (size_t)ORC_N * ORC_F, A, j->marker);
    }
    return NULL;
}

static void *fast_repair_worker(void *arg) {
    struct fast_job *j = (struct fast_job *)arg;
    for (;;) {
        const size_t c = atomic_fetch_add(&j->next, 1);
        if (c >= j->n) break;
        const size_t off = c * (size_t)ORC_CS;
        const size_t keep = j->blob_len - off < ORC_CS ? j->blob_len - off : ORC_CS;
        j->status[c] = fast_repair_chunkset(j->coded + c * (size_t)ORC_N * ORC_F, j->cand + c * ORC_N,
                                            j->out + off, keep, j->poly, j->marker, NULL);
    }
    return NULL;
}

static void fast_pool(struct fast_job *j, void *(*fn)(void *), int nthreads) {
    if (nthreads < 1) nthreads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, fn, j);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
}

/* orc_blob_encode / orc_blob_repair (rlnc_oracle_blob.c) with the blocked GFNI codec; -1 without GFNI */
int orc_fast_blob_encode(const uint8_t *blob, size_t blob_len, const uint8_t *coeffs, uint8_t *out, uint32_t poly,
                         uint8_t marker, int nthreads) {
    if (!orc_fast_supported()) return -1;
    if (blob_len == 0) return ORC_ERR_ARGS;
    struct fast_job j;
    memset(&j, 0, sizeof(j));
    j.blob = blob;
    j.blob_len = blob_len;
    j.n = (blob_len + ORC_CS - 1) / ORC_CS;
    j.coeffs = coeffs;
    j.out = out;
    j.poly = poly;
    j.marker = marker;
    atomic_init(&j.next, 0);
    fast_pool(&j, fast_encode_worker, nthreads);
    return ORC_OK;
}

int orc_fast_blob_repair(const uint8_t *coded, size_t n_chunksets, const uint8_t *cand, size_t blob_len, uint8_t *out,
                         int32_t *status, uint32_t poly, uint8_t marker, int nthreads) {
    if (!orc_fast_supported()) return -1;
    struct fast_job j;
    memset(&j, 0, sizeof(j));
    j.coded = coded;
    j.n = n_chunksets;
    j.cand = cand;
    j.blob_len = blob_len;
    j.out = out;
    j.status = status;
    j.poly = poly;
    j.marker = marker;
    atomic_init(&j.next, 0);
    fast_pool(&j, fast_repair_worker, nthreads);
    return ORC_OK;
}

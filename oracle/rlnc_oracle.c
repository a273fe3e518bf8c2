/*
 * rlnc_oracle.c — plain-C restatement of decds' RLNC chunkset path. TEST INFRASTRUCTURE ONLY
 * (see rlnc_oracle.h for scope, the reference lines each function follows, and parity status).
 */
#include "rlnc_oracle.h"

#include <immintrin.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- GF(2^8) ------------------ */
/* rlnc 0.4.0 Gf256::mul [recalled]: polynomial multiplication reduced by the field polynomial.
 * Restated as the textbook shift-and-add ("Russian peasant") loop. */
uint8_t orc_gf256_mul(uint8_t a, uint8_t b, uint32_t poly) {
    uint32_t acc = 0, x = a;
    for (int i = 0; i < 8; i++) {
        if (b & (1u << i)) acc ^= x;
        x <<= 1;
        if (x & 0x100u) x ^= poly;
    }
    return (uint8_t)acc;
}

/* multiplicative inverse a^-1 = a^254 (a != 0); 0 maps to 0 (never used as a pivot) */
uint8_t orc_gf256_inv(uint8_t a, uint32_t poly) {
    uint8_t r = 1, base = a;
    unsigned e = 254;
    while (e) {
        if (e & 1u) r = orc_gf256_mul(r, base, poly);
        base = orc_gf256_mul(base, base, poly);
        e >>= 1;
    }
    return a ? r : 0;
}

void orc_gf256_mul_table(uint32_t poly, uint8_t *out) {
    for (unsigned a = 0; a < 256; a++)
        for (unsigned b = 0; b < 256; b++) out[a * 256 + b] = orc_gf256_mul((uint8_t)a, (uint8_t)b, poly);
}

/* ---------------------------------------------------------------- synthetic data ----------- */
uint64_t orc_splitmix64_word(uint64_t seed, uint64_t w) {
    uint64_t z = seed + (w + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void orc_fill_random(uint64_t seed, uint64_t byte_offset, uint8_t *out, size_t len) {
    size_t i = 0;
    for (; i < len && ((byte_offset + i) & 7); i++) {
        uint64_t p = byte_offset + i;
        out[i] = (uint8_t)(orc_splitmix64_word(seed, p >> 3) >> (8 * (p & 7)));
    }
    for (; i + 8 <= len; i += 8) {
        uint64_t z = orc_splitmix64_word(seed, (byte_offset + i) >> 3);
        for (int b = 0; b < 8; b++) out[i + b] = (uint8_t)(z >> (8 * b));
    }
    for (; i < len; i++) {
        uint64_t p = byte_offset + i;
        out[i] = (uint8_t)(orc_splitmix64_word(seed, p >> 3) >> (8 * (p & 7)));
    }
}

/* ---------------------------------------------------------------- encoder ------------------ */
/* chunkset.rs:117 pins L = ceil((len + 1) / k): one marker byte, then zero padding */
size_t orc_piece_len(size_t data_len, size_t k) { return (data_len + 1 + k - 1) / k; }

/* rlnc Encoder::new(data, k) [recalled]: data || marker || zeros, k*L bytes, pieces = L-byte rows */
int orc_encoder_pad(const uint8_t *data, size_t len, size_t k, uint8_t marker, uint8_t *out) {
    if (len == 0 || k == 0) return ORC_ERR_ARGS;
    size_t L = orc_piece_len(len, k);
    memcpy(out, data, len);
    out[len] = marker;
    memset(out + len + 1, 0, k * L - len - 1);
    return ORC_OK;
}

/* Row kernels. Default: the scalar table-driven form of rlnc 0.4.0's inner loop [recalled] — one
 * 256-entry product row per constant, one lookup per byte. orc_set_simd(1) switches to the AVX2
 * nibble-table form (c*x = T_lo[x & 15] ^ T_hi[x >> 4], 32 bytes per vpshufb pair) where the CPU has
 * it: same products, so the same bytes; it only makes the CPU baseline a stronger one (bench.py
 * reports both). */
static int g_simd = 0;

int orc_set_simd(int on) {
    g_simd = on && __builtin_cpu_supports("avx2");
    return g_simd;
}

__attribute__((target("avx2"))) static void mul_row_avx2(uint8_t *dst, const uint8_t *src, size_t len,
                                                         uint8_t c, uint32_t poly, int acc) {
    uint8_t lo[16], hi[16];
    for (unsigned x = 0; x < 16; x++) {
        lo[x] = orc_gf256_mul(c, (uint8_t)x, poly);
        hi[x] = orc_gf256_mul(c, (uint8_t)(x << 4), poly);
    }
    const __m256i tl = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)lo));
    const __m256i th = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)hi));
    const __m256i m = _mm256_set1_epi8(0x0F);
    size_t j = 0;
    for (; j + 32 <= len; j += 32) {
        const __m256i v = _mm256_loadu_si256((const __m256i *)(src + j));
        __m256i r = _mm256_xor_si256(_mm256_shuffle_epi8(tl, _mm256_and_si256(v, m)),
                                     _mm256_shuffle_epi8(th, _mm256_and_si256(_mm256_srli_epi16(v, 4), m)));
        if (acc) r = _mm256_xor_si256(r, _mm256_loadu_si256((const __m256i *)(dst + j)));
        _mm256_storeu_si256((__m256i *)(dst + j), r);
    }
    for (; j < len; j++) {
        const uint8_t y = (uint8_t)(lo[src[j] & 15] ^ hi[src[j] >> 4]);
        dst[j] = acc ? (uint8_t)(dst[j] ^ y) : y;
    }
}

/* multiply-accumulate a row by a constant */
static void mul_acc_row(uint8_t *dst, const uint8_t *src, size_t len, uint8_t c, uint32_t poly) {
    if (c == 0) return;
    if (g_simd) {
        mul_row_avx2(dst, src, len, c, poly, 1);
        return;
    }
    uint8_t t[256];
    for (unsigned x = 0; x < 256; x++) t[x] = orc_gf256_mul(c, (uint8_t)x, poly);
    for (size_t j = 0; j < len; j++) dst[j] ^= t[src[j]];
}

static void mul_row(uint8_t *row, size_t len, uint8_t c, uint32_t poly) {
    if (g_simd) {
        mul_row_avx2(row, row, len, c, poly, 0);
        return;
    }
    uint8_t t[256];
    for (unsigned x = 0; x < 256; x++) t[x] = orc_gf256_mul(c, (uint8_t)x, poly);
    for (size_t j = 0; j < len; j++) row[j] = t[row[j]];
}

/* rlnc Encoder::code(rng) with the coding vector made explicit: cv || sum_i cv[i]*piece_i */
void orc_code_with_coding_vector(const uint8_t *padded, size_t piece_len, size_t k,
                                 const uint8_t *cv, uint8_t *out, uint32_t poly) {
    memcpy(out, cv, k);
    uint8_t *payload = out + k;
    memset(payload, 0, piece_len);
    for (size_t i = 0; i < k; i++) mul_acc_row(payload, padded + i * piece_len, piece_len, cv[i], poly);
}

struct enc_job {
    const uint8_t *padded;
    const uint8_t *coeffs;
    uint8_t *out;
    uint32_t poly;
    unsigned first, last;
};

static void *enc_worker(void *arg) {
    struct enc_job *j = (struct enc_job *)arg;
    for (unsigned p = j->first; p < j->last; p++)
        orc_code_with_coding_vector(j->padded, ORC_L, ORC_K, j->coeffs + p * ORC_K,
                                    j->out + (size_t)p * ORC_F, j->poly);
    return NULL;
}

/* chunkset.rs:37-52: size check (38-40 -> InvalidChunksetSize), Encoder::new (43), 16 x code() (45-52) */
int orc_chunkset_encode(const uint8_t *data, size_t len, const uint8_t *coeffs, uint8_t *out,
                        uint32_t poly, uint8_t marker, int nthreads) {
    if (len != ORC_CS) return ORC_ERR_INVALID_CHUNKSET_SIZE;
    uint8_t *padded = (uint8_t *)malloc((size_t)ORC_K * ORC_L);
    if (!padded) return ORC_ERR_ARGS;
    orc_encoder_pad(data, len, ORC_K, marker, padded);
    if (nthreads <= 1) {
        struct enc_job j = {padded, coeffs, out, poly, 0, ORC_N};
        enc_worker(&j);
    } else {
        if (nthreads > (int)ORC_N) nthreads = ORC_N;
        pthread_t th[ORC_N];
        struct enc_job jobs[ORC_N];
        for (int t = 0; t < nthreads; t++) {
            jobs[t] = (struct enc_job){padded, coeffs, out, poly, (unsigned)(t * ORC_N / nthreads),
                                       (unsigned)((t + 1) * ORC_N / nthreads)};
            pthread_create(&th[t], NULL, enc_worker, &jobs[t]);
        }
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    }
    free(padded);
    return ORC_OK;
}

/* ---------------------------------------------------------------- decoder ------------------ */
struct orc_decoder {
    size_t piece_len, k, full_len, rank;
    uint32_t poly;
    uint8_t marker;
    uint8_t *rows;    /* rank rows of full_len bytes, sorted by pivot, RREF on the coefficient part */
    size_t *pivot;    /* pivot column of each row */
    uint8_t *scratch; /* incoming row */
};

orc_decoder *orc_decoder_new(size_t piece_len, size_t k, uint32_t poly, uint8_t marker) {
    if (piece_len == 0 || k == 0) return NULL;
    orc_decoder *d = (orc_decoder *)calloc(1, sizeof(*d));
    d->piece_len = piece_len;
    d->k = k;
    d->full_len = k + piece_len;
    d->poly = poly;
    d->marker = marker;
    d->rows = (uint8_t *)malloc(k * d->full_len);
    d->pivot = (size_t *)calloc(k, sizeof(size_t));
    d->scratch = (uint8_t *)malloc(d->full_len);
    return d;
}

void orc_decoder_free(orc_decoder *d) {
    if (!d) return;
    free(d->rows);
    free(d->pivot);
    free(d->scratch);
    free(d);
}

int orc_decoder_is_decoded(const orc_decoder *d) { return d->rank == d->k; }
size_t orc_decoder_rank(const orc_decoder *d) { return d->rank; }

/* rlnc Decoder::decode [recalled]: append the row, re-reduce to RREF, drop a row that reduced to
 * zero and report it as not useful. Incremental elimination against an RREF basis yields the same
 * (unique) RREF as a full re-elimination. chunkset.rs:181-183 maps any error to ChunkDecodingFailed. */
int orc_decoder_decode(orc_decoder *d, const uint8_t *piece, size_t len) {
    if (d->rank == d->k) return ORC_ERR_RECEIVED_ALL_PIECES;
    if (len != d->full_len) return ORC_ERR_INVALID_PIECE_LENGTH;
    uint8_t *r = d->scratch;
    memcpy(r, piece, len);
    for (size_t e = 0; e < d->rank; e++) {
        uint8_t f = r[d->pivot[e]];
        if (f) mul_acc_row(r, d->rows + e * d->full_len, d->full_len, f, d->poly);
    }
    size_t p = d->k;
    for (size_t c = 0; c < d->k; c++)
        if (r[c]) { p = c; break; }
    if (p == d->k) return ORC_ERR_PIECE_NOT_USEFUL;
    mul_row(r, d->full_len, orc_gf256_inv(r[p], d->poly), d->poly);
    for (size_t e = 0; e < d->rank; e++) {
        uint8_t *row = d->rows + e * d->full_len;
        uint8_t f = row[p];
        if (f) mul_acc_row(row, r, d->full_len, f, d->poly);
    }
    size_t pos = d->rank;
    while (pos > 0 && d->pivot[pos - 1] > p) {
        memcpy(d->rows + pos * d->full_len, d->rows + (pos - 1) * d->full_len, d->full_len);
        d->pivot[pos] = d->pivot[pos - 1];
        pos--;
    }
    memcpy(d->rows + pos * d->full_len, r, d->full_len);
    d->pivot[pos] = p;
    d->rank++;
    return ORC_OK;
}

/* rlnc Decoder::get_decoded_data [recalled]: rows are the identity-reduced pieces in order; the
 * payloads are concatenated and cut at the last boundary marker. chunkset.rs:200-208. */
int orc_decoder_get_decoded_data(const orc_decoder *d, uint8_t *out, size_t cap, size_t *out_len) {
    if (d->rank != d->k) return ORC_ERR_NOT_ALL_PIECES_RECEIVED;
    size_t total = d->k * d->piece_len;
    size_t idx = total;
    for (size_t r = d->k; r-- > 0 && idx == total;) {
        const uint8_t *pl = d->rows + r * d->full_len + d->k;
        for (size_t j = d->piece_len; j-- > 0;)
            if (pl[j] == d->marker) { idx = r * d->piece_len + j; break; }
    }
    if (idx == total) return ORC_ERR_INVALID_DECODED_DATA;
    *out_len = idx;
    size_t w = 0;
    for (size_t r = 0; r < d->k && w < idx; r++) {
        size_t n = d->piece_len;
        if (w + n > idx) n = idx - w;
        if (out && w < cap) memcpy(out + w, d->rows + r * d->full_len + d->k, (w + n > cap ? cap - w : n));
        w += n;
    }
    return ORC_OK;
}

/* ---------------------------------------------------------------- coefficient-only helpers -- */
int orc_rank_push(uint8_t *basis, uint8_t *pivots, size_t *rank, const uint8_t *coeff, size_t k,
                  uint32_t poly) {
    uint8_t r[64];
    if (k > 64 || *rank >= k) return 0;
    memcpy(r, coeff, k);
    for (size_t e = 0; e < *rank; e++) {
        uint8_t f = r[pivots[e]];
        if (f)
            for (size_t c = 0; c < k; c++) r[c] ^= orc_gf256_mul(f, basis[e * k + c], poly);
    }
    size_t p = k;
    for (size_t c = 0; c < k; c++)
        if (r[c]) { p = c; break; }
    if (p == k) return 0;
    uint8_t inv = orc_gf256_inv(r[p], poly);
    for (size_t c = 0; c < k; c++) r[c] = orc_gf256_mul(r[c], inv, poly);
    for (size_t e = 0; e < *rank; e++) {
        uint8_t f = basis[e * k + p];
        if (f)
            for (size_t c = 0; c < k; c++) basis[e * k + c] ^= orc_gf256_mul(f, r[c], poly);
    }
    memcpy(basis + *rank * k, r, k);
    pivots[*rank] = (uint8_t)p;
    (*rank)++;
    return 1;
}

int orc_matrix_inverse(const uint8_t *m, uint8_t *inv, size_t k, uint32_t poly) {
    uint8_t a[64 * 128];
    if (k > 64) return -1;
    size_t w = 2 * k;
    for (size_t i = 0; i < k; i++)
        for (size_t j = 0; j < w; j++) a[i * w + j] = j < k ? m[i * k + j] : (uint8_t)(j - k == i);
    for (size_t c = 0; c < k; c++) {
        size_t p = c;
        while (p < k && !a[p * w + c]) p++;
        if (p == k) return -1;
        if (p != c)
            for (size_t j = 0; j < w; j++) {
                uint8_t t = a[p * w + j];
                a[p * w + j] = a[c * w + j];
                a[c * w + j] = t;
            }
        uint8_t iv = orc_gf256_inv(a[c * w + c], poly);
        for (size_t j = 0; j < w; j++) a[c * w + j] = orc_gf256_mul(a[c * w + j], iv, poly);
        for (size_t i = 0; i < k; i++) {
            uint8_t f = a[i * w + c];
            if (i == c || !f) continue;
            for (size_t j = 0; j < w; j++) a[i * w + j] ^= orc_gf256_mul(f, a[c * w + j], poly);
        }
    }
    for (size_t i = 0; i < k; i++)
        for (size_t j = 0; j < k; j++) inv[i * k + j] = a[i * w + k + j];
    return 0;
}

// blake3_host.cpp — host BLAKE3 over many chunks at once with AVX2 (8 lanes of 32 bits), the
// host-side hashing of the commitment layer: the whole-blob digest of Blob::new (blob.rs:249), the
// chunk digest RepairingBlob::add_chunk / RepairingChunkSet::add_chunk validate with (chunk.rs:40-46,
// 88-110) and the repaired blob's check (handle_repair.rs:129-151). The reference's blake3 crate
// (=1.8.2, not vendored) hashes independent chunks in SIMD lanes; this restates that idea from the
// BLAKE3 specification: lane j compresses chunk j of a group of 16 (AVX-512F) or 8 (AVX2), message
// words transposed into word-major vectors, and the parent levels of a power-of-two subtree are
// compressed 16 / 8 at a time the same way (a parent's 64-byte message is two adjacent 32-byte
// chaining values). Without AVX2 the scalar compression in blake3_impl.h is used.
#include <immintrin.h>

#include <cstring>

#include "blake3_host.h"
#include "blake3_impl.h"

namespace decds {
namespace b3h {

namespace {

#define B3H_AVX2 __attribute__((target("avx2")))

B3H_AVX2 inline __m256i rotr16(__m256i x) {
    const __m256i m = _mm256_setr_epi8(2, 3, 0, 1, 6, 7, 4, 5, 10, 11, 8, 9, 14, 15, 12, 13, 2, 3, 0, 1, 6, 7, 4, 5, 10,
                                       11, 8, 9, 14, 15, 12, 13);
    return _mm256_shuffle_epi8(x, m);
}
B3H_AVX2 inline __m256i rotr8(__m256i x) {
    const __m256i m = _mm256_setr_epi8(1, 2, 3, 0, 5, 6, 7, 4, 9, 10, 11, 8, 13, 14, 15, 12, 1, 2, 3, 0, 5, 6, 7, 4, 9,
                                       10, 11, 8, 13, 14, 15, 12);
    return _mm256_shuffle_epi8(x, m);
}
B3H_AVX2 inline __m256i rotr12(__m256i x) { return _mm256_or_si256(_mm256_srli_epi32(x, 12), _mm256_slli_epi32(x, 20)); }
B3H_AVX2 inline __m256i rotr7(__m256i x) { return _mm256_or_si256(_mm256_srli_epi32(x, 7), _mm256_slli_epi32(x, 25)); }

B3H_AVX2 inline void g(__m256i *v, int a, int b, int c, int d, __m256i x, __m256i y) {
    v[a] = _mm256_add_epi32(_mm256_add_epi32(v[a], v[b]), x);
    v[d] = rotr16(_mm256_xor_si256(v[d], v[a]));
    v[c] = _mm256_add_epi32(v[c], v[d]);
    v[b] = rotr12(_mm256_xor_si256(v[b], v[c]));
    v[a] = _mm256_add_epi32(_mm256_add_epi32(v[a], v[b]), y);
    v[d] = rotr8(_mm256_xor_si256(v[d], v[a]));
    v[c] = _mm256_add_epi32(v[c], v[d]);
    v[b] = rotr7(_mm256_xor_si256(v[b], v[c]));
}

// 8 compressions, lane j: cv[.][j], message m[.][j]; cv <- first 8 output words
B3H_AVX2 inline void compress8(__m256i cv[8], const __m256i m[16], __m256i ctr_lo, __m256i ctr_hi, uint32_t block_len,
                               uint32_t flags) {
    __m256i v[16] = {cv[0],
                     cv[1],
                     cv[2],
                     cv[3],
                     cv[4],
                     cv[5],
                     cv[6],
                     cv[7],
                     _mm256_set1_epi32((int)b3::K3.iv[0]),
                     _mm256_set1_epi32((int)b3::K3.iv[1]),
                     _mm256_set1_epi32((int)b3::K3.iv[2]),
                     _mm256_set1_epi32((int)b3::K3.iv[3]),
                     ctr_lo,
                     ctr_hi,
                     _mm256_set1_epi32((int)block_len),
                     _mm256_set1_epi32((int)flags)};
    for (int r = 0; r < 7; r++) {
        const uint8_t *q = b3::K3.sched[r];
        g(v, 0, 4, 8, 12, m[q[0]], m[q[1]]);
        g(v, 1, 5, 9, 13, m[q[2]], m[q[3]]);
        g(v, 2, 6, 10, 14, m[q[4]], m[q[5]]);
        g(v, 3, 7, 11, 15, m[q[6]], m[q[7]]);
        g(v, 0, 5, 10, 15, m[q[8]], m[q[9]]);
        g(v, 1, 6, 11, 12, m[q[10]], m[q[11]]);
        g(v, 2, 7, 8, 13, m[q[12]], m[q[13]]);
        g(v, 3, 4, 9, 14, m[q[14]], m[q[15]]);
    }
    for (int i = 0; i < 8; i++) cv[i] = _mm256_xor_si256(v[i], v[i + 8]);
}

// 8x8 transpose of 32-bit words: in[j] = 8 words of row j -> out[w] = word w of rows 0..7
B3H_AVX2 inline void transpose8(const __m256i in[8], __m256i out[8]) {
    const __m256i t0 = _mm256_unpacklo_epi32(in[0], in[1]), t1 = _mm256_unpackhi_epi32(in[0], in[1]);
    const __m256i t2 = _mm256_unpacklo_epi32(in[2], in[3]), t3 = _mm256_unpackhi_epi32(in[2], in[3]);
    const __m256i t4 = _mm256_unpacklo_epi32(in[4], in[5]), t5 = _mm256_unpackhi_epi32(in[4], in[5]);
    const __m256i t6 = _mm256_unpacklo_epi32(in[6], in[7]), t7 = _mm256_unpackhi_epi32(in[6], in[7]);
    const __m256i u0 = _mm256_unpacklo_epi64(t0, t2), u1 = _mm256_unpackhi_epi64(t0, t2);
    const __m256i u2 = _mm256_unpacklo_epi64(t1, t3), u3 = _mm256_unpackhi_epi64(t1, t3);
    const __m256i u4 = _mm256_unpacklo_epi64(t4, t6), u5 = _mm256_unpackhi_epi64(t4, t6);
    const __m256i u6 = _mm256_unpacklo_epi64(t5, t7), u7 = _mm256_unpackhi_epi64(t5, t7);
    out[0] = _mm256_permute2x128_si256(u0, u4, 0x20);
    out[1] = _mm256_permute2x128_si256(u1, u5, 0x20);
    out[2] = _mm256_permute2x128_si256(u2, u6, 0x20);
    out[3] = _mm256_permute2x128_si256(u3, u7, 0x20);
    out[4] = _mm256_permute2x128_si256(u0, u4, 0x31);
    out[5] = _mm256_permute2x128_si256(u1, u5, 0x31);
    out[6] = _mm256_permute2x128_si256(u2, u6, 0x31);
    out[7] = _mm256_permute2x128_si256(u3, u7, 0x31);
}

// lane j hashes `blocks` 64-byte blocks at base + j*stride from the IV: chunk chaining values
// (CHUNK_START on the first block, CHUNK_END on the last, counter = counter0 + j) or parents
// (one block, PARENT, counter 0). out: 8 x 32 bytes, lane-major.
B3H_AVX2 void hash8(const uint8_t *base, size_t stride, size_t blocks, uint64_t counter0, bool per_lane_counter,
                    uint32_t first_flags, uint32_t last_flags, uint32_t all_flags, uint8_t *out) {
    __m256i cv[8];
    for (int i = 0; i < 8; i++) cv[i] = _mm256_set1_epi32((int)b3::K3.iv[i]);
    const __m256i lane = _mm256_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7);
    const uint64_t c0 = counter0;
    __m256i lo = _mm256_set1_epi32((int)(uint32_t)c0), hi = _mm256_set1_epi32((int)(uint32_t)(c0 >> 32));
    if (per_lane_counter) {
        const __m256i l2 = _mm256_add_epi32(lo, lane);
        // carry into the high word where the low word wrapped (unsigned l2 < lo)
        const __m256i bias = _mm256_set1_epi32((int)0x80000000u);
        const __m256i wrapped = _mm256_cmpgt_epi32(_mm256_xor_si256(lo, bias), _mm256_xor_si256(l2, bias));
        hi = _mm256_sub_epi32(hi, wrapped);
        lo = l2;
    }
    for (size_t b = 0; b < blocks; b++) {
        __m256i rows[8], m[16];
        for (int j = 0; j < 8; j++) rows[j] = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(base + j * stride + 64 * b));
        transpose8(rows, m);
        for (int j = 0; j < 8; j++)
            rows[j] = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(base + j * stride + 64 * b + 32));
        transpose8(rows, m + 8);
        const uint32_t flags = all_flags | (b == 0 ? first_flags : 0u) | (b + 1 == blocks ? last_flags : 0u);
        compress8(cv, m, lo, hi, 64, flags);
    }
    __m256i t[8];
    transpose8(cv, t);
    for (int j = 0; j < 8; j++) _mm256_storeu_si256(reinterpret_cast<__m256i *>(out + 32 * j), t[j]);
}

// ---- the same with AVX-512F: 16 lanes, native 32-bit rotates (vprord), 32 vector registers ----
#define B3H_AVX512 __attribute__((target("avx512f")))

B3H_AVX512 inline void g16(__m512i *v, int a, int b, int c, int d, __m512i x, __m512i y) {
    v[a] = _mm512_add_epi32(_mm512_add_epi32(v[a], v[b]), x);
    v[d] = _mm512_ror_epi32(_mm512_xor_si512(v[d], v[a]), 16);
    v[c] = _mm512_add_epi32(v[c], v[d]);
    v[b] = _mm512_ror_epi32(_mm512_xor_si512(v[b], v[c]), 12);
    v[a] = _mm512_add_epi32(_mm512_add_epi32(v[a], v[b]), y);
    v[d] = _mm512_ror_epi32(_mm512_xor_si512(v[d], v[a]), 8);
    v[c] = _mm512_add_epi32(v[c], v[d]);
    v[b] = _mm512_ror_epi32(_mm512_xor_si512(v[b], v[c]), 7);
}

B3H_AVX512 inline void compress16(__m512i cv[8], const __m512i m[16], __m512i ctr_lo, __m512i ctr_hi, uint32_t block_len,
                                  uint32_t flags) {
    __m512i v[16];
    for (int i = 0; i < 8; i++) v[i] = cv[i];
    for (int i = 0; i < 4; i++) v[8 + i] = _mm512_set1_epi32((int)b3::K3.iv[i]);
    v[12] = ctr_lo;
    v[13] = ctr_hi;
    v[14] = _mm512_set1_epi32((int)block_len);
    v[15] = _mm512_set1_epi32((int)flags);
    for (int r = 0; r < 7; r++) {
        const uint8_t *q = b3::K3.sched[r];
        g16(v, 0, 4, 8, 12, m[q[0]], m[q[1]]);
        g16(v, 1, 5, 9, 13, m[q[2]], m[q[3]]);
        g16(v, 2, 6, 10, 14, m[q[4]], m[q[5]]);
        g16(v, 3, 7, 11, 15, m[q[6]], m[q[7]]);
        g16(v, 0, 5, 10, 15, m[q[8]], m[q[9]]);
        g16(v, 1, 6, 11, 12, m[q[10]], m[q[11]]);
        g16(v, 2, 7, 8, 13, m[q[12]], m[q[13]]);
        g16(v, 3, 4, 9, 14, m[q[14]], m[q[15]]);
    }
    for (int i = 0; i < 8; i++) cv[i] = _mm512_xor_si512(v[i], v[i + 8]);
}

// 16x16 transpose of 32-bit words: in[j] = row j -> out[w] = word w of rows 0..15. Stage 1 interleaves
// 32-bit and 64-bit elements inside 128-bit lanes (u[4k+e], lane L = element 4L+e of rows 4k..4k+3),
// stage 2 is a 4x4 transpose of 128-bit lanes among u[e], u[4+e], u[8+e], u[12+e].
B3H_AVX512 inline void transpose16(const __m512i in[16], __m512i out[16]) {
    __m512i t[16], u[16];
    for (int k = 0; k < 8; k++) {
        t[2 * k] = _mm512_unpacklo_epi32(in[2 * k], in[2 * k + 1]);
        t[2 * k + 1] = _mm512_unpackhi_epi32(in[2 * k], in[2 * k + 1]);
    }
    for (int k = 0; k < 4; k++) {
        u[4 * k] = _mm512_unpacklo_epi64(t[4 * k], t[4 * k + 2]);
        u[4 * k + 1] = _mm512_unpackhi_epi64(t[4 * k], t[4 * k + 2]);
        u[4 * k + 2] = _mm512_unpacklo_epi64(t[4 * k + 1], t[4 * k + 3]);
        u[4 * k + 3] = _mm512_unpackhi_epi64(t[4 * k + 1], t[4 * k + 3]);
    }
    for (int e = 0; e < 4; e++) {
        const __m512i x0 = _mm512_shuffle_i32x4(u[e], u[4 + e], 0x44), x1 = _mm512_shuffle_i32x4(u[e], u[4 + e], 0xEE);
        const __m512i y0 = _mm512_shuffle_i32x4(u[8 + e], u[12 + e], 0x44), y1 = _mm512_shuffle_i32x4(u[8 + e], u[12 + e], 0xEE);
        out[e] = _mm512_shuffle_i32x4(x0, y0, 0x88);
        out[4 + e] = _mm512_shuffle_i32x4(x0, y0, 0xDD);
        out[8 + e] = _mm512_shuffle_i32x4(x1, y1, 0x88);
        out[12 + e] = _mm512_shuffle_i32x4(x1, y1, 0xDD);
    }
}

// hash8 with 16 lanes: lane j hashes `blocks` blocks at base + j*stride; out: 16 x 32 bytes
B3H_AVX512 void hash16(const uint8_t *base, size_t stride, size_t blocks, uint64_t counter0, bool per_lane_counter,
                       uint32_t first_flags, uint32_t last_flags, uint32_t all_flags, uint8_t *out) {
    __m512i cv[8];
    for (int i = 0; i < 8; i++) cv[i] = _mm512_set1_epi32((int)b3::K3.iv[i]);
    __m512i lo = _mm512_set1_epi32((int)(uint32_t)counter0), hi = _mm512_set1_epi32((int)(uint32_t)(counter0 >> 32));
    if (per_lane_counter) {
        const __m512i l2 = _mm512_add_epi32(lo, _mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15));
        hi = _mm512_mask_add_epi32(hi, _mm512_cmplt_epu32_mask(l2, lo), hi, _mm512_set1_epi32(1));  // carry
        lo = l2;
    }
    for (size_t b = 0; b < blocks; b++) {
        __m512i rows[16], m[16];
        for (int j = 0; j < 16; j++) rows[j] = _mm512_loadu_si512(base + j * stride + 64 * b);
        transpose16(rows, m);
        const uint32_t flags = all_flags | (b == 0 ? first_flags : 0u) | (b + 1 == blocks ? last_flags : 0u);
        compress16(cv, m, lo, hi, 64, flags);
    }
    __m512i rows[16], t[16];
    for (int i = 0; i < 8; i++) rows[i] = cv[i], rows[8 + i] = _mm512_setzero_si512();
    transpose16(rows, t);  // t[j] = lane j's 8 words (+ 8 zero words)
    for (int j = 0; j < 16; j++) _mm256_storeu_si256(reinterpret_cast<__m256i *>(out + 32 * j), _mm512_castsi512_si256(t[j]));
}

bool have_avx512() {
    static const int ok = __builtin_cpu_supports("avx512f") ? 1 : 0;
    return ok != 0;
}

bool have_avx2() {
    static const int ok = __builtin_cpu_supports("avx2") ? 1 : 0;
    return ok != 0;
}

}  // namespace

bool simd_available() { return have_avx2(); }

// chaining value of the complete power-of-two subtree of `nchunks` full chunks at p (chunk counter
// `first`), not finalised; nchunks in [8, MAX_SIMD_SUBTREE] and a power of two, AVX2 present
void simd_subtree(const uint8_t *p, size_t nchunks, uint64_t first, uint32_t cv[8]) {
    alignas(64) uint8_t buf[MAX_SIMD_SUBTREE * 32];
    const bool w16 = have_avx512();
    for (size_t c = 0; c < nchunks;) {
        if (w16 && c + 16 <= nchunks) {
            hash16(p + c * b3::CHUNK, b3::CHUNK, b3::CHUNK / b3::BLOCK, first + c, true, b3::CHUNK_START, b3::CHUNK_END, 0,
                   buf + 32 * c);
            c += 16;
        } else {
            hash8(p + c * b3::CHUNK, b3::CHUNK, b3::CHUNK / b3::BLOCK, first + c, true, b3::CHUNK_START, b3::CHUNK_END, 0,
                  buf + 32 * c);
            c += 8;
        }
    }
    size_t count = nchunks;
    // 16 or 8 parents at a time: parent k's message = values 2k, 2k+1 (64 adjacent bytes); in place
    // (a group reads values [2k, 2k + 2G) before writing [k, k + G))
    while (count >= 16) {
        const size_t np = count / 2;
        for (size_t k = 0; k < np;) {
            if (w16 && k + 16 <= np) {
                hash16(buf + 64 * k, 64, 1, 0, false, 0, 0, b3::PARENT, buf + 32 * k);
                k += 16;
            } else {
                hash8(buf + 64 * k, 64, 1, 0, false, 0, 0, b3::PARENT, buf + 32 * k);
                k += 8;
            }
        }
        count = np;
    }
    uint32_t w[8 * 8];
    for (size_t k = 0; k < count; k++)
        for (int i = 0; i < 8; i++) {
            const uint8_t *q = buf + 32 * k + 4 * i;
            w[8 * k + i] = (uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16 | (uint32_t)q[3] << 24;
        }
    while (count > 1) {  // the last 3 levels (8 -> 1) one parent at a time
        for (size_t k = 0; k < count / 2; k++) b3::parent(&w[16 * k], &w[16 * k + 8], 0, &w[8 * k]);
        count /= 2;
    }
    for (int i = 0; i < 8; i++) cv[i] = w[i];
}

}  // namespace b3h
}  // namespace decds

// blake3_impl.h — BLAKE3 compression shared by the device commitment kernels and the host
// helpers (crate blake3 =1.8.2 in decds' Cargo.lock; restated from the BLAKE3 specification).
// Only what decds' commitment layer needs: unkeyed hashing, 32-byte output.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define B3_HD __host__ __device__
#else
#define B3_HD
#endif

namespace decds {
namespace b3 {

enum : uint32_t { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8 };
constexpr uint32_t BLOCK = 64, CHUNK = 1024;

struct Consts {
    uint32_t iv[8];
    uint8_t sched[7][16];  // message word order of each round (permutation applied r times)
};

constexpr Consts make_consts() {
    Consts c{{0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au, 0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u},
             {}};
    constexpr uint8_t perm[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
    for (int i = 0; i < 16; i++) c.sched[0][i] = (uint8_t)i;
    for (int r = 1; r < 7; r++)
        for (int i = 0; i < 16; i++) c.sched[r][i] = c.sched[r - 1][perm[i]];
    return c;
}
constexpr Consts K3 = make_consts();

B3_HD inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// a + b + c. On gfx950 pinned to one v_add3_u32: left alone, hipcc re-associates G's two
// three-input sums into add pairs (~0.7 extra VALU per G, ~6% of a compression)
B3_HD inline uint32_t add3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(DECDS_B3_NO_ADD3)
    uint32_t r;
    asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
#else
    return a + b + c;
#endif
}

// chaining value (first 8 output words) of one compression
B3_HD inline void compress(const uint32_t cv[8], const uint32_t m[16], uint64_t counter, uint32_t block_len,
                           uint32_t flags, uint32_t out[8]) {
    uint32_t s[16] = {cv[0],    cv[1],    cv[2],    cv[3],    cv[4],          cv[5],
                      cv[6],    cv[7],    K3.iv[0], K3.iv[1], K3.iv[2],       K3.iv[3],
                      (uint32_t)counter, (uint32_t)(counter >> 32), block_len, flags};
#define B3G(a, b, c, d, x, y)      \
    s[a] = add3(s[a], s[b], (x));  \
    s[d] = rotr(s[d] ^ s[a], 16);  \
    s[c] = s[c] + s[d];            \
    s[b] = rotr(s[b] ^ s[c], 12);  \
    s[a] = add3(s[a], s[b], (y));  \
    s[d] = rotr(s[d] ^ s[a], 8);   \
    s[c] = s[c] + s[d];            \
    s[b] = rotr(s[b] ^ s[c], 7);
#pragma unroll
    for (int r = 0; r < 7; r++) {
        const uint8_t *q = K3.sched[r];
        B3G(0, 4, 8, 12, m[q[0]], m[q[1]]);
        B3G(1, 5, 9, 13, m[q[2]], m[q[3]]);
        B3G(2, 6, 10, 14, m[q[4]], m[q[5]]);
        B3G(3, 7, 11, 15, m[q[6]], m[q[7]]);
        B3G(0, 5, 10, 15, m[q[8]], m[q[9]]);
        B3G(1, 6, 11, 12, m[q[10]], m[q[11]]);
        B3G(2, 7, 8, 13, m[q[12]], m[q[13]]);
        B3G(3, 4, 9, 14, m[q[14]], m[q[15]]);
    }
#undef B3G
#pragma unroll
    for (int i = 0; i < 8; i++) out[i] = s[i] ^ s[i + 8];
}

// BLAKE3 of a 64-byte message (decds' Merkle parent_hash, merkle_tree.rs:158-160): one chunk of
// one block, so a single compression with CHUNK_START | CHUNK_END | ROOT
B3_HD inline void hash64(const uint32_t left[8], const uint32_t right[8], uint32_t out[8]) {
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        m[i] = left[i];
        m[i + 8] = right[i];
    }
    compress(K3.iv, m, 0, BLOCK, CHUNK_START | CHUNK_END | ROOT, out);
}

// BLAKE3 tree parent of two chaining values (PARENT, optionally ROOT)
B3_HD inline void parent(const uint32_t left[8], const uint32_t right[8], uint32_t flags, uint32_t out[8]) {
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        m[i] = left[i];
        m[i + 8] = right[i];
    }
    compress(K3.iv, m, 0, BLOCK, PARENT | flags, out);
}

}  // namespace b3
}  // namespace decds

// host_util.cpp — host-side control-path helpers of the C-ABI: the rank step over 10-byte coding
// vectors (rlnc Decoder's "piece useful?" test, chunkset.rs:181-183) and the seeded byte stream.
// These never touch chunk payloads; the payload arithmetic runs only in rlnc_kernels.hip.
#include <cstring>
#include <utility>

#include "../../include/decds_rlnc.h"
#include "capi_internal.h"
#include "rlnc_layout.h"

namespace decds {

uint8_t host_gf_mul(uint8_t a, uint8_t b, uint32_t poly) {
    uint32_t acc = 0, x = a;
    for (int i = 0; i < 8; i++) {
        if (b & (1u << i)) acc ^= x;
        x <<= 1;
        if (x & 0x100u) x ^= poly;
    }
    return (uint8_t)acc;
}

uint8_t host_gf_inv(uint8_t a, uint32_t poly) {
    uint8_t r = 1, b = a;
    for (unsigned e = 254; e; e >>= 1) {
        if (e & 1u) r = host_gf_mul(r, b, poly);
        b = host_gf_mul(b, b, poly);
    }
    return a ? r : 0;
}

uint32_t host_gf_generator(uint32_t poly) {
    for (uint32_t g = 2; g < 256; g++) {
        // order 255 = 3 * 5 * 17 iff g^(255/p) != 1 for each prime p, and g^255 == 1
        auto pw = [&](uint32_t e) {
            uint8_t r = 1, b = (uint8_t)g;
            for (; e; e >>= 1) {
                if (e & 1u) r = host_gf_mul(r, b, poly);
                b = host_gf_mul(b, b, poly);
            }
            return r;
        };
        if (pw(255) == 1 && pw(85) != 1 && pw(51) != 1 && pw(15) != 1) return g;
    }
    return 0;
}

bool host_gf_invert(const uint8_t *m, uint8_t *inv, uint32_t poly) {
    uint8_t a[K][2 * K];
    for (uint32_t i = 0; i < K; i++)
        for (uint32_t j = 0; j < K; j++) a[i][j] = m[i * K + j], a[i][K + j] = i == j;
    for (uint32_t c = 0; c < K; c++) {
        uint32_t p = c;
        while (p < K && !a[p][c]) p++;
        if (p == K) return false;
        if (p != c)
            for (uint32_t j = 0; j < 2 * K; j++) std::swap(a[p][j], a[c][j]);
        const uint8_t f = host_gf_inv(a[c][c], poly);
        for (uint32_t j = 0; j < 2 * K; j++) a[c][j] = host_gf_mul(a[c][j], f, poly);
        for (uint32_t r = 0; r < K; r++)
            if (r != c && a[r][c]) {
                const uint8_t g = a[r][c];
                for (uint32_t j = 0; j < 2 * K; j++) a[r][j] ^= host_gf_mul(g, a[c][j], poly);
            }
    }
    for (uint32_t i = 0; i < K; i++)
        for (uint32_t j = 0; j < K; j++) inv[i * K + j] = a[i][K + j];
    return true;
}

}  // namespace decds

using namespace decds;

extern "C" {

int decds_rank_push(uint8_t *basis, uint8_t *pivots, uint32_t *rank, const uint8_t *coeff, uint32_t poly) {
    if (!basis || !pivots || !rank || !coeff || *rank > K)
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "bad rank_push arguments");
    if (*rank == K) return 0;
    uint8_t r[K];
    std::memcpy(r, coeff, K);
    for (uint32_t e = 0; e < *rank; e++) {
        const uint8_t f = r[pivots[e]];
        if (f)
            for (uint32_t c = 0; c < K; c++) r[c] ^= host_gf_mul(f, basis[e * K + c], poly);
    }
    uint32_t p = K;
    for (uint32_t c = 0; c < K; c++)
        if (r[c]) { p = c; break; }
    if (p == K) return 0;
    const uint8_t inv = host_gf_inv(r[p], poly);
    for (uint32_t c = 0; c < K; c++) r[c] = host_gf_mul(r[c], inv, poly);
    for (uint32_t e = 0; e < *rank; e++) {
        const uint8_t f = basis[e * K + p];
        if (f)
            for (uint32_t c = 0; c < K; c++) basis[e * K + c] ^= host_gf_mul(f, r[c], poly);
    }
    std::memcpy(basis + *rank * K, r, K);
    pivots[*rank] = (uint8_t)p;
    (*rank)++;
    return 1;
}

void decds_fill_random_host(uint64_t seed, uint64_t off, uint8_t *dst, size_t nbytes) {
    auto word = [seed](uint64_t w) {
        uint64_t z = seed + (w + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    size_t i = 0;
    for (; i < nbytes && ((off + i) & 7); i++) dst[i] = (uint8_t)(word((off + i) >> 3) >> (8 * ((off + i) & 7)));
    for (; i + 8 <= nbytes; i += 8) {
        const uint64_t z = word((off + i) >> 3);
        std::memcpy(dst + i, &z, 8);  // little-endian: byte p%8 of the word
    }
    for (; i < nbytes; i++) dst[i] = (uint8_t)(word((off + i) >> 3) >> (8 * ((off + i) & 7)));
}

}  // extern "C"

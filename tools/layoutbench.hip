// layoutbench.hip — does the coded-row layout in HBM bound the encode? The codec kernels' memory
// pattern without the GF arithmetic (as tools/hbmbench.hip's codec_k: per 16-column lane block 10
// input-row loads, then 16 output-row stores), with the coded rows in one of two layouts:
//   rows       row j of chunkset c at (c*16 + j) * pitch (pitch 1,048,704, payload 128-B aligned):
//              a tile's 16 row segments are 1 MiB apart — the shipped device layout
//   tilemajor  [chunkset][tile][row][4096 B]: a tile's 16 row segments are one contiguous 64 KiB
//              (rows are no longer contiguous; a host copy-out would gather them)
// and the flat copy (one float4 per thread, no grid stride) as the reference ceiling. Every variant
// is warmed for --warm-ms, then --reps launches are timed one by one; GB/s = bytes read + written.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/layoutbench.hip -o tools/bin/layoutbench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                            \
    do {                                                                 \
        hipError_t e_ = (x);                                             \
        if (e_ != hipSuccess) {                                          \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
            std::exit(1);                                                \
        }                                                                \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint64_t CSB = 10ull << 20, LB = (CSB + 10) / 10, FB = LB + 10, PITCH = 1048704;
constexpr uint32_t BLOCKS = 65535, TILES = 256, TILE_COLS = 4096;
constexpr uint64_t TM_TILE = 16ull * TILE_COLS;          // one tile of the 16 rows, tile-major
constexpr uint64_t TM_CS = TILES * TM_TILE;               // one chunkset, tile-major (16 MiB)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, 0x80000000u, 0x00020000);
}

// workgroup -> unit: ORDER 0 dispatcher order, 1 each XCD sweeps one contiguous eighth, 2 dispatcher
// order with a unit's tiles strided (tile r + k * 256/UNIT of its chunkset: the resident workgroups
// sweep every chunkset's rows together), ORDER = 100 + R: runs of R consecutive units per XCD in
// global order (blocks b = 8R·grp + 8j + x -> unit 8R·grp + R·x + j; the grid a multiple of 8R), so a
// unit's neighbours share its XCD's L2 except at every R-th edge
template <int ORDER>
__device__ __forceinline__ uint32_t unit_of() {
    uint32_t u = blockIdx.x;
    if constexpr (ORDER == 1) {
        const uint32_t g = gridDim.x, x = u % 8, q = u / 8, per = g / 8, rem = g % 8;
        u = x * per + (x < rem ? x : rem) + q;
    }
    if constexpr (ORDER > 100) {
        constexpr uint32_t R = ORDER - 100;
        const uint32_t x = u % 8, q = u / 8;
        u = (q / R) * 8 * R + x * R + q % R;
    }
    return u;
}

// encode pattern: inputs = pieces of the contiguous chunkset (i * L), outputs in layout TM
template <int UNIT, int ORDER, bool TM>
__global__ __launch_bounds__(256) void enc_k(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, size_t n) {
    extern __shared__ uint8_t lds[];
    const uint32_t t0 = unit_of<ORDER>() * UNIT, cs = t0 / TILES, tile0 = t0 % TILES;
    if (cs >= n) return;
    const auto ri = rsrc(in + cs * CSB);
    const auto ro = rsrc(out + cs * (TM ? TM_CS : 16 * PITCH));
    u32x4 acc = {0, 0, 0, 0};
    constexpr uint32_t UPC = TILES / UNIT;  // units per chunkset
    for (uint32_t k = 0; k < UNIT; k++) {
        const uint32_t t = ORDER == 2 ? (tile0 / UNIT) + k * UPC : tile0 + k;
        const uint32_t b = t * 256 + threadIdx.x;
        const uint32_t col = b < BLOCKS ? b * 16 : 0x80000000u;
        u32x4 x[10];
#pragma unroll
        for (int i = 0; i < 10; i++) x[i] = __builtin_amdgcn_raw_buffer_load_b128(ri, (uint32_t)(i * LB) + col, 0, 0);
#pragma unroll
        for (int i = 0; i < 10; i++) acc ^= x[i];
        // tilemajor: row j of tile t at t*64 KiB + j*4 KiB (+ the lane's column within the tile)
        const uint32_t obase = TM ? (b < BLOCKS ? t * (uint32_t)TM_TILE + threadIdx.x * 16 : 0x80000000u) : 128 + col;
#pragma unroll
        for (int j = 0; j < 16; j++)
            __builtin_amdgcn_raw_buffer_store_b128(acc + (uint32_t)j, ro, obase + (uint32_t)(j * (TM ? TILE_COLS : PITCH)), 0, 0);
    }
    if (acc.x == 0x9E3779B9u && threadIdx.x == 999) lds[0] = 1;  // keeps the LDS allocation referenced
}

// decode pattern: inputs = 10 of the 16 coded rows (rows 0, 2, 3, 5, 6, 8, 9, 11, 13, 15) in layout
// TM, outputs = pieces of the contiguous chunkset
// SPLIT: the piece stores of the real (byte-misaligned) layout cut at 4-byte boundaries inside each
// lane — a 12-byte store of the lane's dword-aligned middle plus 1-2 byte / short stores of its head
// and tail, no cross-lane exchange; A4: one 16-byte store 4-byte aligned (address rounded down, wrong
// bytes: the pattern of a dword-aligned realignment)
enum : int { ST_PLAIN = 0, ST_SPLIT = 1, ST_A4 = 2 };
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
template <int ST>
__device__ __forceinline__ void piece_store(u32x4 v, __amdgpu_buffer_rsrc_t ro, uint32_t o, uint32_t r) {
    if (ST == ST_PLAIN || r == 0) {
        __builtin_amdgcn_raw_buffer_store_b128(v, ro, o, 0, 0);
    } else if (ST == ST_A4) {
        __builtin_amdgcn_raw_buffer_store_b128(v, ro, o - r, 0, 0);
    } else {
        const uint32_t h = 4 - r;
        uint32_t w[5] = {v.x, v.y, v.z, v.w, 0};
        u32x3 mid;
        mid.x = __builtin_amdgcn_alignbyte(w[1], w[0], h);
        mid.y = __builtin_amdgcn_alignbyte(w[2], w[1], h);
        mid.z = __builtin_amdgcn_alignbyte(w[3], w[2], h);
        __builtin_amdgcn_raw_buffer_store_b96(mid, ro, o + h, 0, 0);
        if (r == 1) {
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)w[0], ro, o, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(w[0] >> 8), ro, o + 1, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(w[3] >> 24), ro, o + 15, 0, 0);
        } else if (r == 2) {
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)w[0], ro, o, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(w[3] >> 16), ro, o + 14, 0, 0);
        } else {
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)w[0], ro, o, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(w[3] >> 8), ro, o + 13, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(w[3] >> 24), ro, o + 15, 0, 0);
        }
    }
}

template <int UNIT, bool TM, uint64_t OROW = LB, int ST = ST_PLAIN, int ORDER = 0>
__global__ __launch_bounds__(256) void dec_k(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, size_t n) {
    extern __shared__ uint8_t lds[];
    const uint32_t t0 = unit_of<ORDER>() * UNIT, cs = t0 / TILES, tile0 = t0 % TILES;
    if (cs >= n) return;
    constexpr uint32_t sel[10] = {0, 2, 3, 5, 6, 8, 9, 11, 13, 15};
    const auto ri = rsrc(in + cs * (TM ? TM_CS : 16 * PITCH));
    const auto ro = rsrc(out + cs * CSB);
    u32x4 acc = {0, 0, 0, 0};
    for (uint32_t t = tile0; t < tile0 + UNIT; t++) {
        const uint32_t b = t * 256 + threadIdx.x;
        const uint32_t col = b < BLOCKS ? b * 16 : 0x80000000u;
        const uint32_t ibase = TM ? (b < BLOCKS ? t * (uint32_t)TM_TILE + threadIdx.x * 16 : 0x80000000u) : 128 + col;
        u32x4 x[10];
#pragma unroll
        for (int k = 0; k < 10; k++)
            x[k] = __builtin_amdgcn_raw_buffer_load_b128(ri, ibase + sel[k] * (uint32_t)(TM ? TILE_COLS : PITCH), 0, 0);
#pragma unroll
        for (int k = 0; k < 10; k++) acc ^= x[k];
#pragma unroll
        for (int i = 0; i < 10; i++) piece_store<ST>(acc + (uint32_t)i, ro, (uint32_t)(i * OROW) + col, (uint32_t)(i * OROW) & 3);
    }
    if (acc.x == 0x9E3779B9u && threadIdx.x == 999) lds[0] = 1;
}

// decode pattern with line-aligned stores and all 64 lanes busy: a workgroup's 4 waves store the 256
// aligned granules of their tile (4 KiB per piece, 32 whole lines) — every lane its block's granule,
// whose first i bytes belong to the previous block (another wave's lane 63 for lane 0: an LDS
// exchange in the real kernel). At tile edges the granule reaches into the previous tile, so the
// tile's first lane stores its block at the real (misaligned) offset instead and the tile's last lane
// adds a misaligned store of its own block. The stores only, no arithmetic.
template <int ORDER = 0>
__global__ __launch_bounds__(256) void dec_tile_lines_k(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, size_t n) {
    extern __shared__ uint8_t lds[];
    const uint32_t u = unit_of<ORDER>(), cs = u / TILES, t = u % TILES;
    if (cs >= n) return;
    constexpr uint32_t sel[10] = {0, 2, 3, 5, 6, 8, 9, 11, 13, 15};
    const auto ri = rsrc(in + cs * 16 * PITCH);
    const auto ro = rsrc(out + cs * CSB);
    const uint32_t g = t * 256 + threadIdx.x;
    const uint32_t col = g < BLOCKS ? g * 16 : 0x80000000u;
    u32x4 x[10], acc = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 10; k++) x[k] = __builtin_amdgcn_raw_buffer_load_b128(ri, 128 + col + sel[k] * (uint32_t)PITCH, 0, 0);
#pragma unroll
    for (int k = 0; k < 10; k++) acc ^= x[k];
    const bool first = threadIdx.x == 0, last = threadIdx.x == 255 || g == BLOCKS - 1;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        const uint32_t off = first ? (uint32_t)(i * LB) + col : (uint32_t)(i << 20) + col;  // real offset : aligned granule
        __builtin_amdgcn_raw_buffer_store_b128(acc + (uint32_t)i, ro, off, 0, 0);
    }
    if (last)
#pragma unroll
        for (int i = 0; i < 10; i++) __builtin_amdgcn_raw_buffer_store_b128(acc + (uint32_t)i, ro, (uint32_t)(i * LB) + col, 0, 0);
    if (acc.x == 0x9E3779B9u && threadIdx.x == 999) lds[0] = 1;
}

// decode pattern of a line-aligned walk over T consecutive tiles per workgroup: every lane stores its
// block's aligned granule (the previous block's bytes from the neighbour lane / previous wave / previous
// tile in a real kernel), so every wave store is 8 whole lines; only the walk's first tile's first lane
// stores its block at the real (misaligned) offset and the walk's last lane adds a store at the real
// offset. Workgroup -> walk through unit_of<ORDER> (100 + R: runs of R walks per XCD). The stores only.
template <uint32_t T, int ORDER = 0>
__global__ __launch_bounds__(256) void dec_walk_lines_k(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, size_t n) {
    extern __shared__ uint8_t lds[];
    constexpr uint32_t WPC = TILES / T;  // walks per chunkset
    const uint32_t u = unit_of<ORDER>(), cs = u / WPC, t0 = (u % WPC) * T;
    if (cs >= n) return;
    constexpr uint32_t sel[10] = {0, 2, 3, 5, 6, 8, 9, 11, 13, 15};
    const auto ri = rsrc(in + cs * 16 * PITCH);
    const auto ro = rsrc(out + cs * CSB);
    u32x4 acc = {0, 0, 0, 0};
    for (uint32_t t = t0; t < t0 + T; t++) {
        const uint32_t g = t * 256 + threadIdx.x;
        const uint32_t col = g < BLOCKS ? g * 16 : 0x80000000u;
        u32x4 x[10];
#pragma unroll
        for (int k = 0; k < 10; k++) x[k] = __builtin_amdgcn_raw_buffer_load_b128(ri, 128 + col + sel[k] * (uint32_t)PITCH, 0, 0);
#pragma unroll
        for (int k = 0; k < 10; k++) acc ^= x[k];
        const bool first = t == t0 && threadIdx.x == 0, last = (t == t0 + T - 1 && threadIdx.x == 255) || g == BLOCKS - 1;
#pragma unroll
        for (int i = 0; i < 10; i++) {
            const uint32_t off = first ? (uint32_t)(i * LB) + col : (uint32_t)(i << 20) + col;
            __builtin_amdgcn_raw_buffer_store_b128(acc + (uint32_t)i, ro, off, 0, 0);
        }
        if (last)
#pragma unroll
            for (int i = 0; i < 10; i++) __builtin_amdgcn_raw_buffer_store_b128(acc + (uint32_t)i, ro, (uint32_t)(i * LB) + col, 0, 0);
    }
    if (acc.x == 0x9E3779B9u && threadIdx.x == 999) lds[0] = 1;
}

// decode pattern: a workgroup's 256 lanes compute 256 consecutive blocks, lane 0 the block before the
// tile (recomputed), and lanes 1..248 store 248 aligned granules = 31 whole lines per piece (lanes
// 249..255 idle): no straggler crosses a workgroup; wave runs (63 / 64 / 64 / 57 granules) meet inside
// the workgroup at arbitrary 16-byte boundaries. The stores only.
__global__ __launch_bounds__(256) void dec_wg248_k(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, size_t n) {
    extern __shared__ uint8_t lds[];
    constexpr uint32_t PER = 248, T2 = (BLOCKS + PER - 1) / PER;
    const uint32_t cs = blockIdx.x / T2, t = blockIdx.x % T2;
    if (cs >= n) return;
    constexpr uint32_t sel[10] = {0, 2, 3, 5, 6, 8, 9, 11, 13, 15};
    const auto ri = rsrc(in + cs * 16 * PITCH);
    const auto ro = rsrc(out + cs * CSB);
    const uint32_t l = threadIdx.x;
    const uint32_t g = t * PER + l - 1;
    const bool live = l <= PER && g < BLOCKS;
    const uint32_t col = live ? g * 16 : 0x80000000u;
    u32x4 x[10], acc = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 10; k++) x[k] = __builtin_amdgcn_raw_buffer_load_b128(ri, 128 + col + sel[k] * (uint32_t)PITCH, 0, 0);
#pragma unroll
    for (int k = 0; k < 10; k++) acc ^= x[k];
    const uint32_t ocol = l >= 1 && live ? g * 16 : 0x80000000u;
#pragma unroll
    for (int i = 0; i < 10; i++) __builtin_amdgcn_raw_buffer_store_b128(acc + (uint32_t)i, ro, (uint32_t)(i << 20) + ocol, 0, 0);
    if (acc.x == 0x9E3779B9u && threadIdx.x == 999) lds[0] = 1;
}

// decode pattern of a persistent line-aligned walk: each wave owns R consecutive 1-KiB column runs
// (64 blocks each) and walks them in order; every store instruction is 64 aligned granules = 8 whole
// lines (the previous block's bytes come from the previous iteration's lane 63 in a real kernel),
// except at the start of the wave's walk, where lane 0 stores its block at the real offset, and at its
// end, where lane 63 adds a store of its block at the real offset. The stores only.
template <uint32_t R>
__global__ __launch_bounds__(256) void dec_walk_k(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, size_t n) {
    extern __shared__ uint8_t lds[];
    constexpr uint32_t PER_WG = 4 * 64 * R, T2 = (BLOCKS + PER_WG - 1) / PER_WG;
    const uint32_t cs = blockIdx.x / T2, t = blockIdx.x % T2;
    if (cs >= n) return;
    constexpr uint32_t sel[10] = {0, 2, 3, 5, 6, 8, 9, 11, 13, 15};
    const auto ri = rsrc(in + cs * 16 * PITCH);
    const auto ro = rsrc(out + cs * CSB);
    const uint32_t l = threadIdx.x & 63u, w = threadIdx.x >> 6;
    u32x4 acc = {0, 0, 0, 0};
    for (uint32_t r = 0; r < R; r++) {
        const uint32_t g = t * PER_WG + w * 64 * R + r * 64 + l;
        const uint32_t col = g < BLOCKS ? g * 16 : 0x80000000u;
        u32x4 x[10];
#pragma unroll
        for (int k = 0; k < 10; k++) x[k] = __builtin_amdgcn_raw_buffer_load_b128(ri, 128 + col + sel[k] * (uint32_t)PITCH, 0, 0);
#pragma unroll
        for (int k = 0; k < 10; k++) acc ^= x[k];
        const bool head = r == 0 && l == 0;
#pragma unroll
        for (int i = 0; i < 10; i++)
            __builtin_amdgcn_raw_buffer_store_b128(acc + (uint32_t)i, ro, (head ? (uint32_t)(i * LB) : (uint32_t)(i << 20)) + col, 0, 0);
        if (r == R - 1 && l == 63)
#pragma unroll
            for (int i = 0; i < 10; i++) __builtin_amdgcn_raw_buffer_store_b128(acc + (uint32_t)i, ro, (uint32_t)(i * LB) + col, 0, 0);
    }
    if (acc.x == 0x9E3779B9u && threadIdx.x == 999) lds[0] = 1;
}

// encode pattern with line-aligned input runs (the load side of a DPP-realigned encode): each wave
// loads 57 consecutive 16-byte input granules per piece — lanes 0..56, lanes 57..63 idle — and lanes
// 0..55 store 56 blocks (7 whole lines) of each of the 16 coded rows (payload-aligned rows). ALIGN
// true: pieces 1 MiB apart (granules line-aligned); false: the real pieces at i*L.
template <bool ALIGN>
__global__ __launch_bounds__(256) void enc_lines_k(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, size_t n) {
    extern __shared__ uint8_t lds[];
    constexpr uint32_t PER_WAVE = 56, PER_TILE = 4 * PER_WAVE, T2 = (BLOCKS + PER_TILE - 1) / PER_TILE;
    const uint32_t cs = blockIdx.x / T2, t = blockIdx.x % T2;
    if (cs >= n) return;
    const auto ri = rsrc(in + cs * CSB);
    const auto ro = rsrc(out + cs * 16 * PITCH);
    const uint32_t l = threadIdx.x & 63u;
    const uint32_t g = t * PER_TILE + (threadIdx.x >> 6) * PER_WAVE + l;
    const uint32_t col = l <= PER_WAVE && g < BLOCKS ? g * 16 : 0x80000000u;
    u32x4 x[10], acc = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 10; i++) x[i] = __builtin_amdgcn_raw_buffer_load_b128(ri, (uint32_t)(i * (ALIGN ? (1u << 20) : LB)) + col, 0, 0);
#pragma unroll
    for (int i = 0; i < 10; i++) acc ^= x[i];
    const uint32_t ocol = l < PER_WAVE && g < BLOCKS ? 128 + g * 16 : 0x80000000u;
#pragma unroll
    for (int j = 0; j < 16; j++) __builtin_amdgcn_raw_buffer_store_b128(acc + (uint32_t)j, ro, ocol + (uint32_t)(j * PITCH), 0, 0);
    if (acc.x == 0x9E3779B9u && threadIdx.x == 999) lds[0] = 1;
}

// decode pattern with line-aligned wave stores (the store side of a DPP-realigned decode): each wave
// computes 57 consecutive lane blocks — lane 0 the block before its run, lanes 57..63 idle — and each
// of lanes 1..56 stores one 16-byte granule per output piece: 7 whole 128-byte lines per wave and piece
// (pieces 1 MiB apart). ALIGN false: the same runs at the real piece offsets i*L (byte-misaligned).
template <bool ALIGN>
__global__ __launch_bounds__(256) void dec_lines_k(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, size_t n) {
    extern __shared__ uint8_t lds[];
    constexpr uint32_t PER_WAVE = 56, PER_TILE = 4 * PER_WAVE, T2 = (BLOCKS + PER_TILE - 1) / PER_TILE;
    const uint32_t cs = blockIdx.x / T2, t = blockIdx.x % T2;
    if (cs >= n) return;
    constexpr uint32_t sel[10] = {0, 2, 3, 5, 6, 8, 9, 11, 13, 15};
    const auto ri = rsrc(in + cs * 16 * PITCH);
    const auto ro = rsrc(out + cs * CSB);
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63u;
    const uint32_t g = t * PER_TILE + w * PER_WAVE + l - 1;  // wraps for the chunkset's first lane 0
    const bool in_run = l <= PER_WAVE && g < BLOCKS;
    const uint32_t col = in_run ? g * 16 : 0x80000000u;
    u32x4 x[10], acc = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 10; k++) x[k] = __builtin_amdgcn_raw_buffer_load_b128(ri, 128 + col + sel[k] * (uint32_t)PITCH, 0, 0);
#pragma unroll
    for (int k = 0; k < 10; k++) acc ^= x[k];
    const uint32_t ocol = (l >= 1 && in_run) ? g * 16 : 0x80000000u;
#pragma unroll
    for (int i = 0; i < 10; i++)
        __builtin_amdgcn_raw_buffer_store_b128(acc + (uint32_t)i, ro, (uint32_t)(i * (ALIGN ? (1u << 20) : LB)) + ocol, 0, 0);
    if (acc.x == 0x9E3779B9u && threadIdx.x == 999) lds[0] = 1;
}

__global__ __launch_bounds__(256) void copy_flat(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, size_t n16) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n16) d[i] = s[i];
}

struct Args {
    int warm_ms = 400, reps = 20;
};

template <typename F>
void run(const char *name, size_t n, double bytes, F f, const Args &a) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() < a.warm_ms) {
        for (int i = 0; i < 5; i++) f();
        CK(hipDeviceSynchronize());
    }
    std::vector<float> ms;
    for (int r = 0; r < a.reps; r++) {
        CK(hipEventRecord(e0));
        f();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    std::printf("{\"variant\": \"%s\", \"chunksets\": %zu, \"ms_med\": %.4f, \"GBps_med\": %.1f, \"GBps_best\": %.1f}\n", name, n,
                ms[ms.size() / 2], bytes / ms[ms.size() / 2] / 1e6, bytes / ms[0] / 1e6);
    std::fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

int main(int argc, char **argv) {
    Args a;
    std::string only;
    for (int i = 1; i < argc; i++) {
        if (!std::strcmp(argv[i], "--warm-ms")) a.warm_ms = std::atoi(argv[++i]);
        if (!std::strcmp(argv[i], "--reps")) a.reps = std::atoi(argv[++i]);
        if (!std::strcmp(argv[i], "--only")) only = argv[++i];
    }
    const size_t nmax = 1024;
    uint8_t *src, *coded, *rep;
    CK(hipMalloc(&src, nmax * CSB + 4096));
    CK(hipMalloc(&coded, nmax * 16 * PITCH + 4096));
    CK(hipMalloc(&rep, nmax * CSB + 4096));
    CK(hipMemset(src, 0x3c, nmax * CSB));
    CK(hipMemset(coded, 0x5a, nmax * 16 * PITCH));
    constexpr uint32_t LDS2 = 80 * 1024;  // 2 workgroups per CU, as the codec kernels' VGPRs allow
    for (const void *f : {(const void *)dec_k<1, false>, (const void *)dec_k<1, false, 1u << 20>, (const void *)dec_k<1, false, LB, ST_SPLIT>,
                          (const void *)dec_k<1, false, (1u << 20) + 16>,
                          (const void *)dec_k<1, false, LB, ST_A4>, (const void *)dec_lines_k<true>, (const void *)dec_lines_k<false>,
                          (const void *)enc_lines_k<true>, (const void *)enc_lines_k<false>, (const void *)dec_tile_lines_k<0>, (const void *)dec_tile_lines_k<104>, (const void *)dec_tile_lines_k<108>, (const void *)dec_tile_lines_k<116>,
                          (const void *)dec_k<1, false, LB, ST_PLAIN, 104>, (const void *)dec_k<1, false, LB, ST_PLAIN, 108>, (const void *)dec_k<1, false, LB, ST_PLAIN, 116>, (const void *)dec_k<1, false, 1u << 20, ST_PLAIN, 108>,
                          (const void *)enc_k<1, 108, false>, (const void *)dec_walk_lines_k<4>, (const void *)dec_walk_lines_k<4, 102>,
                          (const void *)dec_walk_lines_k<8>, (const void *)dec_walk_lines_k<2, 104>, (const void *)dec_walk_lines_k<1, 108>, (const void *)dec_wg248_k, (const void *)dec_walk_k<4>, (const void *)dec_walk_k<8>,
                          (const void *)dec_walk_k<16>, (const void *)enc_k<4, 1, false>, (const void *)enc_k<4, 0, false>, (const void *)enc_k<4, 2, false>,
                          (const void *)enc_k<2, 0, false>, (const void *)enc_k<1, 0, false>, (const void *)enc_k<8, 2, false>})
        CK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS2));
    for (size_t n : {103, 256, 1024}) {
        const double eb = (double)n * (CSB + 16 * FB), db = (double)n * (10 * FB + CSB);
        const unsigned g4 = (unsigned)(n * TILES / 4), g1 = (unsigned)(n * TILES), g2 = g1 / 2, g8 = g1 / 8;
        if (only.empty() || only == "occ") {
            run("enc_u4_xcd_2wg", n, eb, [&] { enc_k<4, 1, false><<<g4, 256, LDS2>>>(src, coded, n); }, a);
            run("enc_u4_disp_2wg", n, eb, [&] { enc_k<4, 0, false><<<g4, 256, LDS2>>>(src, coded, n); }, a);
            run("enc_u4_strided_2wg", n, eb, [&] { enc_k<4, 2, false><<<g4, 256, LDS2>>>(src, coded, n); }, a);
            run("enc_u8_strided_2wg", n, eb, [&] { enc_k<8, 2, false><<<g8, 256, LDS2>>>(src, coded, n); }, a);
            run("enc_u2_disp_2wg", n, eb, [&] { enc_k<2, 0, false><<<g2, 256, LDS2>>>(src, coded, n); }, a);
            run("enc_u1_disp_2wg", n, eb, [&] { enc_k<1, 0, false><<<g1, 256, LDS2>>>(src, coded, n); }, a);
            run("enc_u4_strided", n, eb, [&] { enc_k<4, 2, false><<<g4, 256>>>(src, coded, n); }, a);
            if (!only.empty()) continue;
        }
        if (only == "enclines") {
            const unsigned gl = (unsigned)(n * ((BLOCKS + 223) / 224));
            run("enc_u1_disp_2wg", n, eb, [&] { enc_k<1, 0, false><<<g1, 256, LDS2>>>(src, coded, n); }, a);
            run("enc_lines56_inA_2wg", n, eb, [&] { enc_lines_k<true><<<gl, 256, LDS2>>>(src, coded, n); }, a);
            run("enc_lines56_real_2wg", n, eb, [&] { enc_lines_k<false><<<gl, 256, LDS2>>>(src, coded, n); }, a);
            run("copy_flat", n, 2.0 * n * CSB, [&] {
                const size_t n16 = (size_t)n * CSB / 16;
                copy_flat<<<(unsigned)((n16 + 255) / 256), 256>>>((const u32x4 *)src, (u32x4 *)rep, n16);
            }, a);
            continue;
        }
        if (only == "walklines") {
            // line-aligned walks of T tiles (stragglers only at walk ends) against the plain decode
            constexpr uint32_t LDS3 = 52 * 1024;
            run("dec_u1_grp8_3wg", n, db, [&] { dec_k<1, false, LB, ST_PLAIN, 108><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_u1_outA_3wg", n, db, [&] { dec_k<1, false, 1u << 20><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_walklines1_grp8_3wg", n, db, [&] { dec_walk_lines_k<1, 108><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_walklines2_grp4_3wg", n, db, [&] { dec_walk_lines_k<2, 104><<<g1 / 2, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_walklines4_3wg", n, db, [&] { dec_walk_lines_k<4><<<g1 / 4, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_walklines4_grp2_3wg", n, db, [&] { dec_walk_lines_k<4, 102><<<g1 / 4, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_walklines8_3wg", n, db, [&] { dec_walk_lines_k<8><<<g1 / 8, 256, LDS3>>>(coded, rep, n); }, a);
            continue;
        }
        if (only == "xcdgrp") {
            // tile edges on one XCD: do partial lines written from two XCDs' L2s cost the misaligned
            // decode stores? runs of R consecutive tiles per XCD, global order otherwise
            constexpr uint32_t LDS3 = 52 * 1024;
            run("dec_u1_3wg", n, db, [&] { dec_k<1, false><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_u1_grp4_3wg", n, db, [&] { dec_k<1, false, LB, ST_PLAIN, 104><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_u1_grp8_3wg", n, db, [&] { dec_k<1, false, LB, ST_PLAIN, 108><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_u1_grp16_3wg", n, db, [&] { dec_k<1, false, LB, ST_PLAIN, 116><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_u1_outA_3wg", n, db, [&] { dec_k<1, false, 1u << 20><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_u1_outA_grp8_3wg", n, db, [&] { dec_k<1, false, 1u << 20, ST_PLAIN, 108><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_tile_lines_3wg", n, db, [&] { dec_tile_lines_k<0><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_tile_lines_grp4_3wg", n, db, [&] { dec_tile_lines_k<104><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_tile_lines_grp8_3wg", n, db, [&] { dec_tile_lines_k<108><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_tile_lines_grp16_3wg", n, db, [&] { dec_tile_lines_k<116><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("enc_u1_disp_2wg", n, eb, [&] { enc_k<1, 0, false><<<g1, 256, LDS2>>>(src, coded, n); }, a);
            run("enc_u1_grp8_2wg", n, eb, [&] { enc_k<1, 108, false><<<g1, 256, LDS2>>>(src, coded, n); }, a);
            continue;
        }
        if (only == "declines") {
            constexpr uint32_t LDS3 = 52 * 1024;
            const unsigned gl = (unsigned)(n * ((BLOCKS + 223) / 224));
            run("dec_u1_3wg", n, db, [&] { dec_k<1, false><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_u1_outA_3wg", n, db, [&] { dec_k<1, false, 1u << 20><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_lines56_aligned_3wg", n, db, [&] { dec_lines_k<true><<<gl, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_lines56_real_3wg", n, db, [&] { dec_lines_k<false><<<gl, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_lines56_aligned_2wg", n, db, [&] { dec_lines_k<true><<<gl, 256, LDS2>>>(coded, rep, n); }, a);
            const unsigned gw = (unsigned)(n * ((BLOCKS + 247) / 248));
            run("dec_wg248_3wg", n, db, [&] { dec_wg248_k<<<gw, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_walk4_3wg", n, db, [&] { dec_walk_k<4><<<(unsigned)(n * ((BLOCKS + 1023) / 1024)), 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_walk8_3wg", n, db, [&] { dec_walk_k<8><<<(unsigned)(n * ((BLOCKS + 2047) / 2048)), 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_walk16_3wg", n, db, [&] { dec_walk_k<16><<<(unsigned)(n * ((BLOCKS + 4095) / 4096)), 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_tile_lines_3wg", n, db, [&] { dec_tile_lines_k<0><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_tile_lines_2wg", n, db, [&] { dec_tile_lines_k<0><<<g1, 256, LDS2>>>(coded, rep, n); }, a);
            run("dec_u1_2wg", n, db, [&] { dec_k<1, false><<<g1, 256, LDS2>>>(coded, rep, n); }, a);
            continue;
        }
        if (only.empty() || only == "dec") {
            // decode outputs: the chunkset's pieces at i*L (byte-misaligned by i, the real layout) or
            // 1 MiB apart (16-byte aligned), at the decode kernel's occupancy (3 workgroups per CU) and free
            constexpr uint32_t LDS3 = 52 * 1024;
            run("dec_u1_3wg", n, db, [&] { dec_k<1, false><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_u1_outA_3wg", n, db, [&] { dec_k<1, false, 1u << 20><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_u1_outA16_3wg", n, db, [&] { dec_k<1, false, (1u << 20) + 16><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_u1_split_3wg", n, db, [&] { dec_k<1, false, LB, ST_SPLIT><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_u1_a4_3wg", n, db, [&] { dec_k<1, false, LB, ST_A4><<<g1, 256, LDS3>>>(coded, rep, n); }, a);
            run("dec_u1", n, db, [&] { dec_k<1, false><<<g1, 256>>>(coded, rep, n); }, a);
            run("dec_u1_outA", n, db, [&] { dec_k<1, false, 1u << 20><<<g1, 256>>>(coded, rep, n); }, a);
            run("dec_u1_split", n, db, [&] { dec_k<1, false, LB, ST_SPLIT><<<g1, 256>>>(coded, rep, n); }, a);
            if (!only.empty()) continue;
        }
        run("enc_rows_u4_xcd", n, eb, [&] { enc_k<4, 1, false><<<g4, 256>>>(src, coded, n); }, a);
        run("enc_rows_u1_disp", n, eb, [&] { enc_k<1, 0, false><<<g1, 256>>>(src, coded, n); }, a);
        run("enc_tilemajor_u4_xcd", n, eb, [&] { enc_k<4, 1, true><<<g4, 256>>>(src, coded, n); }, a);
        run("enc_tilemajor_u1_disp", n, eb, [&] { enc_k<1, 0, true><<<g1, 256>>>(src, coded, n); }, a);
        run("dec_rows_u1", n, db, [&] { dec_k<1, false><<<g1, 256>>>(coded, rep, n); }, a);
        run("dec_tilemajor_u1", n, db, [&] { dec_k<1, true><<<g1, 256>>>(coded, rep, n); }, a);
        const size_t n16 = (size_t)n * CSB / 16;
        run("copy_flat", n, 2.0 * n * CSB, [&] { copy_flat<<<(unsigned)((n16 + 255) / 256), 256>>>((const u32x4 *)src, (u32x4 *)rep, n16); }, a);
    }
    CK(hipDeviceSynchronize());
    return 0;
}

// copypattern.hip — the decode's own copy ceiling: a kernel with exactly
// rlnc_decode_kernel's HBM address stream and nothing else. Per chunkset c that its plan marks ready
// (RepairPlan::rank == 10), per 16-column lane block b < MAIN_BLOCKS: ten 16-byte loads of the plan's
// selected coded rows at their payload offset (row (c*16 + sel[k]) * pitch + 10 + 16b: 128-byte
// aligned in the payload-aligned layout) and ten 16-byte stores at out + c*CS + i*L + 16b (piece i,
// byte-misaligned by i since L = 2^20 + 1). Piece i receives row sel[i]'s bytes: no tables, no GF
// arithmetic, no tile counter, no edge pass (the 17 tail columns per piece are not written).
// Launch geometries (`variant`), each a plain grid of 256-thread workgroups at full occupancy:
//   0  one block per thread, workgroup = 256 consecutive blocks of one chunkset (dispatch order)
//   1  as 0, workgroup tiles dealt to the XCDs in runs of 8 consecutive tiles (the decode's order)
//   2  two blocks per thread (tile of 512 blocks), dispatch order
//   3  one block per thread, the decode's occupancy: 3 workgroups per CU (LDS-limited), XCD runs
// bench.py loads tools/bin/libdecds_copypattern.so and times every variant on the headline's own plans
// and coded rows after the repaired bytes were checked (it overwrites the repaired output), and reports
// the fastest as roofline.decode.copy_pattern_GBps.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I decds_amd/csrc tools/copypattern.hip
//        -o tools/bin/libdecds_copypattern.so      (decds_amd/build.py build_copypattern)
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "rlnc_layout.h"

namespace copypattern {

using decds::CS;
using decds::K;
using decds::L;
using decds::MAIN_BLOCKS;
using decds::N;
using decds::RepairPlan;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t TILE_BLOCKS = 256;
constexpr uint32_t TILES = (MAIN_BLOCKS + TILE_BLOCKS - 1) / TILE_BLOCKS;  // 256 per chunkset

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, 0x80000000u, 0x00020000);
}

// workgroup -> global tile index; XCD: blocks b = 8R*grp + 8j + x -> tile 8R*grp + R*x + j (R = 8)
template <bool XCD>
__device__ __forceinline__ uint32_t tile_of() {
    const uint32_t b = blockIdx.x;
    if (!XCD) return b;
    constexpr uint32_t R = 8;
    const uint32_t grp = b / (8 * R), r = b % (8 * R);
    return grp * 8 * R + (r % 8) * R + r / 8;
}

template <uint32_t UNIT, bool XCD>
__global__ __launch_bounds__(256) void copy_pattern_kernel(const uint8_t *__restrict__ coded, size_t pitch, size_t n,
                                                           const RepairPlan *__restrict__ plan, uint8_t *__restrict__ out) {
    const uint32_t t = tile_of<XCD>(), tiles = TILES / UNIT + (TILES % UNIT != 0);
    const size_t cs = t / tiles;
    if (cs >= n) return;
    const RepairPlan &p = plan[cs];
    if (p.rank != K) return;
    const auto ri = rsrc(coded + cs * N * pitch);
    const auto ro = rsrc(out + cs * CS);
    uint32_t off[K];
#pragma unroll
    for (uint32_t k = 0; k < K; k++) off[k] = (uint32_t)(p.sel[k] * pitch) + K;
    const uint32_t b0 = (t % tiles) * UNIT * TILE_BLOCKS + threadIdx.x;
#pragma unroll
    for (uint32_t u = 0; u < UNIT; u++) {
        const uint32_t b = b0 + u * TILE_BLOCKS;
        const uint32_t col = b < MAIN_BLOCKS ? b * 16 : 0x80000000u;  // past the descriptor's range: dropped
        u32x4 x[K];
#pragma unroll
        for (uint32_t k = 0; k < K; k++) x[k] = __builtin_amdgcn_raw_buffer_load_b128(ri, off[k] + col, 0, 0);
#pragma unroll
        for (uint32_t i = 0; i < K; i++) {
            const uint32_t o = i * (uint32_t)L + col;
            if (i < K - 1 || col + 16 <= CS - (K - 1) * L)  // piece 9 ends 10 bytes short of L
                __builtin_amdgcn_raw_buffer_store_b128(x[i], ro, o, 0, 0);
        }
    }
}

}  // namespace copypattern

extern "C" {

// variant 0..3 (see the header); returns a hipError_t, 0 = launched
int decds_copy_pattern_decode(const uint8_t *coded, size_t pitch, size_t n, const void *plan, uint8_t *out, int variant,
                              void *stream) {
    using namespace copypattern;
    if (!coded || !plan || !out || n == 0 || pitch < decds::F || variant < 0 || variant > 3) return (int)hipErrorInvalidValue;
    if ((N - 1) * pitch + decds::F > 0x80000000ull) return (int)hipErrorInvalidValue;  // one descriptor per chunkset
    hipStream_t s = static_cast<hipStream_t>(stream);
    const RepairPlan *pl = static_cast<const RepairPlan *>(plan);
    const uint32_t unit = variant == 2 ? 2 : 1;
    const uint32_t tiles = TILES / unit + (TILES % unit != 0);
    uint64_t grid = (uint64_t)n * tiles;
    if (variant == 1 || variant == 3) grid = (grid + 63) / 64 * 64;  // whole XCD groups (extra tiles exit)
    if (grid > 0x7FFFFFFFull) return (int)hipErrorInvalidValue;
    const size_t lds = variant == 3 ? 52 * 1024 : 0;
    switch (variant) {
        case 0: hipLaunchKernelGGL((copy_pattern_kernel<1, false>), dim3((uint32_t)grid), dim3(256), lds, s, coded, pitch, n, pl, out); break;
        case 1: hipLaunchKernelGGL((copy_pattern_kernel<1, true>), dim3((uint32_t)grid), dim3(256), lds, s, coded, pitch, n, pl, out); break;
        case 2: hipLaunchKernelGGL((copy_pattern_kernel<2, false>), dim3((uint32_t)grid), dim3(256), lds, s, coded, pitch, n, pl, out); break;
        default: hipLaunchKernelGGL((copy_pattern_kernel<1, true>), dim3((uint32_t)grid), dim3(256), lds, s, coded, pitch, n, pl, out); break;
    }
    return (int)hipGetLastError();
}

const char *decds_copy_pattern_variant_name(int variant) {
    static const char *names[] = {"one block per thread, dispatch order", "one block per thread, XCD runs of 8 tiles",
                                  "two blocks per thread, dispatch order",
                                  "one block per thread, XCD runs of 8, 3 workgroups per CU (the decode's occupancy)"};
    return variant >= 0 && variant <= 3 ? names[variant] : "";
}

}  // extern "C"

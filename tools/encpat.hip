// encpat.hip — would line-aligned INPUT loads speed up the encode? The encode's memory pattern alone
// (per 16-column lane block: 10 input-row loads, 16 payload-aligned output-row stores; one-tile
// workgroups in dispatch order, 2 per CU like the sweep), with the 10 input pieces
//   mode 0  at i*L (L = 2^20 + 1: piece i misaligned by i bytes — the rlnc layout the encode reads),
//   mode 1  at i*2^20 (every load line-aligned; a timing-only layout),
//   mode 2  line-aligned loads at i*L - i plus, for the wave's last lane, its own misaligned load (the
//           memory operations of an in-register realignment: DPP wave_shl + v_alignbyte, not done here).
// Rounds interleave the modes in one process; GB/s counts the algorithmic bytes (10 MiB read +
// 16 x 1,048,587 written per chunkset).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/encpat.hip -o tools/bin/encpat
// Run:   tools/bin/encpat [chunksets=1639] [rounds=10]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint64_t CS = 10ull << 20, L = (CS + 10) / 10, F = L + 10, PITCH = 1048704;
constexpr uint32_t BLOCKS = 65535, TILES = 256, OOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, 0x80000000u, 0x00020000);
}

template <int MODE>
__global__ __launch_bounds__(256, 2) void encpat(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst) {
    const uint32_t cs = blockIdx.x / TILES, tile = blockIdx.x % TILES, lane = threadIdx.x & 63u;
    const uint32_t block = tile * 256 + threadIdx.x;
    const uint32_t col = block < BLOCKS ? block * 16 : OOB;
    const auto ri = rsrc(src + (size_t)cs * CS);
    const auto ro = rsrc(dst + (size_t)cs * 16 * PITCH);
    u32x4 x[10];
#pragma unroll
    for (uint32_t i = 0; i < 10; i++) {
        const uint32_t roff = MODE == 1 ? i << 20 : MODE == 2 ? (uint32_t)(i * L - i) : (uint32_t)(i * L);
        x[i] = __builtin_amdgcn_raw_buffer_load_b128(ri, roff + col, 0, 0);
        if constexpr (MODE == 2)  // the last lane's own bytes (its neighbour is in the next wave)
            x[i] ^= __builtin_amdgcn_raw_buffer_load_b128(ri, (uint32_t)(i * L) + (lane == 63 ? col : OOB), 0, 0);
    }
    u32x4 y = x[0];
#pragma unroll
    for (int i = 1; i < 10; i++) y ^= x[i];
#pragma unroll
    for (uint32_t j = 0; j < 16; j++) {  // payload j at 128-aligned (j * PITCH + 128 within a 128-aligned dst)
        y = y * 3u + j;
        __builtin_amdgcn_raw_buffer_store_b128(y, ro, (uint32_t)(j * PITCH + 128) + col, 0, 0);
    }
}

int main(int argc, char **argv) {
    const size_t n = argc > 1 ? std::strtoul(argv[1], nullptr, 10) : 1639;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 10;
    uint8_t *src, *dst;
    CK(hipMalloc(&src, n * CS + 64));
    CK(hipMalloc(&dst, n * 16 * PITCH + 256));
    CK(hipMemset(src, 0x5A, n * CS));
    void (*k[3])(const uint8_t *, uint8_t *) = {encpat<0>, encpat<1>, encpat<2>};
    const char *name[3] = {"inputs at i*L (rlnc, misaligned by i)", "inputs at i*2^20 (line-aligned)",
                           "aligned loads at i*L - i + the last lane's own load"};
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const dim3 grid((uint32_t)(n * TILES));
    for (int w = 0; w < 30; w++)
        for (int m = 0; m < 3; m++) hipLaunchKernelGGL(k[m], grid, dim3(256), 0, 0, src, dst);
    CK(hipDeviceSynchronize());
    std::vector<float> t[3];
    for (int r = 0; r < rounds; r++)
        for (int mm = 0; mm < 3; mm++) {
            const int m = (r & 1) ? 2 - mm : mm;
            CK(hipEventRecord(a, 0));
            hipLaunchKernelGGL(k[m], grid, dim3(256), 0, 0, src, dst);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            t[m].push_back(ms);
        }
    const double bytes = (double)n * (CS + 16 * F);
    for (int m = 0; m < 3; m++) {
        std::sort(t[m].begin(), t[m].end());
        const double med = t[m][t[m].size() / 2];
        std::printf("{\"mode\": %d, \"what\": \"%s\", \"n\": %zu, \"ms\": %.4f, \"GBps\": %.1f, \"frac_of_8TBps\": %.4f}\n", m,
                    name[m], n, med, bytes / (med * 1e-3) / 1e9, bytes / (med * 1e-3) / 8e12);
    }
    return 0;
}

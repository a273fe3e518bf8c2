// ldsconf.hip — LDS cost of the decode's table lookups: nibble tables (two conflict-free
// ds_read_b128 per input byte, the shipped form) against byte tables (one ds_read_b128 per input
// byte from a 256-row, 4 KiB table: rows r and r + 16k share a bank quad, so random bytes conflict
// within a 16-lane group) and 8-byte byte-table rows (ds_read_b64, 32-lane groups; only 8 of the
// decode's 10 outputs fit). VERDICT r03 item 3 asked for byte tables in the decode sweep; this
// measures the lookup cost alone, with random bytes, at the decode sweep's occupancy (3 waves/SIMD).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ldsconf.hip -o tools/bin/ldsconf
// Prints one JSON line per mode: LDS time per looked-up input byte per CU, and relative to nibble.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;  // input bytes looked up per lane
constexpr int WGS_PER_CU = 3;

// MODE 0: nibble tables (T_lo at 0, T_hi at 256: 16 rows x 16 B each), 2 x ds_read_b128 per byte
// MODE 1: byte table (256 rows x 16 B at 0), 1 x ds_read_b128 per byte
// MODE 2: byte table of 8-byte rows (256 x 8 B at 0), 1 x ds_read_b64 per byte
template <int MODE>
__global__ __launch_bounds__(256) void lookups(uint32_t seed, uint32_t *sink) {
    __shared__ __attribute__((aligned(16))) uint8_t t[4096];
    for (int i = threadIdx.x; i < 1024; i += 256) reinterpret_cast<uint32_t *>(t)[i] = i * 0x9E3779B1u;
    __syncthreads();
    uint32_t x = seed ^ (blockIdx.x * 256 + threadIdx.x) * 2654435761u;
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll 8
    for (int it = 0; it < ITERS; it++) {
        x = x * 1664525u + 1013904223u;  // one LCG step: the byte is bits 24..31
        const uint32_t b = x >> 24;
        if constexpr (MODE == 0) {
            const u32x4 lo = *reinterpret_cast<const u32x4 *>(t + (b & 15u) * 16);
            const u32x4 hi = *reinterpret_cast<const u32x4 *>(t + 256 + (b >> 4) * 16);
            acc ^= lo ^ hi;
        } else if constexpr (MODE == 1) {
            acc ^= *reinterpret_cast<const u32x4 *>(t + b * 16);
        } else {
            const u32x2 v = *reinterpret_cast<const u32x2 *>(t + b * 8);
            acc.x ^= v.x;
            acc.y ^= v.y;
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

template <int MODE>
static float run(int grid, uint32_t *sink) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 3; w++) hipLaunchKernelGGL(lookups<MODE>, dim3(grid), dim3(256), 0, 0, 7u + w, sink);
    CK(hipEventRecord(a, 0));
    const int reps = 10;
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(lookups<MODE>, dim3(grid), dim3(256), 0, 0, 99u + r, sink);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount, grid = cus * WGS_PER_CU;
    uint32_t *sink;
    CK(hipMalloc(&sink, 4));
    const double bytes = (double)grid * 256 * ITERS;  // input bytes looked up
    const float ms[3] = {run<0>(grid, sink), run<1>(grid, sink), run<2>(grid, sink)};
    const char *name[3] = {"nibble tables, 2 x ds_read_b128 per byte", "byte table, 1 x ds_read_b128 per byte",
                           "byte table 8-B rows, 1 x ds_read_b64 per byte"};
    for (int m = 0; m < 3; m++)
        std::printf("{\"mode\": \"%s\", \"ms\": %.4f, \"G_bytes_per_s\": %.1f, \"vs_nibble\": %.3f, \"cus\": %d, "
                    "\"wgs_per_cu\": %d}\n",
                    name[m], ms[m], bytes / (ms[m] * 1e-3) / 1e9, ms[m] / ms[0], cus, WGS_PER_CU);
    return 0;
}

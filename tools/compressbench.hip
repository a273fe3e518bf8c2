// compressbench.hip — BLAKE3 compressions per second on gfx950 with the message in registers (no
// memory in the loop), at a chosen occupancy: the issue-rate floor of the digest and fused kernels.
// One lane = one chain of ITERS compressions (each compression's output feeds the next one's cv).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Idecds_amd/csrc tools/compressbench.hip -o build/compressbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "blake3_impl.h"

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

constexpr int ITERS = 256;

template <int WAVES, int CHAINS>
__global__ __launch_bounds__(256, WAVES) __attribute__((amdgpu_waves_per_eu(WAVES, WAVES))) void compress_kernel(uint32_t *out) {
    uint32_t cv[CHAINS][8], m[16];
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = threadIdx.x * 16 + i + blockIdx.x;
#pragma unroll
    for (int c = 0; c < CHAINS; c++)
#pragma unroll
        for (int i = 0; i < 8; i++) cv[c][i] = decds::b3::K3.iv[i] + c;
#pragma unroll 1
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) decds::b3::compress(cv[c], m, it, 64, 0, cv[c]);
        m[it & 15] ^= cv[0][it & 7];
    }
    uint32_t x = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; c++)
#pragma unroll
        for (int i = 0; i < 8; i++) x ^= cv[c][i];
    out[blockIdx.x * 256 + threadIdx.x] = x;
}

template <int WAVES, int CHAINS>
void run(int cus, uint32_t *out) {
    const int blocks = cus * WAVES;  // 4 waves per block = one per SIMD
    auto launch = [&] { compress_kernel<WAVES, CHAINS><<<blocks, 256>>>(out); };
    launch();
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
        CK(hipEventRecord(a));
        launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
    }
    const double comps = (double)blocks * 256 * ITERS * CHAINS;
    std::printf("{\"waves_per_simd\": %d, \"chains_per_lane\": %d, \"ms\": %.4f, \"G_compressions_per_s\": %.1f, "
                "\"ns_per_wave_compression_per_simd\": %.1f}\n",
                WAVES, CHAINS, best, comps / best / 1e6, best * 1e6 / (comps / 64 / (cus * 4)));
}

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    uint32_t *out;
    CK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
    run<1, 1>(cus, out);
    run<2, 1>(cus, out);
    run<3, 1>(cus, out);
    run<4, 1>(cus, out);
    run<6, 1>(cus, out);
    run<8, 1>(cus, out);
    run<1, 2>(cus, out);
    run<2, 2>(cus, out);
    run<3, 2>(cus, out);
    run<4, 2>(cus, out);
    CK(hipFree(out));
    return 0;
}

// membench.hip — the encode kernel's memory pattern alone (10 row loads + 16 row stores per
// 16-column lane block, same tiling and grid), with the row geometry as run-time parameters, so
// the rlnc layout (rows misaligned by i*L and r*F + 10) and 16-byte-aligned geometries can be
// timed in ONE process, rounds interleaved, on random data.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/membench.hip -o build/membench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../decds_amd/csrc/rlnc_kernels.hip"

using namespace decds;

struct Geom {
    const char *name;
    uint64_t istride, cstride, ostride, opoff;
};

template <bool LOAD, bool STORE>
__global__ __launch_bounds__(WG, WAVES_PER_SIMD) void pattern_kernel(const uint8_t *__restrict__ src, size_t n,
                                                                   uint8_t *__restrict__ dst, Geom g,
                                                                   uint4 *__restrict__ sink) {
    uint32_t t0, t1;
    tile_range<500>(n, t0, t1);
    uint32_t ioff[K], ooff[N];
#pragma unroll
    for (int i = 0; i < (int)K; i++) ioff[i] = (uint32_t)(i * g.istride);
#pragma unroll
    for (int j = 0; j < (int)N; j++) ooff[j] = (uint32_t)(j * g.ostride + g.opoff);
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (uint32_t t = t0; t < t1; t++) {
        const uint32_t cs = t / TILES_PER_CS, tile = t % TILES_PER_CS;
        const uint8_t *ibase = src + (size_t)cs * g.cstride;
        uint8_t *obase = dst + (size_t)cs * N * g.ostride;
        const uint32_t block = tile * TILE_BLOCKS + threadIdx.x;
        if (block >= MAIN_BLOCKS) continue;
        const uint32_t col0 = block * COLS_PER_LANE;
        uint4 x[K];
        if constexpr (LOAD) {
            load_block<EncTune, K>(x, ibase, ioff, col0);
        } else {
#pragma unroll
            for (int i = 0; i < (int)K; i++) x[i] = make_uint4(t, i, block, 7);
        }
        if constexpr (STORE) {
#pragma unroll
            for (int j = 0; j < (int)N; j++) {
                const uint4 a = x[j % K], b = x[(j + 3) % K];
                strow<-1>(obase, ooff[j] + col0, make_uint4(a.x ^ b.y, a.y ^ b.z, a.z ^ b.w, a.w ^ b.x));
            }
        } else {
#pragma unroll
            for (int i = 0; i < (int)K; i++) acc = make_uint4(acc.x ^ x[i].x, acc.y ^ x[i].y, acc.z ^ x[i].z, acc.w ^ x[i].w);
        }
    }
    if constexpr (!STORE) sink[blockIdx.x * WG + threadIdx.x] = acc;
}

// per tile a wave covers M consecutive KiB of every row (instruction m: bytes [m KiB, (m+1) KiB));
// tiles shrink in count by M. Timing-only: addresses as in the rlnc geometry.
template <int M>
__global__ __launch_bounds__(WG, WAVES_PER_SIMD) void pattern_m_kernel(const uint8_t *__restrict__ src, size_t n,
                                                                     uint8_t *__restrict__ dst, Geom g) {
    constexpr uint32_t TPC = TILES_PER_CS / M;
    const uint64_t total = (uint64_t)n * TPC;
    const uint32_t t0 = (uint32_t)(total * blockIdx.x / gridDim.x), t1 = (uint32_t)(total * (blockIdx.x + 1) / gridDim.x);
    uint32_t ioff[K], ooff[N];
#pragma unroll
    for (int i = 0; i < (int)K; i++) ioff[i] = (uint32_t)(i * g.istride);
#pragma unroll
    for (int j = 0; j < (int)N; j++) ooff[j] = (uint32_t)(j * g.ostride + g.opoff);
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (uint32_t t = t0; t < t1; t++) {
        const uint32_t cs = t / TPC, tile = t % TPC;
        const uint8_t *ibase = src + (size_t)cs * g.cstride;
        uint8_t *obase = dst + (size_t)cs * N * g.ostride;
#pragma unroll
        for (int m = 0; m < M; m++) {
            const uint32_t block = (tile * 4 + wave) * 64 * M + m * 64 + lane;
            if (block >= MAIN_BLOCKS) continue;
            const uint32_t col0 = block * COLS_PER_LANE;
            uint4 x[K];
            load_block<EncTune, K>(x, ibase, ioff, col0);
#pragma unroll
            for (int j = 0; j < (int)N; j++) {
                const uint4 a = x[j % K], b = x[(j + 3) % K];
                strow<-1>(obase, ooff[j] + col0, make_uint4(a.x ^ b.y, a.y ^ b.z, a.z ^ b.w, a.w ^ b.x));
            }
        }
    }
}

// outputs written NP rows at a time: per tile, 16/NP passes each re-loading the 10 input rows
// (the re-loads hit L2) and storing NP output rows -> fewer concurrent write streams per wave
template <int NP>
__global__ __launch_bounds__(WG, WAVES_PER_SIMD) void pattern_np_kernel(const uint8_t *__restrict__ src, size_t n,
                                                                      uint8_t *__restrict__ dst, Geom g) {
    uint32_t t0, t1;
    tile_range<500>(n, t0, t1);
    uint32_t ioff[K], ooff[N];
#pragma unroll
    for (int i = 0; i < (int)K; i++) ioff[i] = (uint32_t)(i * g.istride);
#pragma unroll
    for (int j = 0; j < (int)N; j++) ooff[j] = (uint32_t)(j * g.ostride + g.opoff);
    for (uint32_t t = t0; t < t1; t++) {
        const uint32_t cs = t / TILES_PER_CS, tile = t % TILES_PER_CS;
        const uint8_t *ibase = src + (size_t)cs * g.cstride;
        uint8_t *obase = dst + (size_t)cs * N * g.ostride;
        const uint32_t block = tile * TILE_BLOCKS + threadIdx.x;
        if (block >= MAIN_BLOCKS) continue;
        const uint32_t col0 = block * COLS_PER_LANE;
#pragma unroll
        for (int ps = 0; ps < (int)N / NP; ps++) {
            uint4 x[K];
            load_block<EncTune, K>(x, ibase, ioff, col0);
#pragma unroll
            for (int jj = 0; jj < NP; jj++) {
                const int j = ps * NP + jj;
                const uint4 a = x[j % K], b = x[(j + 3) % K];
                strow<-1>(obase, ooff[j] + col0, make_uint4(a.x ^ b.y, a.y ^ b.z, a.z ^ b.w, a.w ^ b.x));
            }
            __builtin_amdgcn_s_waitcnt(0);  // keep the passes apart
        }
    }
}

__global__ void random_fill(uint64_t *p, size_t nw) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

int main(int argc, char **argv) {
    const size_t n = argc > 1 ? strtoul(argv[1], nullptr, 10) : 1200;
    const int rounds = argc > 2 ? atoi(argv[2]) : 8;
    const uint64_t LA = 1048592;  // L rounded up to 16
    std::vector<Geom> geoms = {
        {"rlnc", L, CS, F, K},
        {"aligned_out", L, CS, LA + 16, 16},
        {"aligned_in", LA, 10 * LA, F, K},
        {"aligned_all", LA, 10 * LA, LA + 16, 16},
    };
    const size_t src_bytes = n * 10 * LA + 64, dst_bytes = n * N * (LA + 16) + 64;
    uint8_t *src, *dst;
    uint4 *sink;
    if (hipMalloc(&src, src_bytes) || hipMalloc(&dst, dst_bytes) || hipMalloc(&sink, 1024 * WG * sizeof(uint4))) {
        printf("alloc failed\n");
        return 1;
    }
    hipLaunchKernelGGL(random_fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t *>(src), src_bytes / 8);
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    LaunchGeom lg{prop.multiProcessorCount};
    const uint32_t grid = stream_grid(lg, n);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    struct Case {
        const char *kind;
        int g;
        std::vector<float> ms;
    };
    std::vector<Case> cases;
    for (int gi = 0; gi < (int)geoms.size(); gi++)
        for (const char *k : {"load+store", "store", "load"}) cases.push_back({k, gi, {}});
    for (const char *k : {"m2", "np4", "np8"}) cases.push_back({k, 0, {}});
    auto launch = [&](const Case &c) {
        const Geom &g = geoms[c.g];
        if (c.kind[0] == 'n' && c.kind[2] == '4')
            hipLaunchKernelGGL((pattern_np_kernel<4>), dim3(grid), dim3(WG), 0, 0, src, n, dst, g);
        else if (c.kind[0] == 'n')
            hipLaunchKernelGGL((pattern_np_kernel<8>), dim3(grid), dim3(WG), 0, 0, src, n, dst, g);
        else if (c.kind[0] == 'm' && c.kind[1] == '2')
            hipLaunchKernelGGL((pattern_m_kernel<2>), dim3(grid), dim3(WG), 0, 0, src, n, dst, g);
        else if (c.kind[0] == 'm')
            hipLaunchKernelGGL((pattern_m_kernel<4>), dim3(grid), dim3(WG), 0, 0, src, n, dst, g);
        else if (c.kind[0] == 'l' && c.kind[4] == '+')
            hipLaunchKernelGGL((pattern_kernel<true, true>), dim3(grid), dim3(WG), 0, 0, src, n, dst, g, sink);
        else if (c.kind[0] == 's')
            hipLaunchKernelGGL((pattern_kernel<false, true>), dim3(grid), dim3(WG), 0, 0, src, n, dst, g, sink);
        else
            hipLaunchKernelGGL((pattern_kernel<true, false>), dim3(grid), dim3(WG), 0, 0, src, n, dst, g, sink);
    };
    for (auto &c : cases) launch(c);  // warm
    hipDeviceSynchronize();
    for (int r = 0; r < rounds; r++) {
        for (size_t ci = 0; ci < cases.size(); ci++) {
            Case &c = cases[r % 2 ? cases.size() - 1 - ci : ci];
            hipEventRecord(a);
            launch(c);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            c.ms.push_back(ms);
        }
    }
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("kernel error\n");
        return 1;
    }
    for (auto &c : cases) {
        std::sort(c.ms.begin(), c.ms.end());
        const double med = c.ms[c.ms.size() / 2];
        const double rd = (double)n * CS, wr = (double)n * N * F;
        const double bytes = (c.kind[0] == 'm' || c.kind[0] == 'n' || c.kind[4] == '+') ? rd + wr : c.kind[0] == 's' ? wr : rd;
        printf("{\"geom\": \"%s\", \"kind\": \"%s\", \"n\": %zu, \"ms\": %.4f, \"GBps\": %.1f}\n", geoms[c.g].name,
               c.kind, n, med, bytes / med / 1e6);
    }
    return 0;
}

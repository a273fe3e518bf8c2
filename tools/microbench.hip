// microbench.hip — ceilings for the encode kernel's two halves on gfx950, same grid and tiling:
//   mem_only : the 10 row loads + 16 row stores per lane block of the encode kernel (rlnc layout,
//              unaligned), compute replaced by a byte shuffle that keeps every load live
//   lds_only : the 320 ds_read_b128 table lookups + XOR/transpose per lane block, inputs
//              synthesised in registers, one store per lane at the end
//   encode   : the shipped encode kernel
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I decds_amd/csrc tools/microbench.hip -o build/microbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../decds_amd/csrc/rlnc_kernels.hip"

using namespace decds;

__global__ __launch_bounds__(WG, WAVES_PER_SIMD) void mem_only_kernel(const uint8_t *__restrict__ src, size_t n,
                                                                         uint8_t *__restrict__ dst, size_t pitch) {
    uint32_t t0, t1;
    tile_range(n, t0, t1);
    uint32_t ioff[K], ooff[N];
#pragma unroll
    for (int i = 0; i < (int)K; i++) ioff[i] = (uint32_t)(i * L);
#pragma unroll
    for (int j = 0; j < (int)N; j++) ooff[j] = (uint32_t)(j * pitch + K);
    for (uint32_t t = t0; t < t1; t++) {
        const uint32_t cs = t / TILES_PER_CS, tile = t % TILES_PER_CS;
        const uint8_t *ibase = src + (size_t)cs * CS;
        uint8_t *obase = dst + (size_t)cs * N * pitch;
        const uint32_t block = tile * TILE_BLOCKS + threadIdx.x;
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

// same traffic, work items (chunkset, phase w < wpc) dealt round-robin to the resident workgroups:
// the WGs in flight sweep neighbouring tiles of the same few chunksets
__global__ __launch_bounds__(WG, WAVES_PER_SIMD) void mem_items_kernel(const uint8_t *__restrict__ src, size_t n,
                                                                          uint8_t *__restrict__ dst, size_t pitch,
                                                                          uint32_t wpc) {
    uint32_t ioff[K], ooff[N];
#pragma unroll
    for (int i = 0; i < (int)K; i++) ioff[i] = (uint32_t)(i * L);
#pragma unroll
    for (int j = 0; j < (int)N; j++) ooff[j] = (uint32_t)(j * pitch + K);
    const uint32_t items = (uint32_t)n * wpc;
    for (uint32_t it = blockIdx.x; it < items; it += gridDim.x) {
        const uint32_t cs = it / wpc, w = it % wpc;
        const uint8_t *ibase = src + (size_t)cs * CS;
        uint8_t *obase = dst + (size_t)cs * N * pitch;
        for (uint32_t tile = w; tile < TILES_PER_CS; tile += wpc) {
            const uint32_t block = tile * TILE_BLOCKS + threadIdx.x;
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

// read side only: the 10 row loads per lane block, folded into one store per lane at the end
__global__ __launch_bounds__(WG, WAVES_PER_SIMD) void load_only_kernel(const uint8_t *__restrict__ src, size_t n,
                                                                          uint8_t *__restrict__ sink) {
    uint32_t t0, t1;
    tile_range(n, t0, t1);
    uint32_t ioff[K];
#pragma unroll
    for (int i = 0; i < (int)K; i++) ioff[i] = (uint32_t)(i * L);
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (uint32_t t = t0; t < t1; t++) {
        const uint32_t cs = t / TILES_PER_CS, tile = t % TILES_PER_CS;
        const uint32_t block = tile * TILE_BLOCKS + threadIdx.x;
        if (block >= MAIN_BLOCKS) continue;
        uint4 x[K];
        load_block<EncTune, K>(x, src + (size_t)cs * CS, ioff, block * COLS_PER_LANE);
#pragma unroll
        for (int i = 0; i < (int)K; i++) acc = make_uint4(acc.x ^ x[i].x, acc.y ^ x[i].y, acc.z ^ x[i].z, acc.w ^ x[i].w);
    }
    reinterpret_cast<uint4 *>(sink)[blockIdx.x * WG + threadIdx.x] = acc;
}

// write side only: the 16 row stores per lane block
__global__ __launch_bounds__(WG, WAVES_PER_SIMD) void store_only_kernel(size_t n, uint8_t *__restrict__ dst,
                                                                           size_t pitch) {
    uint32_t t0, t1;
    tile_range(n, t0, t1);
    uint32_t ooff[N];
#pragma unroll
    for (int j = 0; j < (int)N; j++) ooff[j] = (uint32_t)(j * pitch + K);
    for (uint32_t t = t0; t < t1; t++) {
        const uint32_t cs = t / TILES_PER_CS, tile = t % TILES_PER_CS;
        const uint32_t block = tile * TILE_BLOCKS + threadIdx.x;
        if (block >= MAIN_BLOCKS) continue;
        uint8_t *obase = dst + (size_t)cs * N * pitch;
#pragma unroll
        for (int j = 0; j < (int)N; j++) strow<-1>(obase, ooff[j] + block * COLS_PER_LANE, make_uint4(t, j, block, 7));
    }
}

// plain float4-style copy of the same byte count (src -> dst, grid-stride): the HBM reference
__global__ void copy_kernel(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n16) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// copy with 4 independent 16-B loads in flight per lane
__global__ __launch_bounds__(256) void copy4_kernel(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
        dst[i] = a;
        dst[i + stride] = b;
        dst[i + 2 * stride] = c;
        dst[i + 3 * stride] = d;
    }
    for (; i < n16; i += stride) dst[i] = src[i];
}

// write-only streaming of the same byte count into one contiguous buffer
__global__ __launch_bounds__(256) void fill_kernel(uint4 *__restrict__ dst, size_t n16) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

__global__ __launch_bounds__(WG, WAVES_PER_SIMD) void lds_only_kernel(size_t n, const uint8_t *__restrict__ coeffs,
                                                                         uint8_t *__restrict__ sink, uint32_t poly) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint32_t t0, t1;
    tile_range(n, t0, t1);
    const uint32_t laneoff = (threadIdx.x & 15u) * 16u;
    build_tables<K, N>(lds, coeffs, K, poly);
    __syncthreads();
    uint4 x[K];
#pragma unroll
    for (int i = 0; i < (int)K; i++) x[i] = make_uint4(threadIdx.x * 0x01010101u + i, i * 77u, threadIdx.x, i ^ 0x5a5a5a5au);
    // outputs go to a per-lane scratch row so the stores stay cheap and cached
    uint32_t ooff[N];
#pragma unroll
    for (int j = 0; j < (int)N; j++) ooff[j] = j * 16u;
    uint32_t ioff[K] = {};
    uint8_t *obase = sink + (size_t)(blockIdx.x * WG + threadIdx.x) * 256;
    for (uint32_t t = t0; t < t1; t++) {
        combine_block<EncTune, K, N>(lds, laneoff, x, obase, ooff, 0, nullptr, ioff, 0);
#pragma unroll
        for (int i = 0; i < (int)K; i++) x[i].x += t;
    }
}

int main(int argc, char **argv) {
    const size_t n = argc > 1 ? strtoul(argv[1], nullptr, 10) : 1639;
    const int reps = 10;
    uint8_t *src, *dst, *cv, *sink;
    const size_t pitch = F;
    if (hipMalloc(&src, n * CS + 64) || hipMalloc(&dst, n * N * pitch + 64) || hipMalloc(&cv, n * N * K) ||
        hipMalloc(&sink, (size_t)256 * 2 * WG * 256)) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(src, 0x5b, n * CS);
    hipMemset(cv, 0x37, n * N * K);
    configure_kernels();
    hipFuncSetAttribute(reinterpret_cast<const void *>(lds_only_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                        LDS_BYTES);
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    LaunchGeom g{prop.multiProcessorCount};
    const uint32_t grid = stream_grid(g, n);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const double bytes = (double)n * (CS + N * F);
    auto timeit_b = [&](const char *name, double nbytes, auto launch) {
        for (int w = 0; w < 2; w++) launch();
        hipEventRecord(a);
        for (int r = 0; r < reps; r++) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        ms /= reps;
        printf("{\"kernel\": \"%s\", \"n\": %zu, \"ms\": %.4f, \"GBps_equiv\": %.1f, \"wg\": %u, \"prefetch\": %d}\n", name, n,
               ms, nbytes / ms / 1e6, WG, 0);
    };
    auto timeit = [&](const char *name, auto launch) { timeit_b(name, bytes, launch); };
    timeit("mem_only", [&] { hipLaunchKernelGGL(mem_only_kernel, dim3(grid), dim3(WG), 0, 0, src, n, dst, pitch); });
    timeit_b("load_only", (double)n * CS, [&] { hipLaunchKernelGGL(load_only_kernel, dim3(grid), dim3(WG), 0, 0, src, n, sink); });
    timeit_b("store_only", (double)n * N * F, [&] { hipLaunchKernelGGL(store_only_kernel, dim3(grid), dim3(WG), 0, 0, n, dst, pitch); });
    for (uint32_t wpc : {32u}) {
        char name[64];
        snprintf(name, sizeof name, "mem_items_wpc%u", wpc);
        timeit(name, [&] { hipLaunchKernelGGL(mem_items_kernel, dim3(grid), dim3(WG), 0, 0, src, n, dst, pitch, wpc); });
    }
    {
        // plain copy of the whole src buffer into dst (both hold >= n*CS bytes)
        const size_t n16 = (size_t)n * CS / 16;
        timeit_b("copy", 2.0 * n16 * 16, [&] {
            hipLaunchKernelGGL(copy_kernel, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const uint4 *>(src),
                               reinterpret_cast<uint4 *>(dst), n16);
        });
    }
    {
        const size_t n16 = (size_t)n * CS / 16;
        for (uint32_t gsz : {1024u, 2048u, 8192u}) {
            char name[64];
            snprintf(name, sizeof name, "copy4_grid%u", gsz);
            timeit_b(name, 2.0 * n16 * 16, [&] {
                hipLaunchKernelGGL(copy4_kernel, dim3(gsz), dim3(256), 0, 0, reinterpret_cast<const uint4 *>(src),
                                   reinterpret_cast<uint4 *>(dst), n16);
            });
        }
        const size_t w16 = (size_t)n * N * F / 16;
        timeit_b("fill_contig", 16.0 * w16, [&] {
            hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint4 *>(dst), w16);
        });
    }
    timeit("lds_only", [&] {
        hipLaunchKernelGGL(lds_only_kernel, dim3(grid), dim3(WG), LDS_BYTES, 0, n, cv, sink, 0x11Du);
    });
    timeit("encode", [&] { launch_encode(g, src, n, cv, dst, pitch, 0x11D, 0x81, 0); });
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        printf("error %s\n", hipGetErrorString(e));
        return 1;
    }
    return 0;
}

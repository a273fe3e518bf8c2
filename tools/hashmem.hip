// hashmem.hip — the memory side of the chunk-digest kernel alone: every lane owns one 1 KiB
// BLAKE3 chunk of a 1.73 GB buffer (1648 coded rows) and reads it in segments of S bytes per step
// (S/16 back-to-back dwordx4 loads, then an xor fold), so the DRAM cost of the chunk-parallel
// access order can be priced per segment size against a plain coalesced stream of the same bytes.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/hashmem.hip -o build/hashmem
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

constexpr size_t CHUNK = 1024;

// lane = chunk; S bytes per step
template <int S>
__global__ __launch_bounds__(256) void seg_kernel(const uint8_t *__restrict__ buf, size_t nchunks,
                                                  uint4 *__restrict__ sink, int mis) {
    const size_t c = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= nchunks) return;
    const uint4 *p = reinterpret_cast<const uint4 *>(buf + c * CHUNK + mis);
    uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll 1
    for (int s = 0; s < (int)CHUNK / S; s++) {
        uint4 v[S / 16];
#pragma unroll
        for (int i = 0; i < S / 16; i++) v[i] = p[s * (S / 16) + i];
#pragma unroll
        for (int i = 0; i < S / 16; i++) acc = make_uint4(acc.x ^ v[i].x, acc.y + v[i].y, acc.z ^ v[i].z, acc.w + v[i].w);
    }
    sink[c] = acc;
}

// same bytes, coalesced: wave instruction i reads 1 KiB contiguous
__global__ __launch_bounds__(256) void stream_kernel(const uint8_t *__restrict__ buf, size_t nchunks,
                                                     uint4 *__restrict__ sink) {
    const size_t c = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= nchunks) return;
    const size_t wave0 = c & ~(size_t)63;
    const uint4 *p = reinterpret_cast<const uint4 *>(buf + wave0 * CHUNK) + (threadIdx.x & 63);
    uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll 4
    for (int i = 0; i < 64; i++) {
        const uint4 v = p[i * 64];
        acc = make_uint4(acc.x ^ v.x, acc.y + v.y, acc.z ^ v.z, acc.w + v.w);
    }
    sink[c] = acc;
}

template <typename F>
float timeit(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> t;
    for (int r = 0; r < reps + 2; r++) {
        CK(hipEventRecord(a));
        f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r >= 2) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    const size_t rows = 1648, nchunks = rows * 1024, bytes = nchunks * CHUNK;
    uint8_t *buf;
    uint4 *sink;
    CK(hipMalloc(&buf, bytes + 64));
    CK(hipMalloc(&sink, nchunks * sizeof(uint4)));
    CK(hipMemset(buf, 0x5a, bytes + 64));
    const dim3 grid((unsigned)((nchunks + 255) / 256)), wg(256);
    auto report = [&](const char *name, float ms) {
        std::printf("{\"pattern\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms, bytes / ms / 1e6);
    };
    report("stream", timeit([&] { stream_kernel<<<grid, wg>>>(buf, nchunks, sink); }, 10));
    for (int mis : {0, 4, 11}) {
        char nm[64];
#define SEG(S)                                                                                    \
        std::snprintf(nm, sizeof nm, "seg%d_mis%d", S, mis);                                      \
        report(nm, timeit([&] { seg_kernel<S><<<grid, wg>>>(buf, nchunks, sink, mis); }, 10));
        SEG(64) SEG(128) SEG(256)
    }
    CK(hipDeviceSynchronize());
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}

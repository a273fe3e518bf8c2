// copybench.hip — the chip's streaming ceilings on the box at hand: read-only, write-only and
// copy over 1 GiB, with 1 or 4 16-byte accesses in flight per lane, plain or non-temporal, and
// a copy whose lanes stream R rows at once (the codec kernels read 10 / write 16 or 10 rows per
// lane block). Prints one JSON line per variant (GB/s counts bytes read + bytes written).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/copybench.hip -o build/copybench
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

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_k(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, size_t n16) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t k = i + u * stride;
            if (k < n16) v[u] = NT ? __builtin_nontemporal_load(s + k) : s[k];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t k = i + u * stride;
            if (k < n16) {
                if (NT)
                    __builtin_nontemporal_store(v[u], d + k);
                else
                    d[k] = v[u];
            }
        }
    }
}

template <int U>
__global__ __launch_bounds__(256) void read_k(const u32x4 *__restrict__ s, size_t n16, u32x4 *__restrict__ sink) {
    const size_t stride = (size_t)gridDim.x * 256;
    u32x4 acc = {0, 0, 0, 0};
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride * U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t k = i + u * stride;
            if (k < n16) acc ^= s[k];
        }
    }
    if (acc.x == 0x12345678u) sink[0] = acc;
}

template <int U>
__global__ __launch_bounds__(256) void write_k(u32x4 *__restrict__ d, size_t n16) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride * U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t k = i + u * stride;
            if (k < n16) d[k] = u32x4{(uint32_t)k, 1u, 2u, 3u};
        }
    }
}

// R rows of `rowlen` 16-B words each: the workgroup's lanes walk column blocks of all R rows at
// once (R loads then R stores per lane), like the codec kernels' row streams
template <int R>
__global__ __launch_bounds__(256) void rows_k(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, size_t rowlen,
                                              size_t nsets) {
    const size_t cols = nsets * rowlen;  // (set, column) pairs
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < cols; i += (size_t)gridDim.x * 256) {
        const size_t set = i / rowlen, col = i % rowlen;
        const u32x4 *sp = s + set * R * rowlen + col;
        u32x4 *dp = d + set * R * rowlen + col;
        u32x4 v[R];
#pragma unroll
        for (int r = 0; r < R; r++) v[r] = sp[r * rowlen];
#pragma unroll
        for (int r = 0; r < R; r++) dp[r * rowlen] = v[r];
    }
}

template <typename F>
float timeit(F f, int reps = 10) {
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
    const size_t bytes = (size_t)1 << 30, n16 = bytes / 16;
    u32x4 *s, *d, *sink;
    CK(hipMalloc(&s, bytes));
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(s, 0x3c, bytes));
    CK(hipMemset(d, 0, bytes));
    auto rep = [&](const char *name, int grid, double moved, float ms) {
        std::printf("{\"variant\": \"%s\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", name, grid, ms, moved / ms / 1e6);
    };
    for (int grid : {2048, 8192, 32768}) {
        rep("read_u1", grid, bytes, timeit([&] { read_k<1><<<grid, 256>>>(s, n16, sink); }));
        rep("read_u4", grid, bytes, timeit([&] { read_k<4><<<grid, 256>>>(s, n16, sink); }));
        rep("write_u1", grid, bytes, timeit([&] { write_k<1><<<grid, 256>>>(d, n16); }));
        rep("write_u4", grid, bytes, timeit([&] { write_k<4><<<grid, 256>>>(d, n16); }));
        rep("copy_u1", grid, 2.0 * bytes, timeit([&] { copy_k<1, false><<<grid, 256>>>(s, d, n16); }));
        rep("copy_u4", grid, 2.0 * bytes, timeit([&] { copy_k<4, false><<<grid, 256>>>(s, d, n16); }));
        rep("copy_u4_nt", grid, 2.0 * bytes, timeit([&] { copy_k<4, true><<<grid, 256>>>(s, d, n16); }));
    }
    // row-stream copies: rows of 1 MiB (65536 words), sets of R rows
    const size_t rowlen = 65536;
    for (int grid : {2048, 8192}) {
        rep("rows10_copy", grid, 2.0 * (bytes / (10 * rowlen * 16)) * 10 * rowlen * 16,
            timeit([&] { rows_k<10><<<grid, 256>>>(s, d, rowlen, bytes / (10 * rowlen * 16)); }));
        rep("rows16_copy", grid, 2.0 * (bytes / (16 * rowlen * 16)) * 16 * rowlen * 16,
            timeit([&] { rows_k<16><<<grid, 256>>>(s, d, rowlen, bytes / (16 * rowlen * 16)); }));
        rep("rows1_copy", grid, 2.0 * bytes, timeit([&] { rows_k<1><<<grid, 256>>>(s, d, rowlen, bytes / (rowlen * 16)); }));
    }
    CK(hipDeviceSynchronize());
    return 0;
}

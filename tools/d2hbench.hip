// d2hbench.hip — how fast device → page-locked host copies run, and with which engine: the host blob
// encode path (decds_blob_encode_host) is bound by its D2H of 1.6 coded bytes per blob byte, and a
// rocprofv3 trace of it (r07b) showed those hipMemcpyAsync copies executed as runtime blit kernels
// (__amd_rocclr_copyBuffer, 8 MiB each) with gaps as long as the kernels between them while an H2D
// ran on another stream. Variants, each over BYTES (default 270 MB = one 16-chunkset batch of coded
// rows), median of REPS:
//   memcpy      hipMemcpyAsync D2H alone
//   kernel      a grid-stride copy kernel storing straight into the host buffer (16 B per lane, W
//               workgroups), alone
//   memcpy+h2d  the hipMemcpyAsync D2H beside an H2D hipMemcpyAsync of the same size on another stream
//   kernel+h2d  the kernel D2H beside the same H2D
//   h2dkernel   the reverse direction by kernel: the copy kernel loading from the host buffer into device
//               memory (a gather of host rows without per-run hipMemcpyAsync calls), alone
//   h2dkernel+d2h  that kernel beside a hipMemcpyAsync D2H of the same size on another stream
// With a fifth argument "sizes": only hipMemcpyAsync D2H alone at 1, 4, 16, 64 MiB and BYTES, in one process.
// Prints one JSON line per variant (GB/s of the D2H; the H2D's own rate beside it; for the h2dkernel
// variants the kernel's H2D rate, and the D2H's beside it).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/d2hbench.hip -o tools/bin/d2hbench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

__global__ __launch_bounds__(256) void d2h_k(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, size_t n16) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) d[i] = s[i];
}

static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char **argv) {
    const size_t bytes = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (size_t)270 << 20;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 7;
    const int wgs = argc > 3 ? std::atoi(argv[3]) : 128;
    // host memory kind: 0 hipHostMalloc default (coherent), 1 hipHostMallocNonCoherent (the library's),
    // 2 malloc + hipHostRegister (a caller's decds_host_register)
    const int kind = argc > 4 ? std::atoi(argv[4]) : 0;
    const size_t n16 = bytes / 16;
    void *dsrc, *ddst, *hsrc, *hdst;
    CK(hipMalloc(&dsrc, bytes));
    CK(hipMalloc(&ddst, bytes));
    void *hdst_dev = nullptr;
    if (kind == 2) {
        hsrc = std::aligned_alloc(4096, bytes);
        hdst = std::aligned_alloc(4096, bytes);
        CK(hipHostRegister(hsrc, bytes, hipHostRegisterDefault));
        CK(hipHostRegister(hdst, bytes, hipHostRegisterDefault));
    } else {
        const unsigned fl = kind == 1 ? hipHostMallocNonCoherent : hipHostMallocDefault;
        CK(hipHostMalloc(&hsrc, bytes, fl));
        CK(hipHostMalloc(&hdst, bytes, fl));
    }
    CK(hipHostGetDevicePointer(&hdst_dev, hdst, 0));
    std::memset(hsrc, 1, bytes);
    std::memset(hdst, 0, bytes);
    CK(hipMemset(dsrc, 7, bytes));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t a1, b1, a2, b2;
    for (hipEvent_t *e : {&a1, &b1, &a2, &b2}) CK(hipEventCreate(e));
    void *hsrc_dev = nullptr;
    CK(hipHostGetDevicePointer(&hsrc_dev, hsrc, 0));
    if (argc > 5 && !std::strcmp(argv[5], "sizes")) {  // hipMemcpyAsync D2H alone at 1 MiB ... BYTES, one process
        for (size_t sz : {(size_t)1 << 20, (size_t)4 << 20, (size_t)16 << 20, (size_t)64 << 20, bytes}) {
            if (sz > bytes) continue;
            std::vector<double> ms;
            for (int r = 0; r < reps + 1; r++) {
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(a1, s1));
                CK(hipMemcpyAsync(hdst, dsrc, sz, hipMemcpyDeviceToHost, s1));
                CK(hipEventRecord(b1, s1));
                CK(hipEventSynchronize(b1));
                float m = 0;
                CK(hipEventElapsedTime(&m, a1, b1));
                if (r) ms.push_back(m);
            }
            const double t = median(ms);
            std::printf("{\"variant\": \"memcpy-size\", \"bytes\": %zu, \"d2h_ms\": %.3f, \"d2h_GBps\": %.1f}\n", sz, t,
                        sz / (t * 1e-3) / 1e9);
        }
        std::fflush(stdout);
        return 0;
    }
    for (int variant = 0; variant < 6; variant++) {
        if (variant >= 4) {  // H2D by kernel, alone / beside a D2H memcpy
            const bool d2h = variant == 5;
            std::vector<double> k_ms, d_ms;
            for (int r = 0; r < reps + 1; r++) {
                CK(hipDeviceSynchronize());
                if (d2h) {
                    CK(hipEventRecord(a2, s2));
                    CK(hipMemcpyAsync(hdst, dsrc, bytes, hipMemcpyDeviceToHost, s2));
                    CK(hipEventRecord(b2, s2));
                }
                CK(hipEventRecord(a1, s1));
                hipLaunchKernelGGL(d2h_k, dim3(wgs), dim3(256), 0, s1, (const u32x4 *)hsrc_dev, (u32x4 *)ddst, n16);
                CK(hipEventRecord(b1, s1));
                CK(hipDeviceSynchronize());
                CK(hipGetLastError());
                float m1 = 0, m2 = 0;
                CK(hipEventElapsedTime(&m1, a1, b1));
                if (d2h) CK(hipEventElapsedTime(&m2, a2, b2));
                if (r) {
                    k_ms.push_back(m1);
                    d_ms.push_back(m2);
                }
            }
            unsigned char probe = 0;
            CK(hipMemcpy(&probe, static_cast<unsigned char *>(ddst) + bytes / 2, 1, hipMemcpyDeviceToHost));
            const double t1 = median(k_ms), t2 = median(d_ms);
            std::printf("{\"variant\": \"h2dkernel%s\", \"bytes\": %zu, \"workgroups\": %d, \"h2d_ms\": %.3f, "
                        "\"h2d_GBps\": %.1f, \"d2h_GBps\": %s, \"check\": %s}\n",
                        d2h ? "+d2h" : "", bytes, wgs, t1, bytes / (t1 * 1e-3) / 1e9,
                        d2h ? std::to_string(bytes / (t2 * 1e-3) / 1e9).c_str() : "null", probe == 1 ? "true" : "false");
            std::fflush(stdout);
            continue;
        }
        const bool kern = variant & 1, h2d = variant & 2;
        std::vector<double> d2h_ms, h2d_ms;
        for (int r = 0; r < reps + 1; r++) {
            CK(hipDeviceSynchronize());
            if (h2d) {
                CK(hipEventRecord(a2, s2));
                CK(hipMemcpyAsync(ddst, hsrc, bytes, hipMemcpyHostToDevice, s2));
                CK(hipEventRecord(b2, s2));
            }
            CK(hipEventRecord(a1, s1));
            if (kern)
                hipLaunchKernelGGL(d2h_k, dim3(wgs), dim3(256), 0, s1, (const u32x4 *)dsrc, (u32x4 *)hdst_dev, n16);
            else
                CK(hipMemcpyAsync(hdst, dsrc, bytes, hipMemcpyDeviceToHost, s1));
            CK(hipEventRecord(b1, s1));
            CK(hipDeviceSynchronize());
            CK(hipGetLastError());
            float m1 = 0, m2 = 0;
            CK(hipEventElapsedTime(&m1, a1, b1));
            if (h2d) CK(hipEventElapsedTime(&m2, a2, b2));
            if (r) {
                d2h_ms.push_back(m1);
                h2d_ms.push_back(m2);
            }
        }
        // the host buffer holds the device bytes
        const unsigned char *h = static_cast<const unsigned char *>(hdst);
        const bool ok = h[0] == 7 && h[bytes / 2] == 7 && h[bytes - 1] == 7;
        std::memset(hdst, 0, bytes);
        const double t1 = median(d2h_ms), t2 = median(h2d_ms);
        std::printf("{\"variant\": \"%s%s\", \"host_memory\": \"%s\", \"same_pointer\": %s, \"bytes\": %zu, "
                    "\"workgroups\": %d, \"d2h_ms\": %.3f, \"d2h_GBps\": %.1f, \"h2d_GBps\": %s, \"check\": %s}\n",
                    kern ? "kernel" : "memcpy", h2d ? "+h2d" : "",
                    kind == 2 ? "registered" : kind == 1 ? "hipHostMallocNonCoherent" : "hipHostMallocDefault",
                    hdst_dev == hdst ? "true" : "false", bytes, kern ? wgs : 0, t1, bytes / (t1 * 1e-3) / 1e9,
                    h2d ? std::to_string(bytes / (t2 * 1e-3) / 1e9).c_str() : "null", ok ? "true" : "false");
        std::fflush(stdout);
    }
    return 0;
}

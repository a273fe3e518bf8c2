// hiperr_probe.hip — which HIP call leaves an error on a fresh host thread.
//
// HIP keeps the last error per host thread with CUDA's semantics: hipGetLastError() returns the last
// failure of ANY earlier call on the thread, not the status of the call just made. Round 3's
// concurrent ChunkSet::new test once failed with "fused encode + chunk hashing launch: invalid device
// ordinal (101)" from the hipGetLastError() behind a launch. This probe starts T threads at a barrier;
// each runs the library's lane sequence (hipSetDevice, hipStreamCreateWithFlags, hipMalloc,
// hipHostMalloc, hipMemcpyAsync, first launch of a kernel, hipStreamSynchronize) and records
// hipPeekAtLastError() after every call, so the first call that leaves a pending error is named.
// Mode "lazy": the kernels are launched for the first time by the T threads at once (round 3's
// situation before the eager resolution at context creation). Mode "eager": the main thread resolves
// them first with hipFuncGetAttributes (what decds_ctx_create -> configure_kernels does now).
// Build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/hiperr_probe.hip -o build/hiperr_probe -lpthread
// Run:   build/hiperr_probe [threads] [lazy|eager] [rounds]
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

template <int I>
__global__ void probe_kernel(uint32_t *p, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = (uint32_t)(i * 2654435761u) ^ I;
}

struct Step {
    const char *what;
    hipError_t ret, pending;
};

static std::atomic<int> g_arrived{0};

static void worker(int t, int nthreads, std::vector<Step> *log) {
    g_arrived.fetch_add(1);
    while (g_arrived.load() < nthreads) {
    }
    auto rec = [&](const char *what, hipError_t r) { log->push_back({what, r, hipPeekAtLastError()}); };
    rec("hipSetDevice", hipSetDevice(0));
    hipStream_t s = nullptr;
    rec("hipStreamCreateWithFlags", hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t *d = nullptr, *h = nullptr;
    const size_t n = 1 << 20;
    rec("hipMalloc", hipMalloc(reinterpret_cast<void **>(&d), n * 4));
    rec("hipHostMalloc", hipHostMalloc(reinterpret_cast<void **>(&h), n * 4, hipHostMallocDefault));
    rec("hipMemcpyAsync H2D", hipMemcpyAsync(d, h, n * 4, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(probe_kernel<0>, dim3(n / 256), dim3(256), 0, s, d, n);
    rec("hipLaunchKernelGGL probe_kernel<0> (first launch)", hipSuccess);
    hipLaunchKernelGGL(probe_kernel<1>, dim3(n / 256), dim3(256), 0, s, d, n);
    rec("hipLaunchKernelGGL probe_kernel<1> (first launch)", hipSuccess);
    rec("hipMemcpyAsync D2H", hipMemcpyAsync(h, d, n * 4, hipMemcpyDeviceToHost, s));
    rec("hipStreamSynchronize", hipStreamSynchronize(s));
    rec("hipGetLastError (consumes)", hipGetLastError());
    (void)hipFree(d);
    (void)hipHostFree(h);
    (void)hipStreamDestroy(s);
    (void)t;
}

int main(int argc, char **argv) {
    const int T = argc > 1 ? std::atoi(argv[1]) : 16;
    const bool eager = argc > 2 && std::strcmp(argv[2], "eager") == 0;
    const int rounds = argc > 3 ? std::atoi(argv[3]) : 1;
    int rt = 0, drv = 0;
    (void)hipRuntimeGetVersion(&rt);
    (void)hipDriverGetVersion(&drv);
    if (hipSetDevice(0) != hipSuccess) return 2;
    if (eager) {
        hipFuncAttributes a;
        if (hipFuncGetAttributes(&a, reinterpret_cast<const void *>(probe_kernel<0>)) ||
            hipFuncGetAttributes(&a, reinterpret_cast<const void *>(probe_kernel<1>)))
            return 3;
    }
    int bad_threads = 0;
    for (int r = 0; r < rounds; r++) {
        g_arrived = 0;
        std::vector<std::vector<Step>> logs(T);
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++) th.emplace_back(worker, t, T, &logs[t]);
        for (auto &x : th) x.join();
        for (int t = 0; t < T; t++) {
            const Step *first = nullptr;
            for (const Step &s : logs[t])
                if (s.ret != hipSuccess || s.pending != hipSuccess) {
                    first = &s;
                    break;
                }
            if (!first) continue;
            bad_threads++;
            std::printf("{\"round\": %d, \"thread\": %d, \"first_call\": \"%s\", \"returned\": %d, \"pending\": %d, "
                        "\"pending_text\": \"%s\"}\n",
                        r, t, first->what, (int)first->ret, (int)first->pending, hipGetErrorString(first->pending));
        }
    }
    std::printf("{\"probe\": \"hiperr\", \"mode\": \"%s\", \"threads\": %d, \"rounds\": %d, \"runtime\": %d, "
                "\"driver\": %d, \"threads_with_pending_error\": %d}\n",
                eager ? "eager" : "lazy", T, rounds, rt, drv, bad_threads);
    return 0;
}

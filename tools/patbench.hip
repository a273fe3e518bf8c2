// patbench.hip — memory-pattern ceilings of the codec kernels' work maps (no GF arithmetic): per
// 16-column lane block 10 row loads and 16 (encode shape) or 10 (decode shape) row stores, with the
// rlnc row geometry, walked in the kernels' own orders (walk_tiles: contiguous ranges, super-tiles,
// XCD bands) and with optional store throttles (s_waitcnt vmcnt(0) after every G stores). All
// variants run in ONE process, rounds interleaved (cdna_hip_programming.md §5.4 rule 24).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/patbench.hip -o build/patbench
// usage: build/patbench <n_chunksets> <rounds>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../decds_amd/csrc/rlnc_kernels.hip"

using namespace decds;

// ENC: inputs = pieces of a chunkset (i*L), outputs = coded payloads (j*F + 10).
// DEC: inputs = coded payloads of rows 0..9, outputs = pieces.
template <int MAP, bool ENC, int G, int SY = 0>
__global__ __launch_bounds__(WG, WAVES_PER_SIMD) void pat_kernel(const uint8_t *__restrict__ src, size_t n,
                                                                 uint8_t *__restrict__ dst) {
    constexpr int NOUT = ENC ? (int)N : (int)K;
    uint32_t ioff[K], ooff[NOUT];
#pragma unroll
    for (int i = 0; i < (int)K; i++) ioff[i] = ENC ? (uint32_t)(i * L) : (uint32_t)(i * F + K);
#pragma unroll
    for (int j = 0; j < NOUT; j++) ooff[j] = ENC ? (uint32_t)(j * F + K) : (uint32_t)(j * L);
    walk_tiles<MAP>(n, [&](uint32_t cs, uint32_t tile, uint32_t, bool) {
        if (SY) __builtin_amdgcn_s_barrier();
        const uint8_t *ibase = src + (size_t)cs * (ENC ? CS : N * F);
        uint8_t *obase = dst + (size_t)cs * (ENC ? N * F : CS);
        const uint32_t block = tile * TILE_BLOCKS + threadIdx.x;
        if (block >= MAIN_BLOCKS) return;
        const uint32_t col0 = block * COLS_PER_LANE;
        uint4 x[K];
        load_block<EncTune, K>(x, ibase, ioff, col0);
#pragma unroll
        for (int j = 0; j < NOUT; j++) {
            const uint4 a = x[j % K], b = x[(j + 3) % K];
            strow<-1>(obase, ooff[j] + col0, make_uint4(a.x ^ b.y, a.y ^ b.z, a.z ^ b.w, a.w ^ b.x));
            if (G > 0 && (j + 1) % G == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    });
}

// NP output rows per pass: per block NOUT/NP passes, each re-loading the 10 inputs (L2 hits) and
// storing NP rows behind a vmcnt(0) wait (fewer stores in flight per wave)
template <int NP>
__global__ __launch_bounds__(WG, WAVES_PER_SIMD) void np_kernel(const uint8_t *__restrict__ src, size_t n,
                                                               uint8_t *__restrict__ dst) {
    uint32_t ioff[K], ooff[N];
#pragma unroll
    for (int i = 0; i < (int)K; i++) ioff[i] = (uint32_t)(i * L);
#pragma unroll
    for (int j = 0; j < (int)N; j++) ooff[j] = (uint32_t)(j * F + K);
    walk_tiles<0>(n, [&](uint32_t cs, uint32_t tile, uint32_t, bool) {
        const uint8_t *ibase = src + (size_t)cs * CS;
        uint8_t *obase = dst + (size_t)cs * N * F;
        const uint32_t block = tile * TILE_BLOCKS + threadIdx.x;
        if (block >= MAIN_BLOCKS) return;
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
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    });
}

// MB blocks per lane: a wave covers MB consecutive KiB of every row per tile (lane block of
// instruction m = base + 64m + lane) and stores all MB pieces of a row back to back, so
// each row receives an MB-KiB contiguous burst from one wave at one time (contiguous tile ranges)
template <int MB, bool ENC>
__global__ __launch_bounds__(WG, WAVES_PER_SIMD) void mb_kernel(const uint8_t *__restrict__ src, size_t n,
                                                               uint8_t *__restrict__ dst) {
    constexpr int NOUT = ENC ? (int)N : (int)K;
    constexpr uint32_t TPC = TILES_PER_CS / MB;  // tiles of MB*256 blocks
    uint32_t ioff[K], ooff[NOUT];
#pragma unroll
    for (int i = 0; i < (int)K; i++) ioff[i] = ENC ? (uint32_t)(i * L) : (uint32_t)(i * F + K);
#pragma unroll
    for (int j = 0; j < NOUT; j++) ooff[j] = ENC ? (uint32_t)(j * F + K) : (uint32_t)(j * L);
    const uint64_t total = (uint64_t)n * TPC;
    const uint32_t t0 = (uint32_t)(total * blockIdx.x / gridDim.x), t1 = (uint32_t)(total * (blockIdx.x + 1) / gridDim.x);
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (uint32_t t = t0; t < t1; t++) {
        const uint32_t cs = t / TPC, tile = t % TPC;
        const uint8_t *ibase = src + (size_t)cs * (ENC ? CS : N * F);
        uint8_t *obase = dst + (size_t)cs * (ENC ? N * F : CS);
        uint4 x[MB][K];
        uint32_t blk[MB];
#pragma unroll
        for (int m = 0; m < MB; m++) {
            blk[m] = (tile * 4 + wave) * 64 * MB + m * 64 + lane;
            if (blk[m] < MAIN_BLOCKS) load_block<EncTune, K>(x[m], ibase, ioff, blk[m] * COLS_PER_LANE);
        }
#pragma unroll
        for (int j = 0; j < NOUT; j++)
#pragma unroll
            for (int m = 0; m < MB; m++) {
                const uint4 a = x[m][j % K], b = x[m][(j + 3) % K];
                if (blk[m] < MAIN_BLOCKS)
                    strow<-1>(obase, ooff[j] + blk[m] * COLS_PER_LANE, make_uint4(a.x ^ b.y, a.y ^ b.z, a.z ^ b.w, a.w ^ b.x));
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

struct Case {
    std::string name;
    bool enc;
    void (*fn)(const uint8_t *, size_t, uint8_t *);
    bool band;
    std::vector<float> ms;
    uint32_t gmul = 1;  // grid multiplier (occupancy study; contiguous map only)
    uint32_t np = 0;    // non-persistent: T tiles per workgroup (grid = tiles / T)
};

#define CASE(MAP, ENC, G, NAME) Case{NAME, ENC, pat_kernel<MAP, ENC, G>, MAP == MAP_BAND, {}}
#define CASESY(MAP, ENC, NAME) Case{NAME, ENC, pat_kernel<MAP, ENC, 0, 1>, MAP == MAP_BAND, {}}

int main(int argc, char **argv) {
    const size_t n = argc > 1 ? strtoul(argv[1], nullptr, 10) : 1639;
    const int rounds = argc > 2 ? atoi(argv[2]) : 6;
    const size_t a_bytes = n * N * F + 64, b_bytes = n * CS + 64;
    uint8_t *a, *b;  // a: coded rows, b: chunksets
    if (hipMalloc(&a, a_bytes) || hipMalloc(&b, b_bytes)) {
        printf("alloc failed\n");
        return 1;
    }
    hipLaunchKernelGGL(random_fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t *>(a), a_bytes / 8);
    hipLaunchKernelGGL(random_fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t *>(b), b_bytes / 8);
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    LaunchGeom lg{prop.multiProcessorCount};
    const uint32_t grid = stream_grid(lg, n);
    std::vector<Case> cases = {
        CASE(0, true, 0, "enc_map0"),       CASE(8, true, 0, "enc_map8"),       CASE(MAP_BAND, true, 0, "enc_band"),
        CASE(0, true, 4, "enc_map0_g4"),    CASE(0, true, 8, "enc_map0_g8"),    CASE(0, true, 16, "enc_map0_drain"),
        CASE(MAP_BAND, true, 4, "enc_band_g4"), CASE(MAP_BAND, true, 16, "enc_band_drain"),
        Case{"enc_np4", true, np_kernel<4>, false, {}}, Case{"enc_np8", true, np_kernel<8>, false, {}},
        CASE(2, true, 0, "enc_map2"),       CASE(32, true, 0, "enc_map32"),
        CASESY(0, true, "enc_map0_sync"),   CASESY(MAP_BAND, true, "enc_band_sync"), CASESY(8, true, "enc_map8_sync"),
        CASESY(8, false, "dec_map8_sync"),  CASESY(MAP_BAND, false, "dec_band_sync"),
        Case{"enc_mb2", true, mb_kernel<2, true>, false, {}}, Case{"enc_mb4", true, mb_kernel<4, true>, false, {}},
        Case{"dec_mb2", false, mb_kernel<2, false>, false, {}}, Case{"dec_mb4", false, mb_kernel<4, false>, false, {}},
        Case{"enc_map0_x2", true, pat_kernel<0, true, 0>, false, {}, 2},
        Case{"enc_map0_x4", true, pat_kernel<0, true, 0>, false, {}, 4},
        Case{"enc_np2", true, pat_kernel<-2, true, 0>, false, {}, 1, 2},
        Case{"enc_np8", true, pat_kernel<-8, true, 0>, false, {}, 1, 8},
        Case{"dec_map0_x4", false, pat_kernel<0, false, 0>, false, {}, 4},
        Case{"dec_np8", false, pat_kernel<-8, false, 0>, false, {}, 1, 8},
        CASE(0, false, 0, "dec_map0"),      CASE(8, false, 0, "dec_map8"),      CASE(MAP_BAND, false, 0, "dec_band"),
        CASE(8, false, 5, "dec_map8_g5"),   CASE(MAP_BAND, false, 5, "dec_band_g5"), CASE(MAP_BAND, false, 10, "dec_band_drain"),
    };
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto launch = [&](Case &c) {
        uint32_t g = c.band ? grid & ~7u : grid * c.gmul;
        if (c.np) g = (uint32_t)((n * TILES_PER_CS + c.np - 1) / c.np);
        if (c.enc)
            hipLaunchKernelGGL(c.fn, dim3(g), dim3(WG), 0, 0, b, n, a);
        else
            hipLaunchKernelGGL(c.fn, dim3(g), dim3(WG), 0, 0, a, n, b);
    };
    for (auto &c : cases) launch(c);
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("kernel error\n");
        return 1;
    }
    for (int r = 0; r < rounds; r++) {
        for (size_t ci = 0; ci < cases.size(); ci++) {
            Case &c = cases[r % 2 ? cases.size() - 1 - ci : ci];
            hipEventRecord(e0);
            launch(c);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
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
        const double bytes = c.enc ? (double)n * (CS + N * F) : (double)n * (K * F + CS);
        printf("{\"case\": \"%s\", \"n\": %zu, \"ms\": %.4f, \"min_ms\": %.4f, \"GBps\": %.1f}\n", c.name.c_str(), n,
               med, c.ms[0], bytes / med / 1e6);
    }
    return 0;
}

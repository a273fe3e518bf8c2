// valubench.hip — issue rate of the integer VALU ops a BLAKE3 compression is made of (v_xor_b32,
// v_add_u32, v_add3_u32, v_alignbit_b32, v_perm_b32) and of v_add_f32 for reference, with 8
// independent chains per lane and 8 waves per SIMD, as shader cycles per wave-instruction per SIMD
// (s_memtime ticks over the loop, one timing per wave).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/valubench.hip -o build/valubench
#include <hip/hip_runtime.h>

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

constexpr int ITERS = 8192;

#define OP8(INS)                                                                               \
    asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS         \
                     " %3, %3, %8\n\t" INS " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS           \
                     " %6, %6, %8\n\t" INS " %7, %7, %8"                                        \
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]),      \
                   "+v"(r[6]), "+v"(r[7])                                                       \
                 : "v"(k));
#define OP8_3(INS, IMM)                                                                        \
    asm volatile(INS " %0, %0, %8, " IMM "\n\t" INS " %1, %1, %8, " IMM "\n\t" INS               \
                     " %2, %2, %8, " IMM "\n\t" INS " %3, %3, %8, " IMM "\n\t" INS               \
                     " %4, %4, %8, " IMM "\n\t" INS " %5, %5, %8, " IMM "\n\t" INS               \
                     " %6, %6, %8, " IMM "\n\t" INS " %7, %7, %8, " IMM                          \
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]),      \
                   "+v"(r[6]), "+v"(r[7])                                                       \
                 : "v"(k));
#define OP8_V3(INS)                                                                            \
    asm volatile(INS " %0, %0, %8, %1\n\t" INS " %1, %1, %8, %2\n\t" INS " %2, %2, %8, %3\n\t"    \
                 INS " %3, %3, %8, %4\n\t" INS " %4, %4, %8, %5\n\t" INS " %5, %5, %8, %6\n\t"     \
                 INS " %6, %6, %8, %7\n\t" INS " %7, %7, %8, %0"                                 \
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]),      \
                   "+v"(r[6]), "+v"(r[7])                                                       \
                 : "v"(k));

#define OP8_LIT(INS)                                                                           \
    asm volatile(INS " %0, 0x1234567, %0\n\t" INS " %1, 0x1234567, %1\n\t" INS " %2, 0x1234567, %2\n\t" \
                 INS " %3, 0x1234567, %3\n\t" INS " %4, 0x1234567, %4\n\t" INS " %5, 0x1234567, %5\n\t" \
                 INS " %6, 0x1234567, %6\n\t" INS " %7, 0x1234567, %7"                               \
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]),      \
                   "+v"(r[6]), "+v"(r[7])                                                       \
                 : "v"(k));
#define OP8_E64(INS) OP8(INS)
#define OP8_B3                                                                                 \
    asm volatile("v_bitop3_b32 %0, %0, %8, %1 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %8, %2 bitop3:0x96\n\t" \
                 "v_bitop3_b32 %2, %2, %8, %3 bitop3:0x96\n\tv_bitop3_b32 %3, %3, %8, %4 bitop3:0x96\n\t" \
                 "v_bitop3_b32 %4, %4, %8, %5 bitop3:0x96\n\tv_bitop3_b32 %5, %5, %8, %6 bitop3:0x96\n\t" \
                 "v_bitop3_b32 %6, %6, %8, %7 bitop3:0x96\n\tv_bitop3_b32 %7, %7, %8, %0 bitop3:0x96"    \
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]),      \
                   "+v"(r[6]), "+v"(r[7])                                                       \
                 : "v"(k));
#define SDWB " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
#define OP8_SDWB                                                                               \
    asm volatile("v_and_b32_sdwa %0, %0, %8" SDWB "\n\tv_and_b32_sdwa %1, %1, %8" SDWB                \
                 "\n\tv_and_b32_sdwa %2, %2, %8" SDWB "\n\tv_and_b32_sdwa %3, %3, %8" SDWB              \
                 "\n\tv_and_b32_sdwa %4, %4, %8" SDWB "\n\tv_and_b32_sdwa %5, %5, %8" SDWB              \
                 "\n\tv_and_b32_sdwa %6, %6, %8" SDWB "\n\tv_and_b32_sdwa %7, %7, %8" SDWB              \
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]),      \
                   "+v"(r[6]), "+v"(r[7])                                                       \
                 : "v"(k));
#define SDW " dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0"
#define OP8_SDWA                                                                               \
    asm volatile("v_xor_b32_sdwa %0, %0, %8" SDW "\n\tv_xor_b32_sdwa %1, %1, %8" SDW                \
                 "\n\tv_xor_b32_sdwa %2, %2, %8" SDW "\n\tv_xor_b32_sdwa %3, %3, %8" SDW              \
                 "\n\tv_xor_b32_sdwa %4, %4, %8" SDW "\n\tv_xor_b32_sdwa %5, %5, %8" SDW              \
                 "\n\tv_xor_b32_sdwa %6, %6, %8" SDW "\n\tv_xor_b32_sdwa %7, %7, %8" SDW              \
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]),      \
                   "+v"(r[6]), "+v"(r[7])                                                       \
                 : "v"(k));

template <int OP>
__global__ __launch_bounds__(256) void valu_kernel(uint32_t *out, uint64_t *ticks) {
    uint32_t r[8];
    for (int i = 0; i < 8; i++) r[i] = threadIdx.x * 8 + i;
    const uint32_t k = blockIdx.x | 1u;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; it++) {
        if constexpr (OP == 0) OP8("v_xor_b32")
        if constexpr (OP == 1) OP8("v_add_u32")
        if constexpr (OP == 2) OP8_V3("v_add3_u32")
        if constexpr (OP == 3) OP8_3("v_alignbit_b32", "7")
        if constexpr (OP == 4) OP8_V3("v_perm_b32")
        if constexpr (OP == 5) OP8("v_add_f32")
        if constexpr (OP == 6) OP8_V3("v_xad_u32")
        if constexpr (OP == 7) OP8_SDWA
        if constexpr (OP == 8) OP8_LIT("v_add_u32")
        if constexpr (OP == 9) OP8_V3("v_fma_f32")
        if constexpr (OP == 10) OP8("v_lshlrev_b32")
        if constexpr (OP == 11) OP8_V3("v_lshl_or_b32")
        if constexpr (OP == 12) OP8_E64("v_xor_b32_e64")
        if constexpr (OP == 13) OP8_B3
        if constexpr (OP == 14) OP8_SDWB
        if constexpr (OP == 15) OP8("v_pk_add_u16")
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
    for (int i = 0; i < 8; i++) x ^= r[i];
    out[blockIdx.x * 256 + threadIdx.x] = x;
    if ((threadIdx.x & 63) == 0) ticks[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const char *names[] = {"v_xor_b32", "v_add_u32", "v_add3_u32", "v_alignbit_b32", "v_perm_b32", "v_add_f32",
                           "v_xad_u32", "v_xor_b32_sdwa", "v_add_u32+literal", "v_fma_f32", "v_lshlrev_b32", "v_lshl_or_b32", "v_xor_b32_e64",
                           "v_bitop3_b32", "v_and_b32_sdwa(byte)", "v_pk_add_u16"};
    for (int wps : {8}) {   // waves per SIMD
        const int blocks = cus * wps; // 4 waves per block = one per SIMD
        uint32_t *out;
        uint64_t *ticks;
        CK(hipMalloc(&out, blocks * 256 * 4));
        CK(hipMalloc(&ticks, blocks * 4 * 8));
        for (int op = 0; op < 16; op++) {
            auto launch = [&] {
                switch (op) {
                    case 0: valu_kernel<0><<<blocks, 256>>>(out, ticks); break;
                    case 1: valu_kernel<1><<<blocks, 256>>>(out, ticks); break;
                    case 2: valu_kernel<2><<<blocks, 256>>>(out, ticks); break;
                    case 3: valu_kernel<3><<<blocks, 256>>>(out, ticks); break;
                    case 4: valu_kernel<4><<<blocks, 256>>>(out, ticks); break;
                    case 5: valu_kernel<5><<<blocks, 256>>>(out, ticks); break;
                    case 6: valu_kernel<6><<<blocks, 256>>>(out, ticks); break;
                    case 7: valu_kernel<7><<<blocks, 256>>>(out, ticks); break;
                    case 8: valu_kernel<8><<<blocks, 256>>>(out, ticks); break;
                    case 9: valu_kernel<9><<<blocks, 256>>>(out, ticks); break;
                    case 10: valu_kernel<10><<<blocks, 256>>>(out, ticks); break;
                    case 11: valu_kernel<11><<<blocks, 256>>>(out, ticks); break;
                    case 12: valu_kernel<12><<<blocks, 256>>>(out, ticks); break;
                    case 13: valu_kernel<13><<<blocks, 256>>>(out, ticks); break;
                    case 14: valu_kernel<14><<<blocks, 256>>>(out, ticks); break;
                    case 15: valu_kernel<15><<<blocks, 256>>>(out, ticks); break;
                }
            };
            launch();
            CK(hipDeviceSynchronize());
            hipEvent_t a, b;
            CK(hipEventCreate(&a));
            CK(hipEventCreate(&b));
            CK(hipEventRecord(a));
            launch();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            std::vector<uint64_t> h(blocks * 4);
            CK(hipMemcpy(h.data(), ticks, h.size() * 8, hipMemcpyDeviceToHost));
            double mean = 0;
            for (auto v : h) mean += (double)v;
            mean /= h.size();
            const double instr_per_wave = 8.0 * ITERS;
            // memtime ticks per wave-instruction of ONE wave; x waves sharing the SIMD = SIMD cost
            std::printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ticks_per_instr_per_wave\": %.2f, "
                        "\"simd_cycles_per_instr\": %.2f, \"ms\": %.4f, \"Tops\": %.2f}\n",
                        names[op], wps, mean / instr_per_wave, mean / instr_per_wave / wps, ms,
                        (double)blocks * 256 * instr_per_wave / ms / 1e9);
        }
        CK(hipFree(out));
        CK(hipFree(ticks));
    }
    return 0;
}

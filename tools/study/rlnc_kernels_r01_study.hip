// rlnc_kernels.hip — gfx950 (MI355X / CDNA4) kernels for decds' RLNC chunkset codec.
//
// The hot path is one GF(2^8) linear-combination pass over a batch of chunksets:
//   encode (chunkset.rs:43-52, rlnc Encoder::code x16):   y_j = sum_i C[j][i] * piece_i,  j<16, i<10
//   decode (chunkset.rs:181-204, rlnc Decoder):           piece_i = sum_k D[i][k] * y_k,  D = C_sel^-1
// Both stream 1 MiB piece columns from HBM once and write the results once. The GF multiply by a
// chunkset-uniform coefficient is a table lookup: per input piece i and nibble half h an LDS table
//   T[i][h][n] = { C[j][i] * (n << 4h) : j = 0..15 }   (16 B: all outputs' products at once)
// so one ds_read_b128 gives the contribution of one input nibble to all 16 outputs. Each table row
// is replicated 16x across the 64 LDS banks and lane l reads copy (l & 15): the 16 lanes of every
// ds_read_b128 lane group {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... hit 16 distinct 4-bank slots,
// so the data-dependent lookups are bank-conflict-free by construction (MI355X_MICROARCH.md §LDS).
// Per 16-column lane block: 10 unaligned 16-B loads, 320 conflict-free ds_read_b128, v_bitop3 XOR3
// accumulation into a 16x16 byte block (columns x outputs), a v_perm byte transpose, 16 (or 10)
// 16-B stores. No MFMA: this is byte-wise finite-field work, bounded by HBM (and LDS) bandwidth.
#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>

#include "rlnc_kernels.h"
#include "rlnc_layout.h"

namespace decds {

// ---- geometry ---------------------------------------------------------------------------------
constexpr uint32_t DECDS_NO_CANDIDATE_U8 = 0xFF;
constexpr uint32_t WG = 256;                                  // 4 waves
constexpr uint32_t WGS_PER_CU = 2;                            // 2 x 80 KiB LDS = the CU's 160 KiB
constexpr uint32_t WAVES_PER_SIMD = WGS_PER_CU * WG / 256;    // 2 -> up to 256 VGPRs per lane
constexpr uint32_t TILE_BLOCKS = WG;                          // one 16-col block per lane per tile
constexpr uint32_t TILES_PER_CS = (MAIN_BLOCKS + TILE_BLOCKS - 1) / TILE_BLOCKS;  // 256
constexpr uint32_t ROW_BYTES = 256;                           // 16 replicas x 16 B
constexpr uint32_t TABLE_BYTES = 16 * ROW_BYTES;              // 16 nibble rows
constexpr uint32_t LDS_BYTES = K * 2 * TABLE_BYTES;           // 80 KiB
static_assert(TILES_PER_CS == 256, "tile geometry");

// ---- per-kernel tuning (measured in one process by tools/abbench.py; DESIGN.md "Tuning log") --
//   ASM  : hand-pipelined LDS lookups (8-16 ds_read_b128 in flight per wave) instead of hipcc's
//          schedule (which waits after every column: ~4 in flight)
//   ROLL : the next block's input i is loaded as soon as this block has consumed input i
//   LAUX / SAUX : cache-policy word of the streaming loads / stores (buffer instructions; gfx950:
//          sc0 = 1, nt = 2, sc1 = 16); -1 = plain global_load / global_store
//   SYNC : workgroup barrier per tile (1: at the tile's start, 2: before its stores) so the 4 waves
//          write each row's 4 KiB span of the tile together instead of drifting apart
template <bool ASM_, bool ROLL_, int LAUX_, int SAUX_, int SYNC_ = 0>
struct Tune {
    static constexpr bool ASM = ASM_, ROLL = ROLL_;
    static constexpr int LAUX = LAUX_, SAUX = SAUX_, SYNC = SYNC_;
};
#ifndef DECDS_ENC_TUNE
#define DECDS_ENC_TUNE false, false, -1, -1
#endif
#ifndef DECDS_DEC_TUNE
#define DECDS_DEC_TUNE true, true, -1, 0
#endif
#ifndef DECDS_ENC_SYNC
#define DECDS_ENC_SYNC 0
#endif
#ifndef DECDS_DEC_SYNC
#define DECDS_DEC_SYNC 0
#endif
#ifndef DECDS_ENC_BF
#define DECDS_ENC_BF 1
#endif
#ifndef DECDS_ENC_BF_TUNE
#define DECDS_ENC_BF_TUNE true, true, 0, 0
#endif
using EncTune = Tune<DECDS_ENC_TUNE, DECDS_ENC_SYNC>;
using EncBfTune = Tune<DECDS_ENC_BF_TUNE, DECDS_ENC_SYNC>;  // DECDS_ENC_BF: per-chunkset branch-free segments
using DecTune = Tune<DECDS_DEC_TUNE, DECDS_DEC_SYNC>;

// ---- GF(2^8) ----------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t gf_mul(uint32_t a, uint32_t b, uint32_t poly) {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        acc ^= ((b >> i) & 1u) ? a : 0u;
        a <<= 1;
        a ^= (a & 0x100u) ? poly : 0u;
    }
    return acc & 0xFFu;
}

// Workgroup barrier for the LDS tables only: every wave's LDS accesses have completed, nothing
// else. __syncthreads() also drains each wave's outstanding global stores (a release fence), which
// made every table rebuild cost a full store-queue drain.
__device__ __forceinline__ void lds_barrier() {
#ifdef DECDS_FULL_SYNC
    __syncthreads();
#else
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0); vmcnt / expcnt left unconstrained
    __builtin_amdgcn_s_barrier();
#endif
}

// The 4 coefficient bytes thread p = 8i + 4h + q (< NIN*8) of build_tables combines:
// M[(4q + jj) * ldm + i], jj < 4 (zero for outputs >= NOUT and for idle threads). (Loading it one
// chunkset ahead measured no faster)
template <int NIN, int NOUT>
__device__ __forceinline__ uint32_t table_coeffs(const uint8_t *M, uint32_t ldm) {
    static_assert(NIN * 8 <= (int)WG, "one coefficient word per thread");
    const uint32_t p = threadIdx.x;
    uint32_t w = 0;
    if (p < NIN * 8) {
        const uint32_t q = p & 3u, i = p >> 3;
#pragma unroll
        for (uint32_t jj = 0; jj < 4; jj++)
            if (4 * q + jj < (uint32_t)NOUT) w |= (uint32_t)M[(4 * q + jj) * ldm + i] << (8 * jj);
    }
    return w;
}

// Build the 2*NIN replicated nibble tables of a NOUT x NIN coefficient matrix from the words of
// table_coeffs. Caller brackets with lds_barrier().
// Multiplication by a constant is linear over GF(2), so row (i, h, nib) = XOR of the products of
// C[.][i] with the set bits of nib << 4h: thread (i, h, output quad q) forms the 4 basis words
// { C[4q+jj][i] * x^(4h+k) : jj < 4 } (xtime chains) and the 16 rows' dwords q by one XOR each
// (nib & (nib-1) is nib minus its lowest bit), writing replica 0; a second pass copies each
// 16-byte row into replicas 1..15. ~30 VALU per thread instead of 5120 bit-serial multiplies.
#ifndef DECDS_REPLICA_FLAT
#define DECDS_REPLICA_FLAT 1
#endif
template <int NIN, int NOUT>
__device__ __forceinline__ void build_tables(uint8_t *lds, uint32_t cw, uint32_t poly) {
    const uint32_t p = threadIdx.x;
    if (p < NIN * 8) {
        const uint32_t q = p & 3u, h = (p >> 2) & 1u, i = p >> 3;
        uint32_t bw[4] = {0, 0, 0, 0};
#pragma unroll
        for (uint32_t jj = 0; jj < 4; jj++) {
            uint32_t c = (cw >> (8 * jj)) & 0xFFu;
            if (h) {
#pragma unroll
                for (int k = 0; k < 4; k++) c = (c << 1) ^ ((c & 0x80u) ? poly : 0u);
            }
#pragma unroll
            for (int k = 0; k < 4; k++) {
                bw[k] |= c << (8 * jj);
                c = (c << 1) ^ ((c & 0x80u) ? poly : 0u);
            }
        }
        uint32_t w[16];
        w[0] = 0;
#pragma unroll
        for (int nib = 1; nib < 16; nib++) w[nib] = w[nib & (nib - 1)] ^ bw[__builtin_ctz(nib)];
        // first copy in replica (2i + h) mod 16 (flat builds): the 32 lanes of a write group then
        // hit 32 distinct banks; replica 0 for all would be 8-way conflicts
        uint8_t *base = lds + (i * 2 + h) * TABLE_BYTES + (DECDS_REPLICA_FLAT ? ((i * 2 + h) & 15u) * 16 : 0) + 4 * q;
#pragma unroll
        for (int nib = 0; nib < 16; nib++) *reinterpret_cast<uint32_t *>(base + nib * ROW_BYTES) = w[nib];
    }
    lds_barrier();
#if DECDS_REPLICA_FLAT
    // the other 15 replicas of every row, one 16-byte slot per lane: consecutive lanes write
    // consecutive slots (conflict-free ds_write_b128; the first copy is read as a broadcast). Row-per-thread copies
    // put the 8 lanes of a write group 256 B apart, i.e. on the same banks: 8-way conflicts, ~18 %
    // of the encode kernel's LDS cycles (SQ_LDS_BANK_CONFLICT, r01m).
#pragma unroll 4
    for (uint32_t s = threadIdx.x; s < NIN * 32 * 16; s += blockDim.x) {
        const uint32_t src = (s >> 8) & 15u;  // table 2i + h = s >> 8 was written in replica (2i + h) mod 16
        if ((s & 15u) == src) continue;
        uint8_t *row = lds + (s >> 4) * ROW_BYTES;
        *reinterpret_cast<uint4 *>(row + (s & 15u) * 16) = *reinterpret_cast<const uint4 *>(row + src * 16);
    }
#else
    for (uint32_t r = threadIdx.x; r < NIN * 32; r += blockDim.x) {
        uint8_t *row = lds + r * ROW_BYTES;
        const uint4 val = *reinterpret_cast<const uint4 *>(row);
#pragma unroll
        for (int c = 1; c < 16; c++) *reinterpret_cast<uint4 *>(row + c * 16) = val;
    }
#endif
}

// byte product M[j][i] * x read back from replica 0 of the tables (tail / scalar path)
__device__ __forceinline__ uint32_t tbl_mul(const uint8_t *lds, uint32_t i, uint32_t j, uint32_t x) {
    return lds[(i * 2 + 0) * TABLE_BYTES + (x & 15u) * ROW_BYTES + j] ^
           lds[(i * 2 + 1) * TABLE_BYTES + (x >> 4) * ROW_BYTES + j];
}

// ---- streaming row access ---------------------------------------------------------------------
// Rows are addressed as a wave-uniform 64-bit base plus a 32-bit row offset (a chunkset's rows
// lie within 16 * pitch < 4 GiB of its base): global_load/store's SGPR-base + VGPR-offset form,
// or a buffer descriptor on that base when a cache-policy word is requested. Piece rows start at
// i*L (L = 2^20 + 1) and coded payloads at r*pitch + 10, so most rows are byte-misaligned by the
// rlnc layout itself; gfx9 vector memory accepts unaligned 16-B accesses.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Buffer descriptors cover 2 GiB from the row base (the launchers keep every row offset below). A
// lane with nothing to do passes column OOB_COL: its buffer loads return zeros and its buffer
// stores are dropped by the range check, so a streaming loop needs no per-lane branch (see the
// decode kernel's non-persistent path for why that matters).
constexpr uint32_t BUF_RECORDS = 0x80000000u;
constexpr uint32_t OOB_COL = 0x80000000u;

template <int AUX>
__device__ __forceinline__ uint4 ldrow(const uint8_t *base, uint32_t off) {
    u32x4 v;
    if constexpr (AUX >= 0) {
        const __amdgpu_buffer_rsrc_t r =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(base), 0, BUF_RECORDS, 0x00020000);
        v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
    } else {
        v = *reinterpret_cast<const u32x4 *>(base + off);
    }
    return make_uint4(v.x, v.y, v.z, v.w);
}

template <int AUX>
__device__ __forceinline__ void strow(uint8_t *base, uint32_t off, uint4 v) {
    const u32x4 w = {v.x, v.y, v.z, v.w};
    if constexpr (AUX >= 0) {
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, BUF_RECORDS, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(w, r, off, 0, AUX);
    } else {
        *reinterpret_cast<u32x4 *>(base + off) = w;
    }
}

template <class T, int NIN>
__device__ __forceinline__ void load_block(uint4 (&x)[NIN], const uint8_t *ibase, const uint32_t (&ioff)[NIN],
                                           uint32_t col0) {
#pragma unroll
    for (int i = 0; i < NIN; i++) x[i] = ldrow<T::LAUX>(ibase, ioff[i] + col0);
}

// 4x4 byte transpose: out[b].byte[p] = in[p].byte[b]
__device__ __forceinline__ void transpose4x4(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t &b0,
                                             uint32_t &b1, uint32_t &b2, uint32_t &b3) {
    const uint32_t u0 = __builtin_amdgcn_perm(a1, a0, 0x05010400u);  // a0.0 a1.0 a0.1 a1.1
    const uint32_t u1 = __builtin_amdgcn_perm(a1, a0, 0x07030602u);  // a0.2 a1.2 a0.3 a1.3
    const uint32_t u2 = __builtin_amdgcn_perm(a3, a2, 0x05010400u);  // a2.0 a3.0 a2.1 a3.1
    const uint32_t u3 = __builtin_amdgcn_perm(a3, a2, 0x07030602u);  // a2.2 a3.2 a2.3 a3.3
    b0 = __builtin_amdgcn_perm(u2, u0, 0x05040100u);
    b1 = __builtin_amdgcn_perm(u2, u0, 0x07060302u);
    b2 = __builtin_amdgcn_perm(u3, u1, 0x05040100u);
    b3 = __builtin_amdgcn_perm(u3, u1, 0x07060302u);
}

__device__ __forceinline__ uint32_t word_of(const uint4 &v, int w) {
    return w == 0 ? v.x : w == 1 ? v.y : w == 2 ? v.z : v.w;
}

__device__ __forceinline__ void xor3_into(uint32_t (&acc)[4], const u32x4 &a, const u32x4 &b) {
    // v_bitop3_b32 (gfx950): acc ^ a ^ b in one VALU op (truth table 0x96)
    acc[0] = __builtin_amdgcn_bitop3_b32(acc[0], a.x, b.x, 0x96);
    acc[1] = __builtin_amdgcn_bitop3_b32(acc[1], a.y, b.y, 0x96);
    acc[2] = __builtin_amdgcn_bitop3_b32(acc[2], a.z, b.z, 0x96);
    acc[3] = __builtin_amdgcn_bitop3_b32(acc[3], a.w, b.w, 0x96);
}

// ---- lookups, compiler-scheduled ----------------------------------------------------------------
// address = nibble * 256 + laneoff, assembled by one v_perm: byte0 <- laneoff, byte1 <- the nibble
// of byte p, bytes 2,3 <- 0 (tables >= 64 KiB take byte 2 from laneoff_hi = laneoff | 0x10000)
template <class T, int NIN>
__device__ __forceinline__ void lookups_compiled(uint32_t (&acc)[16][4], uint4 (&x)[NIN], const uint8_t *lds,
                                                 uint32_t laneoff, const uint8_t *ibase, const uint32_t (&ioff)[NIN],
                                                 uint32_t ncol0) {
#pragma unroll
    for (int i = 0; i < NIN; i++) {
        const uint8_t *tlo = lds + (i * 2 + 0) * TABLE_BYTES;
        const uint8_t *thi = lds + (i * 2 + 1) * TABLE_BYTES;
#pragma unroll
        for (int w = 0; w < 4; w++) {
            const uint32_t xw = word_of(x[i], w);
            const uint32_t lo = xw & 0x0F0F0F0Fu, hi = (xw >> 4) & 0x0F0F0F0Fu;
#pragma unroll
            for (int p = 0; p < 4; p++) {
                const uint32_t sel = 0x0C0C0000u | ((4u + p) << 8);
                const uint32_t alo = __builtin_amdgcn_perm(lo, laneoff, sel);
                const uint32_t ahi = __builtin_amdgcn_perm(hi, laneoff, sel);
                const u32x4 a = *reinterpret_cast<const u32x4 *>(tlo + alo);
                const u32x4 b = *reinterpret_cast<const u32x4 *>(thi + ahi);
                xor3_into(acc[4 * w + p], a, b);
            }
        }
        if constexpr (T::ROLL) x[i] = ldrow<T::LAUX>(ibase, ioff[i] + ncol0);
    }
}

// ---- lookups, hand-pipelined --------------------------------------------------------------------
// The lookups of one lane block are cut into 4*NIN groups (input i, dword w: 4 columns x {lo, hi}
// = 8 reads); group g+1 is issued before group g is consumed, so 8-16 reads are in flight per wave.
// Reads are inline asm with immediate table offsets and explicit counted waits
// (cdna_hip_programming.md §5.7 form (ii)): nothing else in this region issues LGKM operations and
// one wave's LDS reads return in order.
template <int G>
__device__ __forceinline__ void lds_issue(u32x4 (&r)[8], uint32_t xw, uint32_t laneoff, uint32_t laneoff_hi) {
    constexpr int i = G >> 2;
    constexpr uint32_t tlo = (2 * i) * TABLE_BYTES, thi = (2 * i + 1) * TABLE_BYTES;
    constexpr bool flo = tlo >= 65536, fhi = thi >= 65536;  // ds offsets are 16-bit
    const uint32_t lo = xw & 0x0F0F0F0Fu;
    const uint32_t hi = (xw >> 4) & 0x0F0F0F0Fu;
#pragma unroll
    for (int p = 0; p < 4; p++) {
        const uint32_t sel_lo = (flo ? 0x0C020000u : 0x0C0C0000u) | ((4u + p) << 8);
        const uint32_t sel_hi = (fhi ? 0x0C020000u : 0x0C0C0000u) | ((4u + p) << 8);
        const uint32_t alo = __builtin_amdgcn_perm(lo, flo ? laneoff_hi : laneoff, sel_lo);
        const uint32_t ahi = __builtin_amdgcn_perm(hi, fhi ? laneoff_hi : laneoff, sel_hi);
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r[2 * p]) : "v"(alo), "i"(flo ? tlo - 65536 : tlo));
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r[2 * p + 1]) : "v"(ahi), "i"(fhi ? thi - 65536 : thi));
    }
}

template <int CNT>
__device__ __forceinline__ void lds_wait(u32x4 (&r)[8]) {
    asm volatile("s_waitcnt lgkmcnt(%8)"
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                 : "i"(CNT)
                 : "memory");
}

template <class T, int NIN, int G>
__device__ __forceinline__ void lds_step(uint32_t (&acc)[16][4], u32x4 (&ra)[8], u32x4 (&rb)[8], uint4 (&x)[NIN],
                                         uint32_t laneoff, uint32_t laneoff_hi, const uint8_t *ibase,
                                         const uint32_t (&ioff)[NIN], uint32_t ncol0) {
    constexpr int NG = 4 * NIN;
    u32x4(&cur)[8] = (G & 1) ? rb : ra;  // group G's results
    u32x4(&nxt)[8] = (G & 1) ? ra : rb;
    if constexpr (G + 1 < NG) {
        lds_issue<G + 1>(nxt, word_of(x[(G + 1) >> 2], (G + 1) & 3), laneoff, laneoff_hi);
        // input (G+1)>>2 is fully issued: its register may now take the next block's bytes
        if constexpr (T::ROLL && ((G + 1) & 3) == 3) x[(G + 1) >> 2] = ldrow<T::LAUX>(ibase, ioff[(G + 1) >> 2] + ncol0);
        lds_wait<8>(cur);
    } else {
        lds_wait<0>(cur);
    }
    constexpr int w = G & 3;
#pragma unroll
    for (int p = 0; p < 4; p++) xor3_into(acc[4 * w + p], cur[2 * p], cur[2 * p + 1]);
}

template <class T, int NIN, int... Gs>
__device__ __forceinline__ void lookups_asm(std::integer_sequence<int, Gs...>, uint32_t (&acc)[16][4], uint4 (&x)[NIN],
                                            uint32_t laneoff, const uint8_t *ibase, const uint32_t (&ioff)[NIN],
                                            uint32_t ncol0) {
    const uint32_t laneoff_hi = laneoff | 0x10000u;
    u32x4 ra[8], rb[8];
    lds_issue<0>(ra, x[0].x, laneoff, laneoff_hi);
    (lds_step<T, NIN, Gs>(acc, ra, rb, x, laneoff, laneoff_hi, ibase, ioff, ncol0), ...);
}

// One 16-column lane block: out_j[col0 .. col0+16) = sum_i M[j][i] * in_i[col0 .. col0+16).
// x holds this block's inputs on entry; with T::ROLL it holds the inputs at column ncol0 on exit
// (each loaded as soon as this block has consumed that input, before this block's stores: gfx9's
// vmcnt counts stores too, so a load issued behind the stores would also wait for them).
template <class T, int NIN, int NOUT>
__device__ __forceinline__ void combine_block(const uint8_t *lds, uint32_t laneoff, uint4 (&x)[NIN], uint8_t *obase,
                                              const uint32_t (&ooff)[NOUT], uint32_t col0, const uint8_t *ibase,
                                              const uint32_t (&ioff)[NIN], uint32_t ncol0) {
    uint32_t acc[16][4];  // acc[column][output group]: byte b = output 4*group + b
#pragma unroll
    for (int c = 0; c < 16; c++)
#pragma unroll
        for (int q = 0; q < 4; q++) acc[c][q] = 0;
    if constexpr (T::ASM)
        lookups_asm<T, NIN>(std::make_integer_sequence<int, 4 * NIN>{}, acc, x, laneoff, ibase, ioff, ncol0);
    else
        lookups_compiled<T, NIN>(acc, x, lds, laneoff, ibase, ioff, ncol0);
    if constexpr (T::SYNC == 2) __builtin_amdgcn_s_barrier();  // the 4 waves store the tile together
    // columns x outputs -> outputs x columns
#pragma unroll
    for (int q = 0; q < 4; q++) {
        if (4 * q >= NOUT) break;
        uint32_t o[4][4];  // o[b][w]: output 4q+b, columns 4w..4w+3
#pragma unroll
        for (int w = 0; w < 4; w++)
            transpose4x4(acc[4 * w + 0][q], acc[4 * w + 1][q], acc[4 * w + 2][q], acc[4 * w + 3][q], o[0][w], o[1][w],
                         o[2][w], o[3][w]);
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int j = 4 * q + b;
            if (j < NOUT) strow<T::SAUX>(obase, ooff[j] + col0, make_uint4(o[b][0], o[b][1], o[b][2], o[b][3]));
        }
    }
}

// ---- work split ---------------------------------------------------------------------------------
// The n*256 tiles (256 lane blocks = 4096 columns each) are walked in one of four orders:
// MAP == 0: equal contiguous ranges, one per resident workgroup (each workgroup rebuilds its LDS
//   tables only when its range crosses into the next chunkset).
// MAP > 0: super-tiles of MAP consecutive tiles of one chunkset dealt round-robin to the
//   workgroups, so the resident workgroups sweep a few whole chunksets side by side, at the price
//   of a table rebuild per super-tile.
// MAP < MAP_BAND: non-persistent — workgroup b takes the T = -MAP consecutive tiles from b*T and
//   exits; the dispatcher sweeps the batch in order and refills a CU as soon as one of its
//   workgroups finishes (encode and decode default, T = 8; both stream their 8 tiles branch-free
//   with stream_range instead of walking them here).
// MAP == MAP_BAND: XCD bands. The dispatcher deals workgroups round-robin over the 8 XCDs
//   (workgroup b runs on XCD b % 8, cdna_hip_programming.md T1), so the P = grid / 8 workgroups of
//   XCD x sweep chunksets x, x + 8, x + 16, ... one at a time, workgroup q = b / 8 taking tiles
//   q, q + P, q + 2P, ...: at any moment each XCD reads and writes one contiguous band of P tiles
//   (P x 4 KiB of every row) of one chunkset; the DRAM sees 8 x 26 wide streams instead of
//   512 x 26 narrow ones. Needs grid % 8 == 0 and n close to a multiple of 8 (launcher checks).
constexpr int MAP_BAND = -1;
constexpr uint32_t NXCD = 8;
// Encode: units of 4 tiles at every batch size. Units of 8 above 512 chunksets (the round-1 default
// until the tile loop went branch-free and the table builds conflict-free) measured +4.5 / +6 / +7 %
// at 600 / 1024 / 1639 chunksets on three boxes (tools/sessions/r01zz9, in-process A/B), and inside
// bench.py's buffers 4.61 vs 4.94-5.25 TB/s at 1639 — only in the DRAM's fast mode, which units of
// 8 reach less often, were they ahead (5.38 vs 5.22-5.25; r01zz10).
#ifndef DECDS_ENC_MAP
#define DECDS_ENC_MAP -4
#endif
// batches of at most DECDS_ENC_SMALL_N chunksets encode with DECDS_ENC_MAP_SMALL (finer-grained at
// the end of a short launch: units of 4 against 8 were -3 % at 103 chunksets on two boxes)
#ifndef DECDS_ENC_MAP_SMALL
#define DECDS_ENC_MAP_SMALL -4
#endif
#ifndef DECDS_ENC_SMALL_N
#define DECDS_ENC_SMALL_N 512
#endif
// tiny decode batches (single RepairingChunkSet repairs): a chunkset is only 256 tiles, 32 workgroups
// of 8; units of 2 / 4 tiles for n <= 2 / 4 keep about 256 workgroups (-7 % / -28 % at n = 2 / 4).
// Encode measured slower with smaller units there (units of 1 / 2: +40…+90 % at n = 1 / 2).
#ifndef DECDS_TINY_MAPS
#define DECDS_TINY_MAPS 1
#endif
#ifndef DECDS_DEC_MAP
#define DECDS_DEC_MAP -8
#endif
#ifndef DECDS_ENC_SHARE
#define DECDS_ENC_SHARE 500
#endif
#ifndef DECDS_DEC_SHARE
#define DECDS_DEC_SHARE 500
#endif
// Contiguous tile range of this workgroup. The grid is 2 workgroups per CU: workgroups
// [0, grid/2) are dispatched first (one per CU) and their waves are older than those of their CU
// partner in [grid/2, grid); the SIMDs arbitrate by age, so the first half runs faster
// (per-wave stamps, tools/tracebench.py: 8-17 % at n = 103 / 1639). SHARE (per mille) is the part
// of the tiles the first half takes, so both halves finish together (500 = equal ranges).
template <uint32_t SHARE>
__device__ __forceinline__ void tile_range(size_t n, uint32_t &t0, uint32_t &t1) {
    const uint64_t total = (uint64_t)n * TILES_PER_CS;
    const uint32_t h = gridDim.x / 2, b = blockIdx.x;
    if (SHARE == 500 || (gridDim.x & 1u)) {
        t0 = (uint32_t)(total * b / gridDim.x);
        t1 = (uint32_t)(total * (b + 1) / gridDim.x);
    } else {
        const uint64_t first = total * SHARE / 1000;
        if (b < h) {
            t0 = (uint32_t)(first * b / h);
            t1 = (uint32_t)(first * (b + 1) / h);
        } else {
            t0 = (uint32_t)(first + (total - first) * (b - h) / h);
            t1 = (uint32_t)(first + (total - first) * (b - h + 1) / h);
        }
    }
}

// Non-persistent workgroup -> position in the batch. The dispatcher deals workgroups round-robin
// over the 8 XCDs (b runs on XCD b % 8). With REMAP each XCD takes its own part of the batch
// instead: DECDS_XCD_CHUNK = 0 one contiguous eighth (its q-th workgroup the q-th of that eighth,
// rotated by SKEW x x workgroups); C > 0 runs of C consecutive workgroups dealt to the XCDs in turn
// (C = 32: one chunkset per XCD at a time, the XCDs on neighbouring chunksets).
#ifndef DECDS_ENC_XCD_REMAP
#define DECDS_ENC_XCD_REMAP 1
#endif
#ifndef DECDS_DEC_XCD_REMAP
#define DECDS_DEC_XCD_REMAP 0
#endif
#ifndef DECDS_XCD_SKEW
#define DECDS_XCD_SKEW 0
#endif
#ifndef DECDS_XCD_CHUNK
#define DECDS_XCD_CHUNK 0
#endif
#ifndef DECDS_XCD_MODE
#define DECDS_XCD_MODE 0  // study variants: 1 odd XCDs sweep their eighth backwards, 2 from its middle
#endif
template <bool REMAP>
__device__ __forceinline__ uint32_t np_block() {
    const uint32_t g = gridDim.x, b = blockIdx.x, x = b % NXCD, q = b / NXCD;
    if constexpr (!REMAP) {
        return b;
    } else if constexpr (DECDS_XCD_CHUNK > 0) {
        constexpr uint32_t C = DECDS_XCD_CHUNK;
        if (b >= g - g % (NXCD * C)) return b;  // the ragged end keeps the dispatcher's order
        return ((q / C) * NXCD + x) * C + q % C;
    } else {
        const uint32_t per = g / NXCD, rem = g % NXCD, cnt = per + (x < rem);
        uint32_t r = DECDS_XCD_SKEW ? (q + x * DECDS_XCD_SKEW) % cnt : q;
        if constexpr (DECDS_XCD_MODE == 1) r = (x & 1u) ? cnt - 1 - r : r;       // odd XCDs walk backwards
        if constexpr (DECDS_XCD_MODE == 2) r = (x & 1u) ? (r + cnt / 2) % cnt : r;  // odd XCDs start mid-range
        return x * per + (x < rem ? x : rem) + r;
    }
}

// Calls f(chunkset, tile, step, next) for this workgroup's tiles in order: when `next`, the
// workgroup's following tile is tile + step of the same chunkset (the ROLL prefetch target).
template <int MAP, uint32_t SHARE = 500, class Fn>
__device__ __forceinline__ void walk_tiles(size_t n, Fn &&f) {
    if constexpr (MAP == 0) {
        uint32_t t0, t1;
        tile_range<SHARE>(n, t0, t1);
        for (uint32_t t = t0; t < t1; t++) {
            const uint32_t cs = t / TILES_PER_CS, tile = t % TILES_PER_CS;
            f(cs, tile, 1u, t + 1 < t1 && tile + 1 < TILES_PER_CS);
        }
    } else if constexpr (MAP > 0) {
        static_assert(TILES_PER_CS % MAP == 0, "super-tile size");
        constexpr uint32_t SPC = TILES_PER_CS / MAP;
        const uint32_t total = (uint32_t)n * SPC;
        for (uint32_t st = blockIdx.x; st < total; st += gridDim.x) {
            const uint32_t cs = st / SPC, tb = (st % SPC) * MAP;
            for (uint32_t k = 0; k < (uint32_t)MAP; k++) f(cs, tb + k, 1u, k + 1 < (uint32_t)MAP);
        }
    } else if constexpr (MAP < MAP_BAND) {
        // non-persistent: workgroup b takes tiles [b*T, (b+1)*T) and exits (grid = tiles / T), so
        // the dispatcher sweeps the batch in order and refills CUs as workgroups finish
        constexpr uint32_t T = (uint32_t)(-MAP);
        const uint64_t total = (uint64_t)n * TILES_PER_CS;
        const uint32_t t0 = blockIdx.x * T, t1 = (uint32_t)(t0 + T < total ? t0 + T : total);
        for (uint32_t t = t0; t < t1; t++) {
            const uint32_t cs = t / TILES_PER_CS, tile = t % TILES_PER_CS;
            f(cs, tile, 1u, t + 1 < t1 && tile + 1 < TILES_PER_CS);
        }
    } else {
        static_assert(MAP == MAP_BAND, "work map");
        const uint32_t P = gridDim.x / NXCD, x = blockIdx.x % NXCD, q = blockIdx.x / NXCD;
        if (q >= P) return;
        for (uint32_t cs = x; cs < n; cs += NXCD)
            for (uint32_t tile = q; tile < TILES_PER_CS; tile += P) f(cs, tile, P, tile + P < TILES_PER_CS);
    }
}

// Column phase: lane blocks cover payload columns from `phase` on (phase < 16, chosen by the
// launcher so that rows with a 16-byte-aligned pitch are read / written on 16-byte boundaries); the
// wave owning tile 0 does the edge columns byte by byte: e < phase is column e, the rest the columns
// after the last block.
// Piece 9's main columns must stay below CS - 9L (its marker and padding are edge columns), so a
// phase above 7 gives up one block: 33 edge columns instead of 17.
constexpr uint32_t MAX_FULL_PHASE = (uint32_t)(CS - (K - 1) * L) - MAIN_COLS;
static_assert(MAX_FULL_PHASE == 7, "layout");
__device__ __forceinline__ uint32_t main_blocks(uint32_t phase) { return MAIN_BLOCKS - (phase > MAX_FULL_PHASE); }
__device__ __forceinline__ uint32_t edge_cols(uint32_t phase) { return (uint32_t)L - main_blocks(phase) * COLS_PER_LANE; }
__device__ __forceinline__ uint32_t edge_col(uint32_t e, uint32_t phase) {
    return e < phase ? e : main_blocks(phase) * COLS_PER_LANE + e;
}

// One tile for this lane: inputs were prefetched by the previous tile when `have` (ROLL), else
// they are loaded now; `next` says whether the following tile is tile + step of this chunkset.
template <class T, int NIN, int NOUT>
__device__ __forceinline__ void stream_tile(const uint8_t *lds, uint32_t laneoff, uint32_t tile, uint32_t step,
                                            bool next, uint32_t phase, const uint8_t *ibase, const uint32_t (&ioff)[NIN],
                                            uint8_t *obase, const uint32_t (&ooff)[NOUT], uint4 (&x)[NIN],
                                            bool &have) {
    if constexpr (T::SYNC == 1) __builtin_amdgcn_s_barrier();  // the 4 waves start the tile together
    const uint32_t block = tile * TILE_BLOCKS + threadIdx.x;
    const uint32_t nmain = main_blocks(phase);
    const bool active = block < nmain;
    if (!(T::ROLL && have) && active) load_block<T, NIN>(x, ibase, ioff, block * COLS_PER_LANE + phase);
    have = next;
    const uint32_t nblock = block + step * TILE_BLOCKS;
    // branch-free prefetch: lanes with no next block re-load their own block (an L2 hit)
    const uint32_t ncol0 = (have && nblock < nmain ? nblock : block) * COLS_PER_LANE + phase;
    if (active)
        combine_block<T, NIN, NOUT>(lds, laneoff, x, obase, ooff, block * COLS_PER_LANE + phase, ibase, ioff, ncol0);
}

// Tiles [ta, tb) of one chunkset, branch-free (ROLL builds only): lanes past the last block use
// OOB_COL, so no lane branches. The loop is entered after the first tile's loads AND NOUT dropped
// stores, the same memory-counter picture as every later tile (NIN prefetched loads, then NOUT
// stores). With a branch around the streaming code, or a reload path inside the loop, hipcc's
// wait-count pass merges paths that issued no stores and waits with vmcnt(NIN-1) for the next
// tile's first input: every tile then waited for the previous tile's stores as well; here it waits
// for the inputs only.
template <class T, int NIN, int NOUT>
__device__ __forceinline__ void stream_range(const uint8_t *lds, uint32_t laneoff, uint32_t ta, uint32_t tb,
                                             uint32_t phase, const uint8_t *ibase, const uint32_t (&ioff)[NIN],
                                             uint8_t *obase, const uint32_t (&ooff)[NOUT], uint4 (&x)[NIN]) {
    static_assert(T::ROLL && T::LAUX >= 0 && T::SAUX >= 0, "branch-free streaming needs prefetch and buffer ops");
    const uint32_t nmain = main_blocks(phase);
    auto col = [&](uint32_t t) {  // this lane's first column of tile t, or out of range
        const uint32_t block = t * TILE_BLOCKS + threadIdx.x;
        return t < tb && block < nmain ? block * COLS_PER_LANE + phase : OOB_COL;
    };
    load_block<T, NIN>(x, ibase, ioff, col(ta));
    asm volatile("" ::: "memory");  // keep the dropped stores after the loads, as in the loop
#pragma unroll
    for (int j = 0; j < NOUT; j++) strow<T::SAUX>(obase, OOB_COL + ooff[j], make_uint4(0, 0, 0, 0));
    // ta < tb (callers): a do-while, so no zero-trip guard lets hipcc sink the prologue loads
    // below the dropped stores. (Two tiles in flight — a second register set, swapped per tile —
    // needs 256 VGPRs and spills in decode; measured not worth it)
    uint32_t t = ta;
#pragma unroll 1
    do {
        if constexpr (T::SYNC == 1) __builtin_amdgcn_s_barrier();  // the 4 waves start each tile together
        combine_block<T, NIN, NOUT>(lds, laneoff, x, obase, ooff, col(t), ibase, ioff, col(t + 1));
    } while (++t < tb);
}

// Timing-study builds only (DECDS_TIMING_TRACE): every wave stamps its start and end with the
// 100 MHz real-time counter; decds_debug_trace copies the stamps out (kernel 0 encode, 1 decode).
#ifdef DECDS_TIMING_TRACE
constexpr uint32_t TRACE_WAVES = 65536;  // non-persistent launches: 128 waves per chunkset
__device__ uint64_t g_trace[2][2 * TRACE_WAVES];
#define TRACE_BEGIN(k)                                                                              \
    const uint32_t trace_w_ = blockIdx.x * (WG / 64) + threadIdx.x / 64;                            \
    if ((threadIdx.x & 63u) == 0 && trace_w_ < TRACE_WAVES) g_trace[k][2 * trace_w_] = __builtin_amdgcn_s_memrealtime()
#define TRACE_END(k) \
    if ((threadIdx.x & 63u) == 0 && trace_w_ < TRACE_WAVES) g_trace[k][2 * trace_w_ + 1] = __builtin_amdgcn_s_memrealtime()
#else
#define TRACE_BEGIN(k)
#define TRACE_END(k)
#endif

template <int MAP>
__global__ __launch_bounds__(WG, WAVES_PER_SIMD) __attribute__((amdgpu_waves_per_eu(WAVES_PER_SIMD, WAVES_PER_SIMD)))
void rlnc_encode_kernel(const uint8_t *__restrict__ src, size_t n, const uint8_t *__restrict__ coeffs,
                        uint8_t *__restrict__ dst, size_t pitch, uint32_t phase, uint32_t poly, uint32_t marker) {
    TRACE_BEGIN(0);
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t laneoff = (lane & 15u) * 16u;
    uint32_t ioff[K], ooff[N];
#pragma unroll
    for (int i = 0; i < (int)K; i++) ioff[i] = (uint32_t)(i * L);              // piece i of the padded chunkset
#pragma unroll
    for (int j = 0; j < (int)N; j++) ooff[j] = (uint32_t)(j * pitch + K);      // payload of coded row j
    uint32_t cur = 0xFFFFFFFFu;
    const uint8_t *ibase = src;
    uint8_t *obase = dst;
    const uint8_t *M = coeffs;
    uint4 x[K];
    if constexpr (DECDS_ENC_BF && (MAP == 0 || MAP < MAP_BAND)) {
        // one chunkset segment [t0, te): rebuild the tables, then stream it branch-free
        auto segment = [&](uint32_t t0, uint32_t te) {
            const uint32_t cs = t0 / TILES_PER_CS, tile0 = t0 % TILES_PER_CS;
            M = coeffs + (size_t)cs * N * K;
            const uint32_t cw = table_coeffs<K, N>(M, K);
            lds_barrier();
            build_tables<K, N>(lds, cw, poly);
            lds_barrier();
            ibase = src + (size_t)cs * CS;
            obase = dst + (size_t)cs * N * pitch;
            if (tile0 == 0) {  // the whole workgroup: one pass over the edge columns
                for (uint32_t idx = threadIdx.x; idx < N * K; idx += WG) obase[(idx / K) * pitch + idx % K] = M[idx];
                for (uint32_t idx = threadIdx.x; idx < edge_cols(phase) * N; idx += WG) {
                    const uint32_t j = idx % N, col = edge_col(idx / N, phase);
                    uint32_t y = 0;
#pragma unroll
                    for (uint32_t i = 0; i < K; i++) {
                        const uint64_t p = (uint64_t)i * L + col;
                        const uint32_t xv = p < CS ? ibase[p] : (p == CS ? marker : 0u);
                        y ^= tbl_mul(lds, i, j, xv);
                    }
                    obase[j * pitch + K + col] = (uint8_t)y;
                }
            }
            stream_range<EncBfTune, K, N>(lds, laneoff, tile0, te - cs * TILES_PER_CS, phase, ibase, ioff, obase, ooff,
                                          x);
        };
        auto walk_range = [&](uint32_t t0, uint32_t t1) {
            while (t0 < t1) {
                const uint32_t cs_end = (t0 / TILES_PER_CS + 1) * TILES_PER_CS;
                const uint32_t te = cs_end < t1 ? cs_end : t1;
                segment(t0, te);
                t0 = te;
            }
        };
        if constexpr (MAP == 0) {
            uint32_t t0, t1;
            tile_range<DECDS_ENC_SHARE>(n, t0, t1);
            walk_range(t0, t1);
        } else if constexpr (MAP < MAP_BAND) {
            // non-persistent: T = -MAP tiles, then exit
            const uint64_t total = (uint64_t)n * TILES_PER_CS;
            const uint32_t t0 = np_block<DECDS_ENC_XCD_REMAP>() * (uint32_t)(-MAP);
            walk_range(t0, (uint32_t)(t0 - MAP < total ? t0 - MAP : total));
        }
        TRACE_END(0);
        return;
    }
    bool have = false;
    [[maybe_unused]] bool built = false;
    walk_tiles<MAP, DECDS_ENC_SHARE>(n, [&](uint32_t cs, uint32_t tile, uint32_t step, bool next) {
        if (cs != cur) {
            cur = cs;
            have = false;
            M = coeffs + (size_t)cs * N * K;
            const uint32_t cw = table_coeffs<K, N>(M, K);
#ifdef DECDS_TIMING_NOREBUILD  // timing study only: keep the first chunkset's tables (wrong output)
            if (!built)
#endif
            {
                lds_barrier();
                build_tables<K, N>(lds, cw, poly);
                lds_barrier();
                built = true;
            }
            ibase = src + (size_t)cs * CS;
            obase = dst + (size_t)cs * N * pitch;
        }
        if (tile == 0) {
            // coding-vector prefix of the 16 full coded pieces (rlnc layout: cv || payload)
            for (uint32_t idx = threadIdx.x; idx < N * K; idx += WG) obase[(idx / K) * pitch + idx % K] = M[idx];
            // the edge columns (edge_col): piece 9 carries the boundary marker, then zero padding
            for (uint32_t idx = threadIdx.x; idx < edge_cols(phase) * N; idx += WG) {
                const uint32_t j = idx % N, col = edge_col(idx / N, phase);
                uint32_t y = 0;
#pragma unroll
                for (uint32_t i = 0; i < K; i++) {
                    const uint64_t p = (uint64_t)i * L + col;
                    const uint32_t xv = p < CS ? ibase[p] : (p == CS ? marker : 0u);
                    y ^= tbl_mul(lds, i, j, xv);
                }
                obase[j * pitch + K + col] = (uint8_t)y;
            }
        }
        stream_tile<EncTune, K, N>(lds, laneoff, tile, step, next, phase, ibase, ioff, obase, ooff, x, have);
    });
    TRACE_END(0);
}

template <int MAP>
__global__ __launch_bounds__(WG, WAVES_PER_SIMD) __attribute__((amdgpu_waves_per_eu(WAVES_PER_SIMD, WAVES_PER_SIMD)))
void rlnc_decode_kernel(const uint8_t *__restrict__ coded, size_t pitch, size_t n, const RepairPlan *__restrict__ plan,
                        uint8_t *__restrict__ dst, int32_t *__restrict__ status, uint32_t phase, uint32_t poly,
                        uint32_t marker) {
    TRACE_BEGIN(1);
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t laneoff = (lane & 15u) * 16u;
    uint32_t ioff[K], ooff[K];
#pragma unroll
    for (int i = 0; i < (int)K; i++) ooff[i] = (uint32_t)(i * L);
#pragma unroll
    for (int k = 0; k < (int)K; k++) ioff[k] = 0;
    uint32_t cur = 0xFFFFFFFFu;
    bool ready = false;
    const uint8_t *ibase = coded;
    uint8_t *obase = dst;
    uint4 x[K];
    if constexpr (MAP < MAP_BAND) {
        // Non-persistent: this workgroup's T tiles lie in one chunkset, streamed branch-free
        constexpr uint32_t T = (uint32_t)(-MAP);
        static_assert(TILES_PER_CS % T == 0, "a workgroup's tiles stay in one chunkset");
        using DT = Tune<DecTune::ASM, true, DecTune::LAUX < 0 ? 0 : DecTune::LAUX, DecTune::SAUX < 0 ? 0 : DecTune::SAUX,
                        DecTune::SYNC>;
        const uint32_t t0 = np_block<DECDS_DEC_XCD_REMAP>() * T, cs = t0 / TILES_PER_CS, tile0 = t0 % TILES_PER_CS;
        if (cs >= n) return;
        const uint32_t *pw = reinterpret_cast<const uint32_t *>(plan + cs);
        const uint32_t w0 = __builtin_amdgcn_readfirstlane(pw[0]);
        const uint32_t w1 = __builtin_amdgcn_readfirstlane(pw[1]);
        const uint32_t w2 = __builtin_amdgcn_readfirstlane(pw[2]);
        if (((w2 >> 16) & 0xFFu) != K) return;  // RepairPlan::rank at byte 10: not ready
        build_tables<K, K>(lds, table_coeffs<K, K>(plan[cs].inv, K), poly);
        lds_barrier();
        const uint32_t sel[K] = {w0 & 0xFFu, (w0 >> 8) & 0xFFu, (w0 >> 16) & 0xFFu, w0 >> 24,
                                 w1 & 0xFFu, (w1 >> 8) & 0xFFu, (w1 >> 16) & 0xFFu, w1 >> 24,
                                 w2 & 0xFFu, (w2 >> 8) & 0xFFu};
#pragma unroll
        for (int k = 0; k < (int)K; k++) ioff[k] = (uint32_t)(sel[k] * pitch + K);
        ibase = coded + (size_t)cs * N * pitch;
        obase = dst + (size_t)cs * CS;
        if (tile0 == 0) {  // the whole workgroup: one pass over the edge columns
            // the edge columns (edge_col); piece 9's must decode to marker || zeros (rlnc
            // get_decoded_data strips them; a mismatch is a repairing failure)
            bool ok = true;
            for (uint32_t idx = threadIdx.x; idx < edge_cols(phase) * K; idx += WG) {
                const uint32_t i = idx % K, col = edge_col(idx / K, phase);
                uint32_t z = 0;
#pragma unroll
                for (uint32_t k = 0; k < K; k++) z ^= tbl_mul(lds, k, i, ibase[ioff[k] + col]);
                const uint64_t p = (uint64_t)i * L + col;
                if (p < CS)
                    obase[p] = (uint8_t)z;
                else
                    ok &= z == (p == CS ? marker : 0u);
            }
            if (__any(!ok) && lane == 0) status[cs] = 6;  // DECDS_ERR_CHUNKSET_REPAIRING_FAILED
        }
        stream_range<DT, K, K>(lds, laneoff, tile0, tile0 + T, phase, ibase, ioff, obase, ooff, x);
        TRACE_END(1);
        return;
    }
    bool have = false;
    [[maybe_unused]] bool built = false;
    walk_tiles<MAP, DECDS_DEC_SHARE>(n, [&](uint32_t cs, uint32_t tile, uint32_t step, bool next) {
        if (cs != cur) {
            cur = cs;
            have = false;
            // plan words are wave-uniform: keep them in SGPRs
            const uint32_t *pw = reinterpret_cast<const uint32_t *>(plan + cs);
            const uint32_t w0 = __builtin_amdgcn_readfirstlane(pw[0]);
            const uint32_t w1 = __builtin_amdgcn_readfirstlane(pw[1]);
            const uint32_t w2 = __builtin_amdgcn_readfirstlane(pw[2]);
            ready = ((w2 >> 16) & 0xFFu) == K;  // RepairPlan::rank at byte 10
            if (ready) {
                const uint32_t cw = table_coeffs<K, K>(plan[cs].inv, K);
#ifdef DECDS_TIMING_NOREBUILD  // timing study only: keep the first chunkset's tables (wrong output)
                if (!built)
#endif
                {
                    lds_barrier();
                    build_tables<K, K>(lds, cw, poly);
                    lds_barrier();
                    built = true;
                }
                const uint32_t sel[K] = {w0 & 0xFFu, (w0 >> 8) & 0xFFu, (w0 >> 16) & 0xFFu, w0 >> 24,
                                         w1 & 0xFFu, (w1 >> 8) & 0xFFu, (w1 >> 16) & 0xFFu, w1 >> 24,
                                         w2 & 0xFFu, (w2 >> 8) & 0xFFu};
#pragma unroll
                for (int k = 0; k < (int)K; k++) ioff[k] = (uint32_t)(sel[k] * pitch + K);
                ibase = coded + (size_t)cs * N * pitch;
                obase = dst + (size_t)cs * CS;
            }
        }
        if (!ready) return;
        if (tile == 0) {
            // the edge columns (edge_col); piece 9's must decode to marker || zeros (rlnc
            // get_decoded_data strips them; a mismatch is a repairing failure)
            bool ok = true;
            for (uint32_t idx = threadIdx.x; idx < edge_cols(phase) * K; idx += WG) {
                const uint32_t i = idx % K, col = edge_col(idx / K, phase);
                uint32_t z = 0;
#pragma unroll
                for (uint32_t k = 0; k < K; k++) z ^= tbl_mul(lds, k, i, ibase[ioff[k] + col]);
                const uint64_t p = (uint64_t)i * L + col;
                if (p < CS)
                    obase[p] = (uint8_t)z;
                else
                    ok &= z == (p == CS ? marker : 0u);
            }
            if (__any(!ok) && lane == 0) status[cs] = 6;  // DECDS_ERR_CHUNKSET_REPAIRING_FAILED
        }
        stream_tile<DecTune, K, K>(lds, laneoff, tile, step, next, phase, ibase, ioff, obase, ooff, x, have);
    });
    TRACE_END(1);
}

// ---- warp-specialised streaming ---------------------------------------------------------------
// One 512-thread workgroup per CU owning the whole 160 KiB of LDS: the 80 KiB nibble tables plus
// two 40 KiB input buffers (10 rows x 256 lane blocks x 16 B). Waves 0-3 ("memory") only move the
// inputs of upcoming tiles from HBM into the free buffer (one tile in registers, one being written
// to LDS); waves 4-7 ("compute") read the current tile from LDS, do the lookups and store the
// outputs. One workgroup barrier per tile hands the buffers over, so each tile's 10 x 4 KiB of
// loads and 16 x 4 KiB of stores leave the CU together, as in the in-step memory pattern that
// tools/patbench.hip measured 5-10 % faster than waves drifting apart.
// ENC: in = chunksets, out = coded rows (coeffs give the tables). !ENC: in = coded rows, out =
// chunksets, the plan gives the tables, the survivors' rows and readiness.
constexpr uint32_t WS_WG = 512;
constexpr uint32_t WS_ROW = TILE_BLOCKS * 16;        // 4 KiB: one input row of a tile
constexpr uint32_t WS_BUF = K * WS_ROW;              // 40 KiB
constexpr uint32_t WS_LDS = LDS_BYTES + 2 * WS_BUF;  // 160 KiB
#ifndef DECDS_WS_ENC_TUNE
#define DECDS_WS_ENC_TUNE true, false, -1, -1
#endif
#ifndef DECDS_WS_DEC_TUNE
#define DECDS_WS_DEC_TUNE true, false, -1, 2
#endif
using WsEncTune = Tune<DECDS_WS_ENC_TUNE>;
using WsDecTune = Tune<DECDS_WS_DEC_TUNE>;

// where chunkset cs's input rows live: encode pieces i*L of the chunkset; decode the payloads of
// the accepted coded rows (plan sel). Returns whether the chunkset is processed at all.
template <bool ENC>
__device__ __forceinline__ bool ws_source(uint32_t cs, const uint8_t *in, size_t pitch, const RepairPlan *plan,
                                          const uint8_t *&base, uint32_t (&off)[K]) {
    if constexpr (ENC) {
        base = in + (size_t)cs * CS;
#pragma unroll
        for (int i = 0; i < (int)K; i++) off[i] = (uint32_t)(i * L);
        return true;
    } else {
        const uint32_t *pw = reinterpret_cast<const uint32_t *>(plan + cs);
        const uint32_t w0 = __builtin_amdgcn_readfirstlane(pw[0]);
        const uint32_t w1 = __builtin_amdgcn_readfirstlane(pw[1]);
        const uint32_t w2 = __builtin_amdgcn_readfirstlane(pw[2]);
        const uint32_t sel[K] = {w0 & 0xFFu, (w0 >> 8) & 0xFFu, (w0 >> 16) & 0xFFu, w0 >> 24,
                                 w1 & 0xFFu, (w1 >> 8) & 0xFFu, (w1 >> 16) & 0xFFu, w1 >> 24,
                                 w2 & 0xFFu, (w2 >> 8) & 0xFFu};
        base = in + (size_t)cs * N * pitch;
#pragma unroll
        for (int k = 0; k < (int)K; k++) off[k] = (uint32_t)(sel[k] * pitch + K);
        return ((w2 >> 16) & 0xFFu) == K;  // RepairPlan::rank at byte 10
    }
}

template <bool ENC>
__global__ __launch_bounds__(WS_WG) __attribute__((amdgpu_waves_per_eu(2, 2)))
void rlnc_ws_kernel(const uint8_t *__restrict__ in, size_t n, const uint8_t *__restrict__ coeffs,
                    const RepairPlan *__restrict__ plan, uint8_t *__restrict__ out, size_t pitch,
                    int32_t *__restrict__ status, uint32_t poly, uint32_t marker) {
    using T = std::conditional_t<ENC, WsEncTune, WsDecTune>;
    constexpr int NOUT = ENC ? (int)N : (int)K;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const bool mem = wave < 4;
    const uint32_t slot = (wave & 3u) * 64u + lane;  // lane block of the tile this lane moves / computes
    const uint32_t laneoff = (lane & 15u) * 16u;
    uint32_t t0, t1;
    tile_range<500>(n, t0, t1);
    if (t0 >= t1) return;

    // memory side: chunkset of the tile in flight, its rows, and the tile's inputs in registers
    uint32_t mcs = 0xFFFFFFFFu;
    bool mready = false;
    const uint8_t *mbase = in;
    uint32_t moff[K];
    uint4 x[K];
    auto mem_load = [&](uint32_t t) {
        const uint32_t cs = t / TILES_PER_CS, block = (t % TILES_PER_CS) * TILE_BLOCKS + slot;
        if (cs != mcs) {
            mcs = cs;
            mready = ws_source<ENC>(cs, in, pitch, plan, mbase, moff);
        }
        if (mready && block < MAIN_BLOCKS) load_block<T, K>(x, mbase, moff, block * COLS_PER_LANE);
    };
    auto mem_stage = [&](uint32_t t) {  // x (tile t) -> buffer t & 1
        const uint32_t block = (t % TILES_PER_CS) * TILE_BLOCKS + slot;
        if (mready && block < MAIN_BLOCKS) {
            uint8_t *b = lds + LDS_BYTES + (t & 1u) * WS_BUF + slot * 16u;
#pragma unroll
            for (int i = 0; i < (int)K; i++) *reinterpret_cast<uint4 *>(b + i * WS_ROW) = x[i];
        }
    };

    // compute side: chunkset whose tables are built, and where its outputs go
    uint32_t cur = 0xFFFFFFFFu;
    bool ready = false;
    const uint8_t *ibase = in;  // for the byte-wise tail columns
    uint32_t ioff[K];
    uint8_t *obase = out;
    uint32_t ooff[NOUT];
#pragma unroll
    for (int j = 0; j < NOUT; j++) ooff[j] = ENC ? (uint32_t)(j * pitch + K) : (uint32_t)(j * L);

    if (mem) {
        mem_load(t0);
        mem_stage(t0);
        if (t0 + 1 < t1) mem_load(t0 + 1);
    }
    for (uint32_t t = t0; t < t1; t++) {
        const uint32_t cs = t / TILES_PER_CS, tile = t % TILES_PER_CS;
        if (cs != cur) {  // every wave takes part in the table rebuild
            cur = cs;
            ready = ws_source<ENC>(cs, in, pitch, plan, ibase, ioff);
            if (ready) {
                const uint32_t cw = ENC ? table_coeffs<K, N>(coeffs + (size_t)cs * N * K, K)
                                        : table_coeffs<K, K>(plan[cs].inv, K);
                lds_barrier();  // the previous chunkset's lookups are done
                build_tables<K, NOUT>(lds, cw, poly);
                obase = out + (size_t)cs * (ENC ? N * pitch : CS);
            }
        }
        lds_barrier();  // tables built; buffer t & 1 staged; buffer (t + 1) & 1 no longer read
        if (mem) {
            if (t + 1 < t1) mem_stage(t + 1);
            if (t + 2 < t1) mem_load(t + 2);
        } else if (ready) {
            if (tile == 0 && wave == 4) {
                if constexpr (ENC) {
                    // coding-vector prefix of the 16 full coded pieces (rlnc layout: cv || payload)
                    const uint8_t *M = coeffs + (size_t)cs * N * K;
                    for (uint32_t idx = lane; idx < N * K; idx += 64) obase[(idx / K) * pitch + idx % K] = M[idx];
                    // last 17 columns: piece 9 carries the boundary marker, then zero padding
                    for (uint32_t idx = lane; idx < TAIL_COLS * N; idx += 64) {
                        const uint32_t j = idx % N, col = MAIN_COLS + idx / N;
                        uint32_t y = 0;
#pragma unroll
                        for (uint32_t i = 0; i < K; i++) {
                            const uint64_t p = (uint64_t)i * L + col;
                            const uint32_t xv = p < CS ? ibase[p] : (p == CS ? marker : 0u);
                            y ^= tbl_mul(lds, i, j, xv);
                        }
                        obase[j * pitch + K + col] = (uint8_t)y;
                    }
                } else {
                    // last 17 columns; piece 9's must decode to marker || zeros
                    bool ok = true;
                    for (uint32_t idx = lane; idx < TAIL_COLS * K; idx += 64) {
                        const uint32_t i = idx % K, col = MAIN_COLS + idx / K;
                        uint32_t z = 0;
#pragma unroll
                        for (uint32_t k = 0; k < K; k++) z ^= tbl_mul(lds, k, i, ibase[ioff[k] + col]);
                        const uint64_t p = (uint64_t)i * L + col;
                        if (p < CS)
                            obase[p] = (uint8_t)z;
                        else
                            ok &= z == (p == CS ? marker : 0u);
                    }
                    if (__any(!ok) && lane == 0) status[cs] = 6;  // DECDS_ERR_CHUNKSET_REPAIRING_FAILED
                }
            }
            const uint32_t block = tile * TILE_BLOCKS + slot;
            if (block < MAIN_BLOCKS) {
                const uint8_t *b = lds + LDS_BYTES + (t & 1u) * WS_BUF + slot * 16u;
                uint4 xin[K];
#pragma unroll
                for (int i = 0; i < (int)K; i++) xin[i] = *reinterpret_cast<const uint4 *>(b + i * WS_ROW);
                // the hand-pipelined lookups count only their own LDS reads in flight
                __builtin_amdgcn_s_waitcnt(0xC07F);
                combine_block<T, K, NOUT>(lds, laneoff, xin, obase, ooff, block * COLS_PER_LANE, ibase, ioff,
                                          block * COLS_PER_LANE);
            }
        }
    }
}

#ifdef DECDS_TIMING_TRACE
extern "C" int decds_debug_trace(int kernel, uint64_t *out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_trace), sizeof(g_trace[0]), (size_t)kernel * sizeof(g_trace[0]),
                                    hipMemcpyDeviceToHost);
}
#endif

// One wave per chunkset. Replays rlnc's incremental rank test over the candidates' 10-byte coding
// vectors in arrival order (chunkset.rs:173-184: a piece is accepted iff it raises the rank;
// after rank 10 every further piece is "ready to repair") and, in the same pass, inverts the
// accepted vectors. Each basis row is augmented: lanes 0..9 hold its coefficient part (kept in
// reduced row-echelon form), lanes 10..19 the combination of accepted raw vectors it equals (the
// k-th accepted vector enters as unit vector k). Because the coefficient part is RREF, the factors
// that reduce a new row against the basis are the new row's own entries at the basis pivots, so
// all reductions of one step are independent (ILP across the basis instead of a serial chain).
// At rank 10 the coefficient parts are unit vectors e_piv, so B = E·R = P and R^-1 = Pᵀ·E: row i
// of the inverse is the combination part of the basis row whose pivot is column i.
// Products use log / exp tables of the generator `gen` in LDS: x * f = exp[log x + log f] — one
// table read per product, and the products of one step are independent reads (a bit-serial
// multiply by a wave-uniform factor is a chain of 8 scalar branches).
__global__ __launch_bounds__(64) void rlnc_plan_kernel(const uint8_t *__restrict__ coded, size_t pitch, size_t n,
                                                       const uint8_t *__restrict__ cand,
                                                       RepairPlan *__restrict__ plan,
                                                       int8_t *__restrict__ verdicts,
                                                       int32_t *__restrict__ status, uint32_t poly,
                                                       uint32_t gen) {
    const size_t cs = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    const bool col = lane < K;
    // the arrival order, and the 10-byte coding vector of every coded row of the chunkset (lane
    // c < 10 loads byte c of rows 0..15): both in flight while the tables below are built
    const uint32_t my_cand = lane < N ? cand[cs * N + lane] : (uint32_t)DECDS_NO_CANDIDATE_U8;
    uint32_t rowcv[N];
#pragma unroll
    for (int r = 0; r < (int)N; r++) rowcv[r] = col ? coded[(cs * N + r) * pitch + lane] : 0u;
    // exp[i] = gen^i for i < 510 (doubled: exp[log a + log b] needs no reduction mod 255),
    // log[gen^i] = i. Lane l starts at gen^(4l) (square-and-multiply) and steps 4 times.
    __shared__ uint8_t s_exp[512], s_log[256], s_cv[N * 16];
    {
        uint32_t v = 1, b = gen;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if ((4 * lane >> k) & 1u) v = gf_mul(v, b, poly);
            b = gf_mul(b, b, poly);
        }
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
            const uint32_t i = 4 * lane + q;
            if (i < 255) {
                s_exp[i] = (uint8_t)v;
                s_exp[i + 255] = (uint8_t)v;
                s_log[v] = (uint8_t)i;
            }
            v = gf_mul(v, gen, poly);
        }
        if (lane == 0) s_log[0] = 0;  // log 0 is never used unmasked; keep the reads defined
    }
    if (col) {
#pragma unroll
        for (int r = 0; r < (int)N; r++) s_cv[r * 16 + lane] = (uint8_t)rowcv[r];
    }
    __syncthreads();
    // Every term below is computed unconditionally and masked by selects: no branch splits the
    // ten independent table reads of a step, so they are all in flight together.
    uint32_t basis[K], lgb[K], piv[K], sel[K];  // lgb[e] = log basis[e] (masked where basis[e] == 0)
#pragma unroll
    for (int e = 0; e < (int)K; e++) basis[e] = lgb[e] = piv[e] = sel[e] = 0;
    uint32_t rank = 0;
    bool ended = false;
    int32_t my_verdict = -1;  // lane a < 16 keeps candidate a's verdict
#pragma unroll
#ifdef DECDS_TIMING_PLAN_SETUP  // timing study only: the setup without the candidate loop (wrong output)
    for (uint32_t a = 0; a < 0; a++) {
#else
    for (uint32_t a = 0; a < N; a++) {
#endif
        const uint32_t r = __builtin_amdgcn_readlane(my_cand, a);
        int32_t v;
        if (ended || r >= N) {
            ended = true;
            v = -1;
        } else if (rank == K) {
            v = 3;  // DECDS_ERR_CHUNKSET_READY_TO_REPAIR
        } else {
            const uint32_t cv = col ? s_cv[r * 16 + lane] : 0u;
            // augmented row [cv | unit(rank)] minus its projection on the basis
            uint32_t row = col ? cv : (lane == K + rank ? 1u : 0u);
#pragma unroll
            for (int e = 0; e < (int)K; e++) {
                const uint32_t f = e < (int)rank ? __builtin_amdgcn_readlane(cv, piv[e]) : 0u;
                const uint32_t t = s_exp[lgb[e] + s_log[f]];
                row ^= (f != 0 && basis[e] != 0) ? t : 0u;
            }
            const uint64_t nz = __ballot(col && row != 0);
            if (!nz) {
                v = 4;  // DECDS_ERR_CHUNK_DECODING_FAILED: piece not useful
            } else {
                const uint32_t p = __builtin_ctzll(nz);
                // row /= row[p]: log of the inverse = 255 - log (exp is doubled, so 255 is fine)
                const uint32_t linv = 255u - s_log[__builtin_amdgcn_readlane(row, p)];
                row = row ? s_exp[s_log[row] + linv] : 0u;
                const uint32_t lrow = s_log[row];
#pragma unroll
                for (int e = 0; e < (int)K; e++) {
                    const uint32_t f = e < (int)rank ? __builtin_amdgcn_readlane(basis[e], p) : 0u;
                    const uint32_t t = s_exp[lrow + s_log[f]];
                    basis[e] ^= (f != 0 && row != 0) ? t : 0u;
                }
#pragma unroll
                for (int e = 0; e < (int)K; e++) {
                    if (e == (int)rank) {
                        basis[e] = row;
                        piv[e] = p;
                        sel[e] = r;
                    }
                    lgb[e] = s_log[basis[e]];
                }
                rank++;
                v = 0;
            }
        }
        if (lane == a) my_verdict = v;
    }
    if (lane < N) verdicts[cs * N + lane] = (int8_t)my_verdict;
    RepairPlan *pl = plan + cs;
    if (lane == 0) pl->rank = (uint8_t)rank;
    if (rank < K) {
        if (lane == 0) status[cs] = 5;  // DECDS_ERR_CHUNKSET_NOT_YET_READY
        return;
    }
    // inverse row piv[e] = combination part of basis row e: lane 10 + k writes inv[piv[e]][k]
    if (lane >= K && lane < 2 * K) {
#pragma unroll
        for (int e = 0; e < (int)K; e++) pl->inv[piv[e] * K + (lane - K)] = (uint8_t)basis[e];
    }
    if (lane == 0) {
#pragma unroll
        for (int e = 0; e < (int)K; e++) pl->sel[e] = (uint8_t)sel[e];
        status[cs] = 0;
    }
}

__device__ __forceinline__ uint64_t splitmix_word(uint64_t seed, uint64_t w) {
    uint64_t z = seed + (w + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// byte_offset and dst are 8-byte aligned on the fast path (checked by the launcher)
__global__ void fill_random_words_kernel(uint64_t seed, uint64_t word0, uint64_t *dst, size_t nwords) {
    for (size_t w = (size_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords;
         w += (size_t)gridDim.x * blockDim.x)
        dst[w] = splitmix_word(seed, word0 + w);
}

__global__ void fill_random_bytes_kernel(uint64_t seed, uint64_t off, uint8_t *dst, size_t nbytes) {
    for (size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x; b < nbytes;
         b += (size_t)gridDim.x * blockDim.x) {
        const uint64_t p = off + b;
        dst[b] = (uint8_t)(splitmix_word(seed, p >> 3) >> (8 * (p & 7)));
    }
}

// ------------------------------------------------------------------------------ launchers ----
static uint32_t stream_grid(const LaunchGeom &g, size_t n) {
    const uint64_t tiles = (uint64_t)n * TILES_PER_CS;
    uint64_t grid = (uint64_t)g.num_cus * (g.wgs_per_cu == 1 ? 1 : WGS_PER_CU);
    return (uint32_t)(tiles < grid ? tiles : grid);
}

// The band walk needs whole XCD groups and a batch that splits evenly enough over the 8 XCDs
// (at most 5 % of XCD-rounds idle); other batches take the fallback map.
static bool band_ok(uint32_t grid, size_t n) {
    return grid >= NXCD && grid % NXCD == 0 && ((NXCD - n % NXCD) % NXCD) * 20 <= n;
}
constexpr int ENC_MAP_FALLBACK = 0, DEC_MAP_FALLBACK = 8;
#ifndef DECDS_ENC_WS
#define DECDS_ENC_WS 0
#endif
#ifndef DECDS_DEC_WS
#define DECDS_DEC_WS 0
#endif
// Column phase of the coded rows' payloads (edge_col): with a 16-byte-aligned pitch every row's
// payload (row + 10) has the same alignment, and blocks starting `phase` columns in are 16-byte
// aligned. Encode uses it (its 16 row stores aligned: -2..-3 %); decode measured slower with its 10
// row loads aligned (+3..+5 %) and keeps phase 0. Other pitches keep phase 0.
#ifndef DECDS_ENC_PHASE
#define DECDS_ENC_PHASE 1
#endif
#ifndef DECDS_DEC_PHASE
#define DECDS_DEC_PHASE 0
#endif
static uint32_t row_phase(bool on, const uint8_t *rows, size_t pitch) {
    if (!on || pitch % 16) return 0;
    return (uint32_t)((16 - ((uintptr_t)rows + K) % 16) % 16);
}

static uint32_t ws_grid(const LaunchGeom &g, size_t n) {  // one workgroup per CU
    const uint64_t tiles = (uint64_t)n * TILES_PER_CS;
    return (uint32_t)(tiles < (uint64_t)g.num_cus ? tiles : (uint64_t)g.num_cus);
}

hipError_t configure_kernels() {
    const void *fns[] = {reinterpret_cast<const void *>(rlnc_encode_kernel<DECDS_ENC_MAP>),
                         reinterpret_cast<const void *>(rlnc_encode_kernel<DECDS_ENC_MAP_SMALL>),
                         reinterpret_cast<const void *>(rlnc_decode_kernel<-2>),
                         reinterpret_cast<const void *>(rlnc_decode_kernel<-4>),
                         reinterpret_cast<const void *>(rlnc_encode_kernel<ENC_MAP_FALLBACK>),
                         reinterpret_cast<const void *>(rlnc_decode_kernel<DECDS_DEC_MAP>),
                         reinterpret_cast<const void *>(rlnc_decode_kernel<DEC_MAP_FALLBACK>)};
    for (const void *f : fns) {
        hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
        if (e != hipSuccess) return e;
    }
    if (DECDS_ENC_WS) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(rlnc_ws_kernel<true>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, WS_LDS);
        if (e != hipSuccess) return e;
    }
    if (DECDS_DEC_WS) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(rlnc_ws_kernel<false>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, WS_LDS);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_encode(const LaunchGeom &g, const uint8_t *src, size_t n, const uint8_t *coeffs,
                         uint8_t *dst, size_t pitch, uint32_t poly, uint32_t marker,
                         hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (DECDS_ENC_WS) {
        hipLaunchKernelGGL(rlnc_ws_kernel<true>, dim3(ws_grid(g, n)), dim3(WS_WG), WS_LDS, stream, src, n, coeffs,
                           (const RepairPlan *)nullptr, dst, pitch, (int32_t *)nullptr, poly, marker);
        return hipGetLastError();
    }
    const uint32_t phase = row_phase(DECDS_ENC_PHASE, dst, pitch);
    auto np = [&](auto map) {  // non-persistent launch, units of T = -MAP tiles
        constexpr int MAP = decltype(map)::value;
        constexpr uint32_t T = (uint32_t)(-MAP);
        hipLaunchKernelGGL(rlnc_encode_kernel<MAP>, dim3((uint32_t)((n * TILES_PER_CS + T - 1) / T)), dim3(WG),
                           LDS_BYTES, stream, src, n, coeffs, dst, pitch, phase, poly, marker);
        return hipGetLastError();
    };
    if (DECDS_ENC_MAP < MAP_BAND && DECDS_ENC_MAP_SMALL < MAP_BAND && n <= DECDS_ENC_SMALL_N)
        return np(std::integral_constant<int, DECDS_ENC_MAP_SMALL>{});
    uint32_t grid = stream_grid(g, n);
    if (DECDS_ENC_MAP < MAP_BAND) grid = (uint32_t)(((uint64_t)n * TILES_PER_CS + (-DECDS_ENC_MAP) - 1) / (-DECDS_ENC_MAP));
    if (DECDS_ENC_MAP == MAP_BAND && band_ok(grid & ~(NXCD - 1), n)) {
        grid &= ~(NXCD - 1);
        hipLaunchKernelGGL(rlnc_encode_kernel<DECDS_ENC_MAP>, dim3(grid), dim3(WG), LDS_BYTES, stream, src, n,
                           coeffs, dst, pitch, phase, poly, marker);
    } else if (DECDS_ENC_MAP != MAP_BAND) {
        hipLaunchKernelGGL(rlnc_encode_kernel<DECDS_ENC_MAP>, dim3(grid), dim3(WG), LDS_BYTES, stream, src, n,
                           coeffs, dst, pitch, phase, poly, marker);
    } else {
        hipLaunchKernelGGL(rlnc_encode_kernel<ENC_MAP_FALLBACK>, dim3(grid), dim3(WG), LDS_BYTES, stream, src, n,
                           coeffs, dst, pitch, phase, poly, marker);
    }
    return hipGetLastError();
}

hipError_t launch_repair_plan(const uint8_t *coded, size_t pitch, size_t n, const uint8_t *cand,
                              uint8_t *plan, int8_t *verdicts, int32_t *status, uint32_t poly,
                              uint32_t gen, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(rlnc_plan_kernel, dim3((uint32_t)n), dim3(64), 0, stream, coded,
                       pitch, n, cand, reinterpret_cast<RepairPlan *>(plan), verdicts, status, poly, gen);
    return hipGetLastError();
}

hipError_t launch_decode(const LaunchGeom &g, const uint8_t *coded, size_t pitch, size_t n,
                         const uint8_t *plan, uint8_t *dst, int32_t *status, uint32_t poly,
                         uint32_t marker, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const RepairPlan *pl = reinterpret_cast<const RepairPlan *>(plan);
    if (DECDS_DEC_WS) {
        hipLaunchKernelGGL(rlnc_ws_kernel<false>, dim3(ws_grid(g, n)), dim3(WS_WG), WS_LDS, stream, coded, n,
                           (const uint8_t *)nullptr, pl, dst, pitch, status, poly, marker);
        return hipGetLastError();
    }
    const uint32_t phase = row_phase(DECDS_DEC_PHASE, coded, pitch);
    auto np = [&](auto map) {  // non-persistent launch, units of T = -MAP tiles
        constexpr int MAP = decltype(map)::value;
        constexpr uint32_t T = (uint32_t)(-MAP);
        hipLaunchKernelGGL(rlnc_decode_kernel<MAP>, dim3((uint32_t)((n * TILES_PER_CS + T - 1) / T)), dim3(WG),
                           LDS_BYTES, stream, coded, pitch, n, pl, dst, status, phase, poly, marker);
        return hipGetLastError();
    };
    if (DECDS_DEC_MAP < MAP_BAND && DECDS_TINY_MAPS && n <= 2) return np(std::integral_constant<int, -2>{});
    if (DECDS_DEC_MAP < MAP_BAND && DECDS_TINY_MAPS && n <= 4) return np(std::integral_constant<int, -4>{});
    uint32_t grid = stream_grid(g, n);
    if (DECDS_DEC_MAP < MAP_BAND) grid = (uint32_t)(((uint64_t)n * TILES_PER_CS + (-DECDS_DEC_MAP) - 1) / (-DECDS_DEC_MAP));
    if (DECDS_DEC_MAP == MAP_BAND && band_ok(grid & ~(NXCD - 1), n)) {
        grid &= ~(NXCD - 1);
        hipLaunchKernelGGL(rlnc_decode_kernel<DECDS_DEC_MAP>, dim3(grid), dim3(WG), LDS_BYTES, stream, coded, pitch,
                           n, pl, dst, status, phase, poly, marker);
    } else if (DECDS_DEC_MAP != MAP_BAND) {
        hipLaunchKernelGGL(rlnc_decode_kernel<DECDS_DEC_MAP>, dim3(grid), dim3(WG), LDS_BYTES, stream, coded, pitch,
                           n, pl, dst, status, phase, poly, marker);
    } else {
        hipLaunchKernelGGL(rlnc_decode_kernel<DEC_MAP_FALLBACK>, dim3(grid), dim3(WG), LDS_BYTES, stream, coded,
                           pitch, n, pl, dst, status, phase, poly, marker);
    }
    return hipGetLastError();
}

hipError_t launch_fill_random(uint64_t seed, uint64_t byte_offset, uint8_t *dst, size_t nbytes,
                              hipStream_t stream) {
    if (nbytes == 0) return hipSuccess;
    if ((byte_offset & 7u) == 0 && (reinterpret_cast<uintptr_t>(dst) & 7u) == 0 && (nbytes & 7u) == 0) {
        const size_t nw = nbytes / 8;
        const uint32_t grid = (uint32_t)((nw + 255) / 256 < 8192 ? (nw + 255) / 256 : 8192);
        hipLaunchKernelGGL(fill_random_words_kernel, dim3(grid), dim3(256), 0, stream, seed, byte_offset / 8,
                           reinterpret_cast<uint64_t *>(dst), nw);
    } else {
        const uint32_t grid = (uint32_t)((nbytes + 255) / 256 < 8192 ? (nbytes + 255) / 256 : 8192);
        hipLaunchKernelGGL(fill_random_bytes_kernel, dim3(grid), dim3(256), 0, stream, seed, byte_offset, dst,
                           nbytes);
    }
    return hipGetLastError();
}

}  // namespace decds

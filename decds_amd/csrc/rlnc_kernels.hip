// rlnc_kernels.hip — gfx950 (MI355X / CDNA4) kernels for decds' RLNC chunkset codec.
//
// The hot path is one GF(2^8) linear-combination pass over a batch of chunksets:
//   encode (chunkset.rs:43-52, rlnc Encoder::code x16):   y_j = sum_i C[j][i] * piece_i,  j<16, i<10
//   decode (chunkset.rs:181-204, rlnc Decoder):           piece_i = sum_k D[i][k] * y_k,  D = C_sel^-1
// Both stream 1 MiB piece columns from HBM once and write the results once. The GF multiply by a
// chunkset-uniform coefficient is a table lookup: per input piece i and nibble half h an LDS table
//   T[i][h][n] = { C[j][i] * (n << 4h) : j = 0..15 }   (16 B: all outputs' products at once)
// so one ds_read_b128 gives the contribution of one input nibble to all 16 outputs. A table is 16
// rows x 16 B = 256 B = one pass over the 64 LDS banks: row n sits on banks 4n..4n+3. The 16 lanes
// of a ds_read_b128 lane group read rows of the same table, so two lanes either read the same row
// (identical addresses broadcast) or rows on disjoint banks: the data-dependent lookups are
// bank-conflict-free by construction (MI355X_MICROARCH.md §LDS) with no replicas — 5 KiB of tables
// per workgroup, built with 16 ds_write_b32 by 80 threads (round 1 replicated every row 16x:
// 80 KiB and ~3 µs of CU time per build, which made workgroups of fewer tiles lose, profiles/HISTORY.md §8).
// Per 16-column lane block: 10 unaligned 16-B loads, 320 conflict-free ds_read_b128, v_bitop3 XOR3
// accumulation into a 16x16 byte block (columns x outputs), a v_perm byte transpose, 16 (or 10)
// 16-B stores. No MFMA: this is byte-wise finite-field work, bounded by HBM bandwidth.
//
// Only the shipped configuration lives here, plus three study hooks that compile to nothing by default
// (DECDS_PHASE_TRACE: per-workgroup phase stamps of the encode sweep for tools/phasetrace.py;
// DECDS_STUDY_NO_EDGE: the encode without its edge pass, timing only; DECDS_STUDY_PATTERN: the
// kernels' memory pattern without their lookups — the pattern ceilings bench.py reports;
// DECDS_STUDY_ALIGNED_PIECES=1/2/3: piece i of a chunkset addressed at i * L rounded down to 256 bytes /
// at i * (L - 1) - 16 i / - 4 i in the streaming kernels, timing only — what the pieces' i-byte
// misalignment costs). The round-1 study variants
// (persistent walks, XCD bands, per-half work shares, per-tile barriers, the warp-specialised kernel)
// are in git history (tools/study/rlnc_kernels_r01_study.hip at a5d9101) with their measurements in
// profiles/HISTORY.md §8.
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <cstring>

#include <algorithm>
#include <atomic>
#include <utility>

#include "blake3_impl.h"
#include "commit_kernels.h"
#include "hip_status.h"
#include "rlnc_kernels.h"
#include "rlnc_layout.h"

namespace decds {

// ---- geometry ---------------------------------------------------------------------------------
constexpr uint32_t DECDS_NO_CANDIDATE_U8 = 0xFF;
constexpr uint32_t WG = 256;                                  // 4 waves
constexpr uint32_t TILE_BLOCKS = WG;                          // one 16-col block per lane per tile
constexpr uint32_t ROW_BYTES = 16;                            // one nibble row: 16 outputs' products
constexpr uint32_t TABLE_BYTES = 16 * ROW_BYTES;              // 16 nibble rows = 256 B = the 64 banks once
constexpr uint32_t LDS_BYTES = K * 2 * TABLE_BYTES;           // 5 KiB
constexpr uint32_t SWEEP_LDS = 2 * LDS_BYTES + 48;             // two table buffers + the next-tile slot + TailLds
constexpr uint32_t DEC_LDS = LDS_BYTES + 32;                   // one-tile decode: tables + TailLds
// (the tables sit at LDS address 0 of the dynamic area: the inline-asm ds_read_b128 lookups address
// them absolutely, so a kernel holding them must not declare static __shared__ variables — those
// would be placed first and move the dynamic area)

#ifndef DECDS_BUILD_XOR
#define DECDS_BUILD_XOR 1  // table builds in a bank-conflict-free row order (build_tables)
#endif
// encode lookup groups of 2 bytes (8 reads in flight per wave) against 4 (16 in flight): -1.0...-1.6 %
// encode time at 103-1639 chunksets (r05g, same 2 waves/SIMD); groups of 1 byte +4.5 %, also at the
// 3 waves/SIMD they make room for (167 VGPRs, r05g)
#ifndef DECDS_ENC_HB
#define DECDS_ENC_HB 2  // encode lookup group size (bytes of an input dword per group)
#endif
#ifndef DECDS_ENC_SMALL_HB
#define DECDS_ENC_SMALL_HB 2  // the same for the 8-column small-batch form (4 waves/SIMD: groups of 4 spill)
#endif
#ifndef DECDS_DEC_UNIT
#define DECDS_DEC_UNIT 1  // decode tiles per workgroup (+3...+11 % against 8 once the tables stopped being replicated, r02e)
#endif
#ifndef DECDS_PREFETCH_FIRST
#define DECDS_PREFETCH_FIRST 1  // 1: a decode workgroup's first tile loads are issued before its table build
#endif
constexpr uint32_t DEC_UNIT = DECDS_DEC_UNIT;
#ifndef DECDS_DEC_XCD_RUN
#define DECDS_DEC_XCD_RUN 8  // decode: consecutive tiles per XCD (1 = plain dispatch order)
#endif
constexpr uint32_t DEC_XCD_RUN = DECDS_DEC_XCD_RUN;
// The shipped work splits: the encode is one persistent sweep fed by a tile
// counter for every batch (0.69-0.73 of 8 TB/s at 103-1639 chunksets against 0.64-0.66 for round 2's
// non-persistent units of 4 tiles per XCD eighth, r02r; that form is in git history, rlnc_kernels.hip
// at 227db28); the decode runs non-persistent workgroups of one tile.

// A wave-uniform 64-bit value in SGPRs. __builtin_amdgcn_readfirstlane returns int: each half goes
// back through uint32_t, or a low half with bit 31 set would sign-extend into the high half (an
// address above 2 GiB within its 4 GiB window became 0xFFFFFFFF'xxxxxxxx: GPUTEST r02i).
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// Workgroup barrier for the LDS tables only: every wave's LDS accesses have completed, nothing
// else. __syncthreads() also drains each wave's outstanding global stores (a release fence).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0); vmcnt / expcnt left unconstrained
    __builtin_amdgcn_s_barrier();
}

// The 4 coefficient bytes thread p = 8i + 4h + q (< NIN*8) of build_tables combines:
// M[(4q + jj) * ldm + i], jj < 4 (zero for outputs >= NOUT and for idle threads).
template <int NIN, int NOUT>
__device__ __forceinline__ uint32_t table_coeffs(const uint8_t *M, uint32_t ldm, uint32_t ldi = 1) {
    static_assert(NIN * 8 <= (int)WG, "one coefficient word per thread");
    const uint32_t p = threadIdx.x;
    uint32_t w = 0;
    if (p < NIN * 8) {
        const uint32_t q = p & 3u, i = p >> 3;
#pragma unroll
        for (uint32_t jj = 0; jj < 4; jj++)
            if (4 * q + jj < (uint32_t)NOUT) w |= (uint32_t)M[(4 * q + jj) * ldm + i * ldi] << (8 * jj);
    }
    return w;
}

// table_coeffs with every lane loading (lanes past NIN*8 read lane 0's bytes and drop them): no
// branch around the loads, so a loop that issues them keeps one memory-counter picture (stream_range)
template <int NIN, int NOUT>
__device__ __forceinline__ uint32_t table_coeffs_all(const uint8_t *M, uint32_t ldm) {
    static_assert(NOUT == 16, "every coefficient word has 4 live outputs");
    const bool live = threadIdx.x < NIN * 8;
    const uint32_t p = live ? threadIdx.x : 0u, q = p & 3u, i = p >> 3;
    uint32_t w = 0;
#pragma unroll
    for (uint32_t jj = 0; jj < 4; jj++) w |= (uint32_t)M[(4 * q + jj) * ldm + i] << (8 * jj);
    return live ? w : 0u;
}

// table_coeffs_all in two steps for a loop that loads the next tile's coefficients at its top and
// builds their tables at the next iteration: the bytes (load) and, after the tile's lookups and stores
// are issued, the word (pack). Packed where they are loaded, the scheduler puts the packing among the
// first lookups, where waiting for the four byte loads — the latest vector memory operations issued —
// is vmcnt(0): a wait for the previous tile's 16 stores as well, every tile (and, for a workgroup's
// only tile, for all ten of its inputs before the first lookup).
struct CoeffBytes {
    uint32_t b[4];
};
template <int NIN, int NOUT>
__device__ __forceinline__ CoeffBytes table_coeff_bytes(const uint8_t *M, uint32_t ldm) {
    static_assert(NOUT == 16, "every coefficient word has 4 live outputs");
    const uint32_t p = threadIdx.x < NIN * 8 ? threadIdx.x : 0u, q = p & 3u, i = p >> 3;
    CoeffBytes c;
#pragma unroll
    for (uint32_t jj = 0; jj < 4; jj++) c.b[jj] = M[(4 * q + jj) * ldm + i];
    return c;
}
template <int NIN>
__device__ __forceinline__ uint32_t table_coeff_pack(CoeffBytes &c) {
    asm volatile("" : "+v"(c.b[0]), "+v"(c.b[1]), "+v"(c.b[2]), "+v"(c.b[3]));
    const uint32_t w = c.b[0] | (c.b[1] << 8) | (c.b[2] << 16) | (c.b[3] << 24);
    return threadIdx.x < NIN * 8 ? w : 0u;
}

// table_coeffs_all for the decode sweep's loop, from the plan's input-major inverse (input i's
// coefficients for outputs 0..9 are the 10 bytes at i * K): lane quad q's word is those of outputs
// 4q..4q+3 — one dword load, not four byte loads (fewer registers pending across the lookups). It
// loads outputs r0..r0+3 with r0 = min(4q, NOUT-4), never past input i's row, and shifts the word
// down by the outputs it read before 4q (outputs past NOUT-1 are zero). One buffer base (wave-
// uniform) and one lane offset, recomputed per call (not hoisted into a register).
template <int NIN, int NOUT>
__device__ __forceinline__ uint32_t table_coeffs_imaj(const uint8_t *M) {
    static_assert(NOUT >= 4 && NOUT <= 16, "quads of outputs");
    uint32_t p = threadIdx.x;
    asm volatile("" : "+v"(p));
    const bool live = p < NIN * 8;
    p = live ? p : 0u;
    const uint32_t q = p & 3u, i = p >> 3;
    const uint32_t r0 = 4 * q < (uint32_t)NOUT - 4 ? 4 * q : (uint32_t)NOUT - 4, sh = 8 * (4 * q - r0);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(M), 0, NIN * NOUT, 0x00020000);
    uint32_t w = __builtin_amdgcn_raw_buffer_load_b32(rs, i * NOUT + r0, 0, 0);
    w = sh < 32 ? w >> sh : 0u;
    return live ? w : 0u;
}

// Build the 2*NIN nibble tables of a NOUT x NIN coefficient matrix from the words of table_coeffs.
// Caller brackets with lds_barrier().
// Multiplication by a constant is linear over GF(2), so row (i, h, nib) = XOR of the products of
// C[.][i] with the set bits of nib << 4h: thread (i, h, output quad q) forms the 4 basis words
// { C[4q+jj][i] * x^(4h+k) : jj < 4 } (xtime chains) and the 16 rows' dwords q by one XOR each
// (nib & (nib-1) is nib minus its lowest bit). The 16 ds_write_b32 per thread go out in a staggered
// row order (DECDS_BUILD_XOR) so that no two tables of a lane group write the same banks (the plain
// order was 8-way conflicted: 5 % of the encode's LDS cycles, r05a PMC). In-process A/B (r05b):
// ±0.3 % — the build is not what bounds the encode; neither is the second barrier per tile (double-
// buffered tables with one barrier per tile measured the same and were removed).
// REMAT: recompute the thread's row addresses at every call. In a loop the compiler otherwise hoists
// the 16 per-lane ds_write addresses of the XOR order out of it, and a 4-wave kernel spills them.
template <int NIN, int NOUT, bool REMAT = false>
__device__ __forceinline__ void build_tables(uint8_t *lds, uint32_t cw, uint32_t poly) {
    uint32_t p = threadIdx.x;
    if constexpr (REMAT) asm volatile("" : "+v"(p));
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
        uint8_t *base = lds + (i * 2 + h) * TABLE_BYTES + 4 * q;
#if DECDS_BUILD_XOR
        // conflict-free order: table s = (2i + h) mod 16 writes row nib ^ s at step nib. The 8 tables of
        // a ds_write_b32 lane group (32 lanes) then hit 8 distinct rows mod 8 = 32 distinct banks instead
        // of one row's 4 banks (8-way). Rows are linear in the nibble: w[nib ^ s] = w[nib] ^ w[s].
        const uint32_t s = (i * 2 + h) & 15u;
        const uint32_t ws = ((s & 1u) ? bw[0] : 0u) ^ ((s & 2u) ? bw[1] : 0u) ^ ((s & 4u) ? bw[2] : 0u) ^
                            ((s & 8u) ? bw[3] : 0u);
#pragma unroll
        for (uint32_t nib = 0; nib < 16; nib++)
            *reinterpret_cast<uint32_t *>(base + ((nib ^ s) * ROW_BYTES)) = w[nib] ^ ws;
#else
#pragma unroll
        for (int nib = 0; nib < 16; nib++) *reinterpret_cast<uint32_t *>(base + nib * ROW_BYTES) = w[nib];
#endif
    }
}

// The lookups' inline-asm ds_read_b128 address the tables absolutely, from LDS byte 0 of the dynamic
// area: a static __shared__ variable in the kernel would be placed first and move every table (round
// 4's first TailLds build read wrong bytes that way). __builtin_amdgcn_groupstaticsize() is the
// kernel's static LDS size, a constant the backend resolves: 0 compiles this to nothing, anything else
// to a trap at the kernel's entry — the contract checked inside the kernel, not only by
// tests/test_isa.py's look at the built code.
__device__ __forceinline__ void tables_at_lds_zero() {
    if (__builtin_amdgcn_groupstaticsize() != 0) __builtin_trap();
}

// byte product M[j][i] * x read back from the built tables (edge columns)
__device__ __forceinline__ uint32_t tbl_mul(const uint8_t *lds, uint32_t i, uint32_t j, uint32_t x) {
    return lds[(i * 2 + 0) * TABLE_BYTES + (x & 15u) * ROW_BYTES + j] ^
           lds[(i * 2 + 1) * TABLE_BYTES + (x >> 4) * ROW_BYTES + j];
}

// ---- streaming row access ---------------------------------------------------------------------
// Rows are addressed as a wave-uniform base plus a 32-bit row offset through a buffer descriptor
// covering 2 GiB from the base (the launchers keep every row offset below). Piece rows start at
// i*L (L = 2^20 + 1) and coded payloads at r*pitch + 10, so most rows are byte-misaligned by the
// rlnc layout itself; gfx9 vector memory accepts unaligned accesses. A lane with nothing to do
// passes column OOB_COL: its buffer loads return zeros and its buffer stores are dropped by the
// range check, so the streaming loop needs no per-lane branch (stream_range).
// DW = dwords per lane per row: 4 (16-column lane blocks) or 2 (8-column blocks: half the
// accumulator and input registers, for more workgroups per CU).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
template <int DW> struct VecT;
template <> struct VecT<4> { using T = u32x4; };
template <> struct VecT<2> { using T = u32x2; };
template <int DW> using Vec = typename VecT<DW>::T;
constexpr uint32_t BUF_RECORDS = 0x80000000u;
constexpr uint32_t OOB_COL = 0x80000000u;

// A row access at byte soff + voff of base: soff is wave-uniform (a row's offset), voff the lane's
// column; both go into the VGPR offset. (The row offset in the instructions' SGPR offset field
// instead, sharing one column VGPR across a tile's rows, measured 1.5 % slower encodes, r05p.)
template <int DW>
__device__ __forceinline__ Vec<DW> ldrow(const uint8_t *base, uint32_t soff, uint32_t voff) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(base), 0, BUF_RECORDS, 0x00020000);
    if constexpr (DW == 4)
        return __builtin_amdgcn_raw_buffer_load_b128(r, soff + voff, 0, 0);
    else
        return __builtin_amdgcn_raw_buffer_load_b64(r, soff + voff, 0, 0);
}

template <int DW, int AUX = 0>
__device__ __forceinline__ void strow(uint8_t *base, uint32_t soff, uint32_t voff, Vec<DW> v) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, BUF_RECORDS, 0x00020000);
    if constexpr (DW == 4)
        __builtin_amdgcn_raw_buffer_store_b128(v, r, soff + voff, 0, AUX);
    else
        __builtin_amdgcn_raw_buffer_store_b64(v, r, soff + voff, 0, AUX);
}

template <int NIN, int DW>
__device__ __forceinline__ void load_block(Vec<DW> (&x)[NIN], const uint8_t *ibase, const uint32_t (&ioff)[NIN],
                                           uint32_t col0) {
#pragma unroll
    for (int i = 0; i < NIN; i++) x[i] = ldrow<DW>(ibase, ioff[i], col0);
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

__device__ __forceinline__ void xor3_into(uint32_t (&acc)[4], const u32x4 &a, const u32x4 &b) {
    // v_bitop3_b32 (gfx950): acc ^ a ^ b in one VALU op (truth table 0x96)
    acc[0] = __builtin_amdgcn_bitop3_b32(acc[0], a.x, b.x, 0x96);
    acc[1] = __builtin_amdgcn_bitop3_b32(acc[1], a.y, b.y, 0x96);
    acc[2] = __builtin_amdgcn_bitop3_b32(acc[2], a.z, b.z, 0x96);
    acc[3] = __builtin_amdgcn_bitop3_b32(acc[3], a.w, b.w, 0x96);
}

// ---- hand-pipelined lookups ---------------------------------------------------------------------
// The lookups of one lane block are cut into DW*NIN groups (input i, dword w: 4 columns x {lo, hi}
// = 8 reads); group g+1 is issued before group g is consumed, so 8-16 reads are in flight per wave
// (hipcc's own schedule waits after every column: ~4 in flight). Reads are inline asm with
// immediate table offsets and explicit counted waits (cdna_hip_programming.md §5.7 form (ii)):
// nothing else in this region issues LGKM operations and one wave's LDS reads return in order.
// The row address of a lookup is nibble * 16 (the table base is the instruction's offset): byte p's
// high nibble masked in place (xw >> 8p) & 0xF0, its low nibble masked and shifted up by 4 — hipcc
// turns both into one SDWA op each (v_and_b32_sdwa / v_lshlrev_b32_sdwa with a byte select).
// HB = bytes of the input dword per group (4: 8 reads per group, 16 in flight; 2: 4 reads per group,
// 8 in flight and half the result registers — for kernels that need the VGPRs for occupancy).
// The row addresses of byte P of an input dword: lo nibble * 16, hi nibble * 16. SDWA: one op per
// address by inline asm, byte P picked by the SDWA source select (hipcc emits a shift + and pair for
// most of them): 8 % fewer VALU instructions, −1.4…−1.9 % fused ChunkSet::new time (issue-bound),
// +0.3…+0.9 % encode / decode time (not issue-bound; r05za) — so the fused kernel only.
template <int P, bool SDWA>
__device__ __forceinline__ void nibble_addr(uint32_t xw, uint32_t lo4, uint32_t &alo, uint32_t &ahi) {
    if constexpr (SDWA) {
        // one op per address, byte P picked by the SDWA source select: (lo4.byte P) << 4 and
        // (xw.byte P) & 0xF0 (byte 0's high nibble a plain full-rate v_and)
        asm("v_lshlrev_b32_sdwa %0, 4, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_%c2"
            : "=v"(alo)
            : "v"(lo4), "i"(P));
        if constexpr (P == 0)
            ahi = xw & 0xF0u;
        else
            asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_%c3 src1_sel:DWORD"
                : "=v"(ahi)
                : "v"(xw), "v"(0xF0u), "i"(P));
    } else {
        alo = ((lo4 >> (8 * P)) & 0xFFu) << 4;
        ahi = (xw >> (8 * P)) & 0xF0u;
    }
}

template <int G, int DW, uint32_t TB, int HB, bool SDWA, int Q>
__device__ __forceinline__ void lds_issue_q(u32x4 (&r)[2 * HB], uint32_t xw, uint32_t lo4) {
    constexpr int PARTS = 4 / HB, g2 = G / PARTS, part = G % PARTS;
    constexpr int i = g2 / DW;
    constexpr uint32_t tlo = TB + (2 * i) * TABLE_BYTES, thi = TB + (2 * i + 1) * TABLE_BYTES;
    uint32_t alo, ahi;
    nibble_addr<part * HB + Q, SDWA>(xw, lo4, alo, ahi);
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r[2 * Q]) : "v"(alo), "i"(tlo));
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r[2 * Q + 1]) : "v"(ahi), "i"(thi));
}

template <int G, int DW, uint32_t TB, int HB, bool SDWA, int... Qs>
__device__ __forceinline__ void lds_issue_qs(std::integer_sequence<int, Qs...>, u32x4 (&r)[2 * HB], uint32_t xw) {
    const uint32_t lo4 = xw & 0x0F0F0F0Fu;
    (lds_issue_q<G, DW, TB, HB, SDWA, Qs>(r, xw, lo4), ...);
}

template <int G, int DW, uint32_t TB, int HB = 4, bool SDWA = false>
__device__ __forceinline__ void lds_issue(u32x4 (&r)[2 * HB], uint32_t xw) {
    lds_issue_qs<G, DW, TB, HB, SDWA>(std::make_integer_sequence<int, HB>{}, r, xw);
}

template <int CNT>
__device__ __forceinline__ void lds_wait(u32x4 (&r)[8]) {
    asm volatile("s_waitcnt lgkmcnt(%8)"
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                 : "i"(CNT)
                 : "memory");
}
template <int CNT>
__device__ __forceinline__ void lds_wait(u32x4 (&r)[2]) {
    asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(r[0]), "+v"(r[1]) : "i"(CNT) : "memory");
}
template <int CNT>
__device__ __forceinline__ void lds_wait(u32x4 (&r)[4]) {
    asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]) : "i"(CNT) : "memory");
}

// Group G of the lookups; input i's register takes the next block's bytes (ncol0) as soon as that
// input's lookups are all issued — before this block's stores: gfx9's vmcnt counts stores too, so
// a load issued behind the stores would also wait for them.
template <int NIN, int DW, uint32_t TB, int G, int HB = 4, bool SDWA = false>
__device__ __forceinline__ void lds_step(uint32_t (&acc)[4 * DW][4], u32x4 (&ra)[2 * HB], u32x4 (&rb)[2 * HB],
                                         Vec<DW> (&x)[NIN], const uint8_t *ibase, const uint32_t (&ioff)[NIN],
                                         uint32_t ncol0) {
    constexpr int PARTS = 4 / HB, NGI = DW * PARTS, NG = NGI * NIN;  // groups per input, in all
    u32x4(&cur)[2 * HB] = (G & 1) ? rb : ra;  // group G's results
    u32x4(&nxt)[2 * HB] = (G & 1) ? ra : rb;
    if constexpr (G + 1 < NG) {
        constexpr int H = G + 1, hi = H / NGI, hw = (H / PARTS) % DW;
        lds_issue<H, DW, TB, HB, SDWA>(nxt, x[hi][hw]);
        if constexpr ((H % NGI) == NGI - 1) x[hi] = ldrow<DW>(ibase, ioff[hi], ncol0);
        lds_wait<2 * HB>(cur);
    } else {
        lds_wait<0>(cur);
    }
    constexpr int w = (G / PARTS) % DW, part = G % PARTS;
#pragma unroll
    for (int q = 0; q < HB; q++) xor3_into(acc[4 * w + part * HB + q], cur[2 * q], cur[2 * q + 1]);
}

template <int NIN, int DW, uint32_t TB, int HB, bool SDWA, int... Gs>
__device__ __forceinline__ void lookups(std::integer_sequence<int, Gs...>, uint32_t (&acc)[4 * DW][4],
                                        Vec<DW> (&x)[NIN], const uint8_t *ibase, const uint32_t (&ioff)[NIN],
                                        uint32_t ncol0) {
    u32x4 ra[2 * HB], rb[2 * HB];
    lds_issue<0, DW, TB, HB, SDWA>(ra, x[0][0]);
    (lds_step<NIN, DW, TB, Gs, HB, SDWA>(acc, ra, rb, x, ibase, ioff, ncol0), ...);
}

// One lane block of 4*DW columns: out_j[col0 ..) = sum_i M[j][i] * in_i[col0 ..), tables at LDS
// byte TB. x holds this block's inputs on entry and on exit the inputs at column ncol0 of the rows
// at ibase + ioff (the next block's: the same chunkset's rows, or the next tile's chunkset's).
// sink(j, v): also hand output j's bytes elsewhere (the fused commitment's LDS message slots)
struct NoSink {
    template <typename V>
    __device__ void operator()(int, const V &) const {}
};
template <int NIN, int NOUT, int DW, uint32_t TB = 0, typename Sink = NoSink, int SAUX = 0, bool GSTORE = true,
          int HB = 4, bool SDWA = false>
__device__ __forceinline__ void combine_block(Vec<DW> (&x)[NIN], uint8_t *obase, const uint32_t (&ooff)[NOUT],
                                              uint32_t col0, const uint8_t *ibase, const uint32_t (&ioff)[NIN],
                                              uint32_t ncol0, Sink sink = Sink{}) {
    uint32_t acc[4 * DW][4];  // acc[column][output group]: byte b = output 4*group + b
#pragma unroll
    for (int c = 0; c < 4 * DW; c++)
#pragma unroll
        for (int q = 0; q < 4; q++) acc[c][q] = 0;
#ifdef DECDS_STUDY_PATTERN
    // pattern-ceiling builds only (bench.py's roofline.*.pattern_GBps, tools/bin/libdecds_pattern.so):
    // the kernel's own loads, stores, tile order and table builds with the LDS lookups replaced by one
    // XOR per input dword — input i's next-block load issued as soon as input i is consumed, as in
    // lds_step. Wrong bytes by design; never in the product library.
#pragma unroll
    for (int i = 0; i < NIN; i++) {
#pragma unroll
        for (int w = 0; w < DW; w++) acc[4 * w + (i & 3)][(i >> 2) & 3] ^= x[i][w];
        x[i] = ldrow<DW>(ibase, ioff[i], ncol0);
    }
#else
    lookups<NIN, DW, TB, HB, SDWA>(std::make_integer_sequence<int, DW * NIN * (4 / HB)>{}, acc, x, ibase, ioff, ncol0);
#endif
    // columns x outputs -> outputs x columns
#pragma unroll
    for (int q = 0; q < 4; q++) {
        if (4 * q >= NOUT) break;
        uint32_t o[4][DW];  // o[b][w]: output 4q+b, columns 4w..4w+3
#pragma unroll
        for (int w = 0; w < DW; w++)
            transpose4x4(acc[4 * w + 0][q], acc[4 * w + 1][q], acc[4 * w + 2][q], acc[4 * w + 3][q], o[0][w], o[1][w],
                         o[2][w], o[3][w]);
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int j = 4 * q + b;
            Vec<DW> v;
#pragma unroll
            for (int w = 0; w < DW; w++) v[w] = o[b][w];
            if (j < NOUT) {
                if constexpr (GSTORE) strow<DW, SAUX>(obase, ooff[j], col0, v);
                sink(j, v);
            }
        }
    }
}

// ---- geometry per lane-block width, column phase and edge columns -------------------------------
// Lane blocks of COLS = 4*DW columns; a tile is 256 blocks. Blocks cover payload columns from
// `phase` on (phase < COLS, chosen by the launcher so that coded rows at a COLS-aligned pitch are
// written on COLS-byte boundaries); the workgroup owning tile 0 does the edge columns byte by byte:
// e < phase is column e, the rest the columns after the last block. Piece 9's main columns must stay
// below CS - 9L (its marker and padding are edge columns), so a phase above 7 gives up one block.
//
// Message tiling (phase MSG_PHASE = 6, i.e. 16-byte-aligned rows): the chunk digest's message is
// le64 ids (16 B) || row, so payload column p is message byte p + 26 and a block starting at column
// 16m - 26 is message block m. Tiles then start MSG_SHIFT = 2 blocks early (tile t = message blocks
// [256t, 256t + 256), its first two lanes idle in tile 0) and the last block joins the edge columns
// (6 head + 27 tail): a tile is exactly 4 BLAKE3 chunks of every row, and the fused commitment
// (rlnc_encode_hash_kernel) walks the same geometry in 128-byte steps. On rows at 16 mod 128 every
// wave's store run is then 128-byte aligned.
constexpr uint32_t MAX_FULL_PHASE = (uint32_t)(CS - (K - 1) * L) - MAIN_COLS;
// piece i's byte offset in a chunkset (the study build rounds it down to 256 bytes: timing only)
__device__ __forceinline__ uint32_t piece_off(int i) {
#if DECDS_STUDY_ALIGNED_PIECES == 1
    return (uint32_t)(i * L) & ~255u;
#elif DECDS_STUDY_ALIGNED_PIECES == 2  // 16-byte aligned, lines not (never past i * L: stays in bounds)
    return (uint32_t)(i * (L - 1) - 16 * i);
#elif DECDS_STUDY_ALIGNED_PIECES == 3  // dword aligned
    return (uint32_t)(i * (L - 1) - 4 * i);
#else
    return (uint32_t)(i * L);
#endif
}
static_assert(MAX_FULL_PHASE == 7, "layout");
template <int DW> constexpr uint32_t COLS = 4 * DW;
template <int DW> constexpr uint32_t BLOCKS = MAIN_COLS / COLS<DW>;                 // 65535 / 131070
template <int DW> constexpr uint32_t TILES = (BLOCKS<DW> + TILE_BLOCKS - 1) / TILE_BLOCKS;  // 256 / 512
static_assert(BLOCKS<4> * COLS<4> == MAIN_COLS && BLOCKS<2> * COLS<2> == MAIN_COLS, "tiling covers the main columns");
constexpr uint32_t MSG_PHASE = (16 - (16 + K) % 16) % 16;
template <int DW> constexpr uint32_t MSG_SHIFT = (16 + K + MSG_PHASE) / COLS<DW>;   // 2 / 4 blocks
template <int DW> constexpr uint32_t MSG_MAIN = (MAIN_COLS - 16) / COLS<DW>;        // 65534 / 131068
static_assert(MSG_PHASE == 6 && MSG_PHASE < COLS<2> && MSG_SHIFT<4> * COLS<4> == 32 && MSG_SHIFT<2> * COLS<2> == 32,
              "message block m = payload block m - MSG_SHIFT");
static_assert((MSG_SHIFT<4> + MSG_MAIN<4>) == TILES<4> * TILE_BLOCKS && (MSG_SHIFT<2> + MSG_MAIN<2>) == TILES<2> * TILE_BLOCKS,
              "message tiles end where the 1024 full BLAKE3 chunks end");
// MSG (compile time): message tiling, phase fixed at MSG_PHASE; else `phase` as passed
template <int DW, bool MSG>
__device__ __forceinline__ uint32_t main_blocks(uint32_t phase) {
    if constexpr (MSG) return MSG_MAIN<DW>;
    return BLOCKS<DW> - (phase > MAX_FULL_PHASE);
}
template <int DW, bool MSG>
__device__ __forceinline__ uint32_t edge_cols(uint32_t phase) { return (uint32_t)L - main_blocks<DW, MSG>(phase) * COLS<DW>; }
template <int DW, bool MSG>
__device__ __forceinline__ uint32_t edge_col(uint32_t e, uint32_t phase) {
    const uint32_t ph = MSG ? MSG_PHASE : phase;
    return e < ph ? e : main_blocks<DW, MSG>(phase) * COLS<DW> + e;
}

// this lane's first column of tile t of a range ending at tb, or out of range (with message tiling
// the lanes of the two blocks before column MSG_PHASE wrap to a huge block index: out of range too)
template <int DW, bool MSG>
__device__ __forceinline__ uint32_t tile_col(uint32_t t, uint32_t tb, uint32_t phase) {
    const uint32_t block = t * TILE_BLOCKS + threadIdx.x - (MSG ? MSG_SHIFT<DW> : 0u);
    return t < tb && block < main_blocks<DW, MSG>(phase) ? block * COLS<DW> + (MSG ? MSG_PHASE : phase) : OOB_COL;
}

// Tiles [ta, tb) of one chunkset, branch-free: lanes past the last block use OOB_COL, so no lane
// branches. The loop is entered after the first tile's loads AND NOUT dropped stores, the same
// memory-counter picture as every later tile (NIN prefetched loads, then NOUT stores). With a
// branch around the streaming code, or a reload path inside the loop, hipcc's wait-count pass
// merges paths that issued no stores and waits with vmcnt(NIN-1) for the next tile's first input:
// every tile then waited for the previous tile's stores as well; here it waits for the inputs only.
// HAVE: x already holds tile ta's inputs (loaded before the workgroup's table build).
template <int NIN, int NOUT, int DW, bool HAVE, bool MSG = false, int HB = 4, int SAUX = 0>
__device__ __forceinline__ void stream_range(uint32_t ta, uint32_t tb, uint32_t phase, const uint8_t *ibase,
                                             const uint32_t (&ioff)[NIN], uint8_t *obase,
                                             const uint32_t (&ooff)[NOUT], Vec<DW> (&x)[NIN]) {
    auto col = [&](uint32_t t) { return tile_col<DW, MSG>(t, tb, phase); };
    if constexpr (!HAVE) load_block<NIN, DW>(x, ibase, ioff, col(ta));
    asm volatile("" ::: "memory");  // keep the dropped stores after the loads, as in the loop
#pragma unroll
    for (int j = 0; j < NOUT; j++) strow<DW>(obase, ooff[j], OOB_COL, Vec<DW>{});
    // ta < tb (callers): a do-while, so no zero-trip guard lets hipcc sink the prologue loads
    // below the dropped stores (it did: vmcnt(9) again, profiles/HISTORY.md §8)
    uint32_t t = ta;
#pragma unroll 1
    do {
        combine_block<NIN, NOUT, DW, 0, NoSink, SAUX, true, HB>(x, obase, ooff, col(t), ibase, ioff, col(t + 1));
    } while (++t < tb);
}

// ---- fused commitment, wave-step form (ChunkSet::new, chunkset.rs:43-63) ------------------------
// The unit-hash form above re-reads each unit's 256 KiB of coded rows after its stores (no longer in
// L2 by then: 1.7 GB of extra traffic at cfg2). Here no coded byte is read back. A wave owns BLAKE3
// chunks [4U, 4U + 4) of all 16 rows of one chunkset — 64 chunks, one per lane (lane h: row h >> 2,
// chunk 4U + (h & 3)) — and walks them in steps of STEP = 16 lane blocks of message bytes (128 with
// 8-column blocks, 256 with 16-column blocks): the step's 4 x STEP coded columns (4 runs of 16 lane
// blocks) are encoded, stored to HBM in whole 128-byte lines (rows 16 bytes past a 128-byte boundary:
// message byte m of a row sits at m mod 128 of a line) and written into the wave's LDS slots, from
// which each lane reads its chunk's STEP / 64 blocks and compresses them. The next step's inputs are
// in flight across the compressions (the rolling prefetch of combine_block).
// Lanes then fold their row's 4 chunk values into the aligned 4-chunk subtree (sub: n x 16 x 256 chaining
// values). LDS: chunk slot h = STEP bytes at h * STEP, its 16-byte pieces XOR-swizzled by key(h) so that the
// 16 lanes of every ds_read_b128 group read 16 distinct bank quads and every store group fills whole
// bank rows without conflicts.
constexpr uint32_t FH_WAVE_CHUNKS = 4;                                 // chunks per row per wave
constexpr uint32_t FH_WAVE_UNITS = 1024 / FH_WAVE_CHUNKS;              // 256 wave units per chunkset
constexpr uint32_t FH_WAVES = WG / 64;                                 // 4
constexpr uint32_t FH_WG_UNITS = FH_WAVE_UNITS / FH_WAVES;             // 64 workgroups per chunkset
constexpr uint32_t MSG_HEAD = 16 + K + MSG_PHASE;                      // message byte of the first lane block
static_assert(MSG_HEAD == 32, "message tiling");
// coded-row stores non-temporal: the rows are never read back here, and out of L2 they leave it to the
// input lines whose second half the next step reads (PMC reads 1.69 -> 1.44 GB per cfg2 launch, -0.6 %)
constexpr int FH_STORE_AUX = 2;
// lookup groups of 2 bytes in the fused kernel too: -1.3 % at 103 / 256 chunksets (r05e); at 4
// waves/SIMD (117 VGPRs) -0.9 / -1.4 %: the compressions, not occupancy, set its time
#ifndef DECDS_FH_HB
#define DECDS_FH_HB 2
#endif
constexpr int FH_HB = DECDS_FH_HB;
template <int DW> constexpr uint32_t FH_STEP = 16 * COLS<DW>;           // 128 / 256 message bytes per chunk
// (byte tables — one lookup per input byte, 40 KiB of tables, 2 workgroups per CU — measured +2.6 /
// +2.1 / -2.1 % at 103 / 256 / 1024 chunksets, r05o; in git history at f15b23c)
constexpr uint32_t FH_TBL = LDS_BYTES;
template <int DW> constexpr uint32_t FH_LDS = FH_TBL + FH_WAVES * 64 * FH_STEP<DW>;  // 37 / 69 KiB
template <int DW>
__device__ __forceinline__ uint32_t fh_key(uint32_t slot) {
    constexpr uint32_t R = 256 / FH_STEP<DW>, P = FH_STEP<DW> / 16;  // slots per bank row, pieces per slot
    return (slot / R) & (P - 1);
}

// lanes 4g .. 4g+3 hold 4 consecutive chaining values of one aligned group -> all 4 hold its parent
// (level k pairs lanes q, q ^ 2^k)
__device__ __forceinline__ void fold4(uint32_t (&cv)[8], uint32_t h) {
#pragma unroll
    for (uint32_t k = 0; k < 2; k++) {
        uint32_t sib[8], lo[8], hi[8];
        const bool right = (h >> k) & 1u;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            sib[i] = __shfl_xor(cv[i], 1 << k, 4);
            lo[i] = right ? sib[i] : cv[i];
            hi[i] = right ? cv[i] : sib[i];
        }
        b3::parent(lo, hi, 0, cv);
    }
}

template <int DW, int WAVES>
__global__ __launch_bounds__(WG, WAVES) __attribute__((amdgpu_waves_per_eu(WAVES, WAVES)))
void rlnc_encode_hash_kernel(const uint8_t *__restrict__ src, size_t n, const uint8_t *__restrict__ coeffs,
                             uint8_t *__restrict__ dst, size_t pitch, uint32_t poly, uint32_t marker,
                             uint64_t first_id, const uint64_t *__restrict__ ids, uint32_t *__restrict__ sub) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    tables_at_lds_zero();
    constexpr uint32_t STEP = FH_STEP<DW>, STEPS = b3::CHUNK / STEP, BPS = STEP / b3::BLOCK;  // blocks per step
    const uint32_t cs = blockIdx.x / FH_WG_UNITS, gu = blockIdx.x % FH_WG_UNITS;
    if (cs >= n) return;
    const uint32_t h = threadIdx.x & 63u;
    const uint32_t U = __builtin_amdgcn_readfirstlane(gu * FH_WAVES + (threadIdx.x >> 6));
    const uint8_t *M = coeffs + (size_t)cs * N * K;
    const uint8_t *ibase = src + (size_t)cs * CS;
    uint8_t *obase = dst + (size_t)cs * N * pitch;
    uint32_t ioff[K], ooff[N];
#pragma unroll
    for (int i = 0; i < (int)K; i++) ioff[i] = (uint32_t)(i * L);
#pragma unroll
    for (int j = 0; j < (int)N; j++) ooff[j] = (uint32_t)(j * pitch + K);
    // encode lane: run eq = h >> 4 (chunk 4U + eq), lane block eb = h & 15 of the step's STEP bytes;
    // message byte m is payload column m - 26 (ids 16 B, coding vector 10 B); m < 32 are not lane columns
    const uint32_t eq = h >> 4, eb = h & 15u;
    const uint32_t m0 = (FH_WAVE_CHUNKS * U + eq) * b3::CHUNK + COLS<DW> * eb;
    auto col = [&](uint32_t st) {
        const uint32_t m = m0 + st * STEP;
        return st < STEPS && m >= MSG_HEAD ? m - (16 + K) : OOB_COL;
    };
    const uint32_t cw = table_coeffs<K, N>(M, K);
    Vec<DW> x[K];
    load_block<K, DW>(x, ibase, ioff, col(0));
    build_tables<K, N>(lds, cw, poly);
    lds_barrier();
    if (gu == 0) {  // the chunkset's first workgroup: coding-vector prefixes and the edge columns
        for (uint32_t idx = threadIdx.x; idx < N * K; idx += WG) obase[(idx / K) * pitch + idx % K] = M[idx];
        for (uint32_t idx = threadIdx.x; idx < edge_cols<DW, true>(MSG_PHASE) * N; idx += WG) {
            const uint32_t j = idx % N, c = edge_col<DW, true>(idx / N, MSG_PHASE);
            uint32_t y = 0;
#pragma unroll
            for (uint32_t i = 0; i < K; i++) {
                const uint64_t p = (uint64_t)i * L + c;
                const uint32_t xv = p < CS ? ibase[p] : (p == CS ? marker : 0u);
                y ^= tbl_mul(lds, i, j, xv);
            }
            obase[j * pitch + K + c] = (uint8_t)y;
        }
        __syncthreads();  // the edge bytes are in L2 before wave 0 reads row bytes 0..15 back
    }
    const uint32_t j = h >> 2, c = FH_WAVE_CHUNKS * U + (h & 3u);  // this lane's chunk: row j, chunk c
    // chunk 0's first block = ids || row bytes 0..15 (coding vector, 6 head edge columns)
    u32x4 head = {0, 0, 0, 0};
    if (U == 0)
        head = __builtin_amdgcn_raw_buffer_load_b128(
            __builtin_amdgcn_make_buffer_rsrc(obase, 0, BUF_RECORDS, 0x00020000), j * (uint32_t)pitch, 0, 1);
    asm volatile("" ::: "memory");  // the loop's memory-counter picture: inputs, then 16 dropped stores
#pragma unroll
    for (int jj = 0; jj < (int)N; jj++) strow<DW>(obase, ooff[jj], OOB_COL, Vec<DW>{});
    uint8_t *wl = lds + FH_TBL + (threadIdx.x >> 6) * 64 * STEP;
    // encode lane's LDS address for rows jj = jm (mod 4) (the swizzle key of slot 4jj + eq depends on
    // jj mod 4 only); row jj adds 4 jj slots
    uint32_t wx[4];
#pragma unroll
    for (uint32_t jm = 0; jm < 4; jm++) {
        const uint32_t piece = DW == 4 ? eb : eb >> 1, half = DW == 4 ? 0u : (eb & 1u);
        wx[jm] = STEP * eq + 16 * (piece ^ fh_key<DW>(4 * jm + eq)) + 8 * half;
    }
    const uint32_t rbase = h * STEP + 16 * fh_key<DW>(h);
    auto sink = [&](int jj, const Vec<DW> &v) { *reinterpret_cast<Vec<DW> *>(wl + wx[jj & 3] + 4 * STEP * jj) = v; };
    uint32_t cv[8];
#pragma unroll
    for (int i = 0; i < 8; i++) cv[i] = b3::K3.iv[i];
    // chunkset.rs:47; ids (coalesced ChunkSet::new callers): one chunkset id per batch entry
    const uint64_t cs_id = ids ? uniform_u64(ids[cs]) : first_id + cs, chunk_id = cs_id * N + j;
    uint32_t st = 0;
#pragma unroll 1
    do {
        combine_block<K, N, DW, 0, decltype(sink), FH_STORE_AUX, true, FH_HB, true>(x, obase, ooff, col(st), ibase, ioff,
                                                                             col(st + 1), sink);
        // one wave: its LDS accesses complete in order, no barrier between the slot writes and reads
#pragma unroll
        for (uint32_t kb = 0; kb < BPS; kb++) {
            uint32_t mw[16];
#pragma unroll
            for (uint32_t w = 0; w < 4; w++) {
                const u32x4 v = *reinterpret_cast<const u32x4 *>(wl + (rbase ^ (16 * (4 * kb + w))));
                mw[4 * w] = v.x, mw[4 * w + 1] = v.y, mw[4 * w + 2] = v.z, mw[4 * w + 3] = v.w;
            }
            if (kb == 0 && U == 0 && st == 0) {
                const bool c0 = c == 0;
                mw[0] = c0 ? (uint32_t)cs_id : mw[0];
                mw[1] = c0 ? (uint32_t)(cs_id >> 32) : mw[1];
                mw[2] = c0 ? (uint32_t)chunk_id : mw[2];
                mw[3] = c0 ? (uint32_t)(chunk_id >> 32) : mw[3];
                mw[4] = c0 ? head.x : mw[4];
                mw[5] = c0 ? head.y : mw[5];
                mw[6] = c0 ? head.z : mw[6];
                mw[7] = c0 ? head.w : mw[7];
            }
            const uint32_t k = st * BPS + kb;  // block of the chunk
            b3::compress(cv, mw, c, b3::BLOCK, (k == 0 ? b3::CHUNK_START : 0u) | (k == 15 ? b3::CHUNK_END : 0u), cv);
        }
    } while (++st < STEPS);
    // row j's 4 chunk values (lanes 4j .. 4j+3) -> their aligned 4-chunk subtree. (Folding on across the
    // workgroup's 4 waves, one barrier at the end, measured 1-2 % slower in total than the fold kernel's
    // 2 extra levels: r03h/i.)
    fold4(cv, h);
    if ((h & 3u) == 0) {
        uint32_t *o = sub + (((size_t)cs * N + j) * FH_WAVE_UNITS + U) * 8;
#pragma unroll
        for (int i = 0; i < 8; i++) o[i] = cv[i];
    }
}

// Encode as a persistent sweep: G = gridDim.x resident workgroups; workgroup b encodes tiles b, b + G,
// b + 2G, ... of the whole batch (chunkset-major), so at any moment the tiles in flight are about G
// consecutive ones — the order of one-tile workgroups in dispatch order, the fastest access pattern
// of the encode at the kernels' occupancy (tools/layoutbench, r02n: 5.7-5.9 TB/s against 5.4-5.5 for
// units of 4 tiles per XCD eighth) — without a workgroup start per tile: the next tile's coefficient
// bytes and inputs are loaded while this tile computes (rolling prefetch across the chunkset change)
// and its tables are built into the other of two LDS table buffers, one LDS barrier per tile. The edge
// columns of chunksets b, b + G, ... are done first, outside the tile loop, so the loop issues the same
// memory operations on every path (stream_range's vmcnt picture: inputs waited for, never stores).
// QUEUE: after the first G tiles (tile = blockIdx.x) every next tile comes from a tile counter
// (one atomic add per workgroup and tile, issued a tile ahead), so the tiles in flight stay one
// resident grid wide however the workgroups' speeds differ — a fixed stride lets them drift apart.
// counter == NULL (batches of at most G tiles): one tile per workgroup, no counter. counter[0] is the
// tile counter, counter[1] the exit count; both start at 0 (zeroed with the context) and the last
// workgroup to finish zeroes them again.
// EDGE_SPLIT (the small-batch form): the last min(n, EDGE_WGS) workgroups of the grid do the
// prefixes and edge columns, one chunkset each in turn, beside the tile workgroups instead of ahead of
// their first tile (at n = 1 the edge pass — byte-wise loads, a few dependent HBM round trips — sat on
// the one critical path of a 13 µs launch). The launcher keeps the whole grid co-resident.
constexpr uint32_t EDGE_WGS = 64;
// The sweeps end only because every workgroup's next tile lies strictly past its current one: the
// counter only grows, and a workgroup's next grab is issued after its previous one returned. A counter
// value read before its atomic has landed breaks that — in the 3-wave encode build of round 4 (r06z14)
// hipcc spilled the pending return register straight after the atomic, so the spill slot held the
// atomic's data operand (1) and every workgroup took tile G + 1 again and again: a silent hang, not a
// fault (profiles/HISTORY.md §8). Here a violated order ends the kernel with a trap (a named kernel fault on the
// host side) instead of spinning. next and cur are wave-uniform (SGPRs): one compare per tile.
// Both sweeps take their second tile statically (tile b + G of workgroup b) and only the third one on
// from the counter (2G + the counter's value), so a workgroup's first grab goes out at its first loop
// head and has a whole tile to return. Taken at kernel start and waited for before the first tile, the
// G first grabs — all at once, on one counter line — held every workgroup's first tables back by 6-10
// µs at 16-64 chunksets (phase trace r07d: first tables 6.6 µs after entry at the earliest, against
// 2-4 µs for a launch without a counter). 0: round 4's order (study builds, A/B).
#ifndef DECDS_STATIC_SECOND
#define DECDS_STATIC_SECOND 1
#endif
#ifndef DECDS_SWEEP_GUARD
#define DECDS_SWEEP_GUARD 1  // 0: study builds only (the guard's cost A/B)
#endif
__device__ __forceinline__ void sweep_guard(uint32_t next, uint32_t cur) {
    if (DECDS_SWEEP_GUARD && next <= cur) __builtin_trap();
}
// coded-row store cache policy (SAUX, the buffer stores' aux bits): `sc1` (16, write-through) below
// DECDS_ENC_NT_MIN_N chunksets, `nt` (2) from there on. A plain store leaves its line dirty in the
// XCD's L2, so a small batch's coded rows were written back by the end-of-kernel release, after its
// last wave: write-through moves that into the launch (-12...-16 % at 1-2 chunksets, -3 % at 16,
// r06p / r06q). From 256 chunksets on `sc1` costs +0.5 % and `nt` gains 0.5-1.5 % (profiles/HISTORY.md §8).
constexpr int STORE_SC1 = 16, STORE_NT = 2;
// Study builds only (DECDS_PHASE_TRACE, tools/phasetrace.py): wave 0 of each workgroup stamps the
// 100 MHz real-time counter at its phases — entry, edge pass done, first tables ready, last lookups
// issued, stores drained — plus its tile count (vector stores; decds_debug_phase_trace copies them out).
#ifdef DECDS_PHASE_TRACE
constexpr uint32_t PT_WGS = 8192, PT_SLOTS = 32;  // slots 8 + k: tile k's tables ready (k < 16)
__device__ uint64_t g_phase_trace[PT_WGS * PT_SLOTS];
#define PT_SET(slot, v)                                                                   \
    do {                                                                                  \
        if (threadIdx.x == 0 && blockIdx.x < PT_WGS) g_phase_trace[blockIdx.x * PT_SLOTS + (slot)] = (v); \
    } while (0)
#define PT_STAMP(slot) PT_SET(slot, __builtin_amdgcn_s_memrealtime())
#else
#define PT_SET(slot, v) \
    do {                \
    } while (0)
#define PT_STAMP(slot) PT_SET(slot, 0)
#endif
template <int DW, int WAVES, bool MSG, bool QUEUE = false, bool EDGE_SPLIT = false, int SAUX = 0>
__global__ __launch_bounds__(WG, WAVES) __attribute__((amdgpu_waves_per_eu(WAVES, WAVES)))
void rlnc_encode_sweep_kernel(const uint8_t *__restrict__ src, size_t n, const uint8_t *__restrict__ coeffs,
                              uint8_t *__restrict__ dst, size_t pitch, uint32_t phase, uint32_t poly, uint32_t marker,
                              uint32_t *__restrict__ counter) {
    // no static __shared__ here: the lookups' inline-asm ds_reads address the tables from LDS byte 0,
    // so everything lives in the dynamic allocation (2 table buffers, then the next-tile slot)
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    tables_at_lds_zero();
    PT_STAMP(0);
#ifdef DECDS_PHASE_TRACE
    {  // where the workgroup runs: HW_ID (CU / SH / SE in bits 8-15) and the XCD
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        PT_SET(6, hw);
        PT_SET(7, xcc);
    }
#endif
    constexpr uint32_t T = TILES<DW>;
    uint32_t ioff[K], ooff[N];
#pragma unroll
    for (int i = 0; i < (int)K; i++) ioff[i] = piece_off(i);
#pragma unroll
    for (int j = 0; j < (int)N; j++) ooff[j] = (uint32_t)(j * pitch + K);
    // 1. coding-vector prefixes and edge columns of chunksets b, b + G, ... (tables in buffer 1); with
    // EDGE_SPLIT, when the launcher gave one workgroup per tile plus NE more, by those NE edge
    // workgroups at the end of the grid, which then leave
    const uint64_t total = (uint64_t)n * T;
    const uint32_t NE = EDGE_SPLIT && gridDim.x > total ? (uint32_t)(gridDim.x - total) : 0u;
    const uint32_t G = gridDim.x - NE;  // tile workgroups
    const bool edge_wg = NE && blockIdx.x >= G;
#ifdef DECDS_STUDY_NO_EDGE  // timing studies only: no edge pass at all (wrong bytes in the edge columns)
    for (size_t cs = n; cs < n; cs++) {
#else
    for (size_t cs = NE ? (edge_wg ? blockIdx.x - G : n) : blockIdx.x; cs < n; cs += NE ? NE : G) {
#endif
        const uint8_t *M = coeffs + cs * N * K;
        const uint8_t *ibase = src + cs * CS;
        uint8_t *obase = dst + cs * N * pitch;
        const uint32_t cw = table_coeffs<K, N>(M, K);
        lds_barrier();
        build_tables<K, N>(lds + LDS_BYTES, cw, poly);
        lds_barrier();
        for (uint32_t idx = threadIdx.x; idx < N * K; idx += WG) obase[(idx / K) * pitch + idx % K] = M[idx];
        for (uint32_t idx = threadIdx.x; idx < edge_cols<DW, MSG>(phase) * N; idx += WG) {
            const uint32_t j = idx % N, col = edge_col<DW, MSG>(idx / N, phase);
            uint32_t y = 0;
#pragma unroll
            for (uint32_t i = 0; i < K; i++) {
                const uint64_t p = (uint64_t)i * L + col;
                const uint32_t xv = p < CS ? ibase[p] : (p == CS ? marker : 0u);
                y ^= tbl_mul(lds + LDS_BYTES, i, j, xv);
            }
            obase[j * pitch + K + col] = (uint8_t)y;
        }
    }
    // 2. the sweep over tiles blockIdx.x, + G, ... (sweeps per XCD eighth measured slower, r02p)
    PT_STAMP(1);
    uint32_t t = blockIdx.x;
#ifdef DECDS_PHASE_TRACE
    if (edge_wg || t >= total) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        PT_STAMP(4);
        return;
    }
    uint32_t pt_tiles = 0;
#else
    if (edge_wg || t >= total) return;
#endif
    auto col_of = [&](uint32_t tt) { return tile_col<DW, MSG>(tt % T, T, phase); };
    uint32_t cs = t / T;
    // prologue = the loop's memory-counter picture at its head: this tile's coefficient bytes, its
    // inputs, then 16 dropped stores
    // The tile counter is bumped by inline asm: a compiler-visible atomic's result becomes a phi at the
    // end of the lane-0 branch, where hipcc waits for it with vmcnt(0) — i.e. for every store in
    // flight. Here it is waited for explicitly, a step later, with vmcnt(16): this step's 16 stores
    // may stay in flight. (The compiler's own counts then miss one operation, which only ever makes
    // its waits stricter.)
    auto grab_next = [&]() -> uint32_t {
        uint32_t r = 0;
        if (QUEUE && counter && threadIdx.x == 0)
            asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(r) : "v"(counter), "v"(1u) : "memory");
        return r;
    };
    // The first loop head waits for the coefficient bytes with vmcnt(26) — the ten input loads and 16
    // dropped stores still in flight — so the first tile's lookups take each input as it lands. (With
    // DECDS_STATIC_SECOND 0 the first grab goes out here, ahead of those loads, and that wait covers it.)
    uint32_t grab = DECDS_STATIC_SECOND ? 0u : grab_next();  // (static second tile: first grab at the loop head)
    asm volatile("" ::: "memory");
    uint32_t cw = table_coeffs_all<K, N>(coeffs + (size_t)cs * N * K, K);
    Vec<DW> x[K];
    load_block<K, DW>(x, src + (size_t)cs * CS, ioff, col_of(t));
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < (int)N; j++) strow<DW>(dst, ooff[j], OOB_COL, Vec<DW>{});
    // One tile per iteration: build its tables from the coefficient bytes the previous iteration
    // loaded (issued before that iteration's stores, so the build waits for them alone), barrier, load
    // the next tile's coefficient bytes, then the lookups with the rolling prefetch of the next tile's
    // inputs and this tile's stores, and a barrier before the tables are rebuilt.
    lds_barrier();  // the edge pass's table readers are done
    uint32_t &s_next = *reinterpret_cast<uint32_t *>(lds + 2 * LDS_BYTES);
    uint32_t more;
    bool first = true;
#pragma unroll 1
    do {
#ifdef DECDS_PHASE_TRACE
        if (first) {  // slot 24: the first tile's coefficient bytes are in; slot 25: its tables are built
            asm volatile("s_waitcnt vmcnt(26)" ::: "memory");
            PT_STAMP(24);
        }
#endif
        build_tables<K, N>(lds, cw, poly);
#ifdef DECDS_PHASE_TRACE
        if (first) PT_STAMP(25);
#endif
        if constexpr (QUEUE) {
            // the counter's answer: at the first tile everything but its ten input loads and the 16
            // dropped stores, later everything but the previous tile's 16 stores (waited for whether
            // or not a counter was passed — with none, one tile per workgroup, grab is 0 — so that on
            // every path the pending atomic register is read after its wait: tests/test_isa.py)
            if (first)
                asm volatile("s_waitcnt vmcnt(26)" ::: "memory");
            else
                asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
            if (threadIdx.x == 0) s_next = DECDS_STATIC_SECOND ? (first ? t + G : 2 * G + grab) : G + grab;
        }
        first = false;
        lds_barrier();
#ifdef DECDS_PHASE_TRACE
        if (pt_tiles < 16) PT_STAMP(8 + pt_tiles);
        if (pt_tiles++ == 0) PT_STAMP(2);
#endif
        const uint32_t tn = QUEUE ? __builtin_amdgcn_readfirstlane(s_next) : t + G;
        sweep_guard(tn, t);
        grab = grab_next();
        more = tn < total;
        const uint32_t csn = more ? tn / T : cs;
        CoeffBytes cb = table_coeff_bytes<K, N>(coeffs + (size_t)csn * N * K, K);
        combine_block<K, N, DW, 0, NoSink, SAUX, true, DW == 4 ? DECDS_ENC_HB : DECDS_ENC_SMALL_HB>(x, dst + (size_t)cs * N * pitch, ooff, col_of(t),
                                                                  src + (size_t)csn * CS, ioff, more ? col_of(tn) : OOB_COL);
        cw = table_coeff_pack<K>(cb);
        lds_barrier();
        t = tn;
        cs = csn;
    } while (more);
#ifdef DECDS_PHASE_TRACE
    PT_STAMP(3);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    PT_STAMP(4);
    PT_SET(5, pt_tiles);
#endif
    // the last workgroup out resets the counter pair (tile counter, exit count) for the next launch
    // that takes this slot: no reset launch on the stream (a hipMemsetAsync was ~5 µs per encode)
    if (QUEUE && counter && threadIdx.x == 0) {
        if (atomicAdd(counter + 1, 1u) == G - 1) {
            __atomic_store_n(counter, 0u, __ATOMIC_RELAXED);
            __atomic_store_n(counter + 1, 0u, __ATOMIC_RELAXED);
        }
    }
}

// rlnc Decoder::get_decoded_data (chunkset.rs:202-204, restated in oracle/rlnc_oracle.c
// orc_decoder_get_decoded_data) cuts the concatenated decoded pieces (CS + 10 bytes) at the LAST
// boundary marker; no marker at all is an error (-> ChunksetRepairingFailed). An intact chunkset ends
// in marker || 9 zeros, so its cut is at CS. The edge pass decodes the 10 tail bytes [CS, CS + 10)
// (piece 9's last columns) and notes each and the highest marker among them in LDS (tail_note);
// after a barrier, when no tail byte is the marker (only corrupted rows, accepted unvalidated, get
// there), tail_scan_decoded looks for the last marker among the decoded bytes [0, CS), and
// tail_finish writes the repair info (decoded length, tail bytes) and the status.
struct TailLds {
    uint32_t cut;       // 1 + index of the last marker among the tail bytes, 0: none
    uint32_t bytes[3];  // the 10 tail bytes
    uint32_t scan;      // 1 + position of the last marker in [0, CS) (tail_scan_decoded), 0: none
    uint32_t pad[3];
};
constexpr uint32_t TAIL_LDS = sizeof(TailLds);
static_assert(TAIL_LDS == 32, "LDS layout");
__device__ __forceinline__ void tail_reset(TailLds &t) {
    if (threadIdx.x < TAIL_LDS / 4) reinterpret_cast<uint32_t *>(&t)[threadIdx.x] = 0;
}
__device__ __forceinline__ void tail_note(TailLds &t, uint64_t p, uint32_t z, uint32_t marker) {
    const uint32_t j = (uint32_t)(p - CS);
    reinterpret_cast<uint8_t *>(t.bytes)[j] = (uint8_t)z;
    if (z == marker) atomicMax(&t.cut, j + 1);
}
// The whole workgroup, after a barrier behind every tail_note; returns at once when a tail byte is
// the marker. Otherwise the decoded bytes are decoded again here from the accepted rows (the
// chunkset's tiles are being written by other workgroups at the same time), from the end of the
// chunkset down, WG x 16 positions per step, until a step holds a marker. A thread's 16 positions
// lie in one piece except at the 9 piece boundaries: it loads them as one unaligned 16-byte access
// per accepted row (10 loads, one round trip — round 4 loaded every byte: 160 loads per 16 positions,
// ADVICE r04), and byte by byte only across a boundary. tbl: the decode tables (input k, output i).
// Reached only by rows accepted unvalidated whose tail holds no marker; a chunkset with no marker at
// all is decoded once more in full by this one workgroup (tests/test_gpu_parity.py times that case).
__device__ __forceinline__ void tail_scan_decoded(TailLds &t, const uint8_t *tbl, const uint8_t *ibase, const uint32_t (&ioff)[K],
                                  uint32_t marker) {
    if (__builtin_amdgcn_readfirstlane(t.cut)) return;
    constexpr uint32_t STEP = WG * 16;
    static_assert(CS % STEP == 0, "whole steps");
    for (uint32_t blk = (uint32_t)CS; blk > 0;) {
        blk -= STEP;
        uint32_t h = 0;
        const uint32_t p0 = blk + threadIdx.x * 16, i0 = p0 / (uint32_t)L, col0 = p0 - i0 * (uint32_t)L;
        if (col0 + 16 <= (uint32_t)L) {
            u32x4 x[K];
#pragma unroll
            for (uint32_t k = 0; k < K; k++) x[k] = ldrow<4>(ibase, ioff[k], col0);
#pragma unroll
            for (uint32_t b = 0; b < 16; b++) {
                uint32_t z = 0;
#pragma unroll
                for (uint32_t k = 0; k < K; k++) z ^= tbl_mul(tbl, k, i0, (x[k][b >> 2] >> (8 * (b & 3))) & 0xFFu);
                if (z == marker) h = p0 + b + 1;  // positions rise with b: the last hit is the highest
            }
        } else {
#pragma unroll 1
            for (uint32_t b = 0; b < 16; b++) {
                const uint32_t p = p0 + b, i = p / (uint32_t)L, col = p - i * (uint32_t)L;
                uint32_t z = 0;
#pragma unroll
                for (uint32_t k = 0; k < K; k++) z ^= tbl_mul(tbl, k, i, ibase[ioff[k] + col]);
                if (z == marker) h = p + 1;
            }
        }
        // (not __syncthreads_or: HIP's keeps a static __shared__ word, which would move the dynamic
        // LDS area the tables' inline-asm reads address from byte 0)
        if (h) atomicMax(&t.scan, h);
        __syncthreads();
        const uint32_t found = __builtin_amdgcn_readfirstlane(t.scan);
        __syncthreads();  // every wave has read t.scan before a later step may raise it
        if (found) return;
    }
}
// after tail_scan_decoded; info: 4 dwords per chunkset (decds_repair_info)
__device__ __forceinline__ void tail_finish(const TailLds &t, uint32_t c, int32_t *status, uint32_t *info) {
    if (threadIdx.x != 0) return;
    if (info) {
        uint32_t *o = info + 4 * (size_t)c;
        o[0] = t.cut ? (uint32_t)CS + t.cut - 1 : t.scan ? t.scan - 1 : 0u;
        o[1] = t.bytes[0];
        o[2] = t.bytes[1];
        o[3] = t.bytes[2];
    }
    if (!t.cut && !t.scan) status[c] = 6;  // DECDS_ERR_CHUNKSET_REPAIRING_FAILED: no marker anywhere
}

// Decode: workgroup = UNIT consecutive tiles of one chunkset. The accepted rows of chunkset cs are
// rows plan.sel[k] of its 16-row group at coded + cs*16*pitch, or — gather form, in_bases != NULL —
// rows plan.sel[k] at in_bases[cs] + sel*pitch, written to out_bases[cs] (the incremental
// RepairingBlob keeps each chunkset's accepted rows in its own device slot).
// 4 waves per SIMD with lookup groups of 2 bytes (8 reads in flight per wave, 128 VGPRs) against
// round 2's 2 waves with groups of 4 (16 in flight, 149 VGPRs): -2...-6 % decode time at 103-1639
// chunksets on two boxes (r05e, r05f). More waves keep more piece stores in flight; groups of 1
// byte (105 VGPRs) lose some of it back, 5 waves spill. (Round 2's 3 waves were with groups of 4.)
#ifndef DECDS_DEC_WAVES
#define DECDS_DEC_WAVES 4
#endif
#ifndef DECDS_DEC_HB
#define DECDS_DEC_HB 2  // decode lookup group size (bytes of an input dword per group)
#endif
// piece stores of the one-tile decode write-through (`sc1`) for batches of up to DEC_WT_MAX_N
// chunksets: -4 % at 1 and 2 chunksets (end-of-kernel write-back, as the encode's), +1 % at 16,
// +6 % at 103 and +8 % at 255 (r06r); plain stores above
constexpr size_t DEC_WT_MAX_N = 2;
#ifndef DECDS_DEC_DW
#define DECDS_DEC_DW 4  // decode lane-block width in dwords (4: 16 columns per lane)
#endif
// DW: lane-block width of the one-tile form — DECDS_DEC_DW (16 columns), or 2 (8 columns: 512 tiles per
// chunkset) for batches up to DECDS_DEC_NARROW_MAX_N, where a chunkset's 256 wide tiles leave one workgroup
// per CU and its lookups run at half the CU's LDS rate (phase trace r09r: 4.7-5 us of a 1-chunkset repair)
template <uint32_t UNIT, int SAUX = 0, int DW = DECDS_DEC_DW>
__global__ __launch_bounds__(WG, DECDS_DEC_WAVES) __attribute__((amdgpu_waves_per_eu(DECDS_DEC_WAVES, DECDS_DEC_WAVES)))
void rlnc_decode_kernel(const uint8_t *__restrict__ coded, size_t pitch, size_t n, const RepairPlan *__restrict__ plan,
                        uint8_t *__restrict__ dst, int32_t *__restrict__ status, const uint64_t *__restrict__ in_bases,
                        const uint64_t *__restrict__ out_bases, uint32_t poly, uint32_t marker,
                        uint32_t *__restrict__ info) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    tables_at_lds_zero();
    TailLds &s_tail = *reinterpret_cast<TailLds *>(lds + LDS_BYTES);
    constexpr uint32_t T = TILES<DW>;
    static_assert(T % UNIT == 0, "a workgroup's tiles stay in one chunkset");
    constexpr uint32_t phase = 0;  // aligned decode loads measured slower (+3…+5 %, profiles/HISTORY.md §8)
    // Workgroups are dealt round-robin over the 8 XCDs. Piece i's stores start i bytes past a line
    // boundary, so the line at every tile edge is written partly by each of two workgroups; when those
    // sit on different XCDs both L2s write back a partial line. Runs of R consecutive tiles go to one
    // XCD instead (block 8R·g + 8j + x -> tile 8R·g + R·x + j), global order otherwise: only every R-th
    // tile edge crosses an L2 (-3 % decode time, profiles/HISTORY.md §8).
    uint32_t u = blockIdx.x;
    if constexpr (DEC_XCD_RUN > 1) {
        constexpr uint32_t R = DEC_XCD_RUN;
        if (gridDim.x % (8 * R) == 0) u = (u / (8 * R)) * 8 * R + (u % 8) * R + (u / 8) % R;
    }
    const uint32_t t0 = u * UNIT, cs = t0 / T, tile0 = t0 % T;
    PT_STAMP(0);
    if (cs >= n) return;
    const uint32_t *pw = reinterpret_cast<const uint32_t *>(plan + cs);
    const uint32_t w0 = __builtin_amdgcn_readfirstlane(pw[0]);
    const uint32_t w1 = __builtin_amdgcn_readfirstlane(pw[1]);
    const uint32_t w2 = __builtin_amdgcn_readfirstlane(pw[2]);
    if (((w2 >> 16) & 0xFFu) != K) return;  // RepairPlan::rank at byte 10: not ready
    const uint32_t sel[K] = {w0 & 0xFFu, (w0 >> 8) & 0xFFu, (w0 >> 16) & 0xFFu, w0 >> 24,
                             w1 & 0xFFu, (w1 >> 8) & 0xFFu, (w1 >> 16) & 0xFFu, w1 >> 24,
                             w2 & 0xFFu, (w2 >> 8) & 0xFFu};
    uint32_t ioff[K], ooff[K];
#pragma unroll
    for (int k = 0; k < (int)K; k++) ioff[k] = (uint32_t)(sel[k] * pitch + K);
#pragma unroll
    for (int i = 0; i < (int)K; i++) ooff[i] = piece_off(i);
    const uint8_t *ibase;
    uint8_t *obase;
    if (in_bases) {
        ibase = reinterpret_cast<const uint8_t *>(uniform_u64(in_bases[cs]));
        obase = reinterpret_cast<uint8_t *>(uniform_u64(out_bases[cs]));
    } else {
        ibase = coded + (size_t)cs * N * pitch;
        obase = dst + (size_t)cs * CS;
    }
    // the input-major inverse's coefficient words as one dword load each, ahead of the tile's loads so
    // that the table build waits for it alone (the byte-wise table_coeffs, with a branch per output
    // past 10, waited for each of its loads in turn: three HBM round trips before the tile's own loads
    // were issued, r06z4)
    const uint32_t cw = table_coeffs_imaj<K, K>(plan[cs].inv);
    Vec<DW> x[K];
    if constexpr (DECDS_PREFETCH_FIRST) load_block<K, DW>(x, ibase, ioff, tile_col<DW, false>(tile0, tile0 + UNIT, phase));
    if (tile0 == 0) tail_reset(s_tail);
    build_tables<K, K>(lds, cw, poly);
    lds_barrier();
    PT_STAMP(4);
    auto edge_pass = [&]() {
        // the workgroup of tile 0 makes one pass over the edge columns — after its tile, so that no
        // branch ahead of the tile's stream merges memory-counter pictures (which had the lookups wait for
        // all ten loads, vmcnt(0), instead of each as it is consumed). With the one-dword coefficient
        // load: -6 / -6 / -2 % decode time at 1 / 16 / 64 chunksets, ±1 % at 103-255 (r06z4, r06z5)
        if (tile0 == 0) {
            // the 10 bytes past the chunkset (piece 9's marker || zeros when intact) decide where
            // get_decoded_data cuts (tail_note, chunkset.rs:202-204)
            for (uint32_t idx = threadIdx.x; idx < edge_cols<DW, false>(phase) * K; idx += WG) {
                const uint32_t i = idx % K, col = edge_col<DW, false>(idx / K, phase);
                uint32_t z = 0;
#pragma unroll
                for (uint32_t k = 0; k < K; k++) z ^= tbl_mul(lds, k, i, ibase[ioff[k] + col]);
                const uint64_t p = (uint64_t)i * L + col;
                if (p < CS)
                    obase[p] = (uint8_t)z;
                else
                    tail_note(s_tail, p, z, marker);
            }
            lds_barrier();
            tail_scan_decoded(s_tail, lds, ibase, ioff, marker);
            tail_finish(s_tail, cs, status, info);
        }
    };
    // (realigning the piece stores — pieces start i bytes past alignment — through LDS staging or a DPP
    // wave shift measured 4-5 % slower / spilled: r02v/w)
    stream_range<K, K, DW, DECDS_PREFETCH_FIRST, false, DECDS_DEC_HB, SAUX>(tile0, tile0 + UNIT, phase, ibase, ioff, obase, ooff, x);
    PT_STAMP(5);
    edge_pass();
#ifdef DECDS_PHASE_TRACE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    PT_STAMP(6);
#endif
}

// 3 waves/SIMD for the decode sweep: at 4 (128 VGPRs) its loop spills, the tile counter's pending
// return register among what it spills (tests/test_isa.py checks the built code for exactly that)
#ifndef DECDS_DEC_REMAT
// the decode sweep recomputes its table-build addresses per tile: 149 against 165 VGPRs, time ±0.1 %
// (r05v); the same in the encode sweep cost 5.6 % (r05u, not used there)
#define DECDS_DEC_REMAT 1
#endif
#ifndef DECDS_DEC_SWEEP_WAVES
#define DECDS_DEC_SWEEP_WAVES 3
#endif

// A chunkset's decode operands: coded-row offsets of the accepted chunks, input/output bases and
// whether it is ready. The raw loads are issued first (load) and turned into wave-uniform values
// later (resolve), so their latency hides behind whatever the caller issues in between.
struct DecodeDesc {
    uint32_t v0, v1, v2;
    uint64_t vin, vout;
    uint32_t ioff[K];
    const uint8_t *ibase;
    uint8_t *obase;
    bool ready;
    __device__ __forceinline__ void load(const RepairPlan *plan, const uint64_t *in_bases, const uint64_t *out_bases,
                                         uint32_t c) {
        const uint32_t *pw = reinterpret_cast<const uint32_t *>(plan + c);
        v0 = pw[0];
        v1 = pw[1];
        v2 = pw[2];
        if (in_bases) {
            vin = in_bases[c];
            vout = out_bases[c];
        }
    }
    __device__ __forceinline__ void resolve(const uint8_t *coded, uint8_t *dst, size_t pitch,
                                            const uint64_t *in_bases, uint32_t c) {
        const uint32_t w0 = __builtin_amdgcn_readfirstlane(v0), w1 = __builtin_amdgcn_readfirstlane(v1),
                       w2 = __builtin_amdgcn_readfirstlane(v2);
        ready = ((w2 >> 16) & 0xFFu) == K;  // RepairPlan::rank at byte 10
        const uint32_t sel[K] = {w0 & 0xFFu, (w0 >> 8) & 0xFFu, (w0 >> 16) & 0xFFu, w0 >> 24,
                                 w1 & 0xFFu, (w1 >> 8) & 0xFFu, (w1 >> 16) & 0xFFu, w1 >> 24,
                                 w2 & 0xFFu, (w2 >> 8) & 0xFFu};
#pragma unroll
        for (int k = 0; k < (int)K; k++) ioff[k] = (uint32_t)((sel[k] & 15u) * pitch + K);
        if (in_bases) {
            ibase = reinterpret_cast<const uint8_t *>(uniform_u64(vin));
            obase = reinterpret_cast<uint8_t *>(uniform_u64(vout));
        } else {
            ibase = coded + (size_t)c * N * pitch;
            obase = dst + (size_t)c * CS;
        }
    }
};

// The decode as a persistent sweep (study variant, DECDS_DEC_SWEEP): resident workgroups take tiles
// in global order from a tile counter, like the encode sweep, so a workgroup's next tile's coded
// rows load while it combines the current one (the one-tile workgroups of rlnc_decode_kernel wait
// for their loads up front: 42 % of their wave cycles are spent waiting, r05h PMC). A tile's rows
// depend on its chunkset's plan, so the counter runs one tile further ahead than in the encode: the
// next tile is known at the top of an iteration and its plan loads there, under the table build.
template <int DW, int WAVES, int HB>
__global__ __launch_bounds__(WG, WAVES) __attribute__((amdgpu_waves_per_eu(WAVES, WAVES)))
void rlnc_decode_sweep_kernel(const uint8_t *__restrict__ coded, size_t pitch, size_t n,
                              const RepairPlan *__restrict__ plan, uint8_t *__restrict__ dst,
                              int32_t *__restrict__ status, const uint64_t *__restrict__ in_bases,
                              const uint64_t *__restrict__ out_bases, uint32_t poly, uint32_t marker,
                              uint32_t *__restrict__ counter, uint32_t *__restrict__ info) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    tables_at_lds_zero();
    TailLds &s_tail = *reinterpret_cast<TailLds *>(lds + 2 * LDS_BYTES + 16);
    constexpr uint32_t T = TILES<DW>;
    constexpr uint32_t phase = 0;
    uint32_t ooff[K];
#pragma unroll
    for (int i = 0; i < (int)K; i++) ooff[i] = piece_off(i);
    // 1. edge columns of the ready chunksets b, b + gridDim, ... (tables in buffer 1)
    for (uint32_t c = blockIdx.x; c < n; c += gridDim.x) {
        DecodeDesc d;
        d.load(plan, in_bases, out_bases, c);
        d.resolve(coded, dst, pitch, in_bases, c);
        if (!d.ready) continue;
        const uint32_t cw = table_coeffs_imaj<K, K>(plan[c].inv);  // input-major inverse, one dword load
        lds_barrier();  // also: the previous chunkset's tail_finish has read s_tail
        tail_reset(s_tail);
        build_tables<K, K>(lds + LDS_BYTES, cw, poly);
        lds_barrier();
        // the tail bytes decide where get_decoded_data cuts (chunkset.rs:202-204, as rlnc_decode_kernel)
        for (uint32_t idx = threadIdx.x; idx < edge_cols<DW, false>(phase) * K; idx += WG) {
            const uint32_t i = idx % K, col = edge_col<DW, false>(idx / K, phase);
            uint32_t z = 0;
#pragma unroll
            for (uint32_t k = 0; k < K; k++) z ^= tbl_mul(lds + LDS_BYTES, k, i, d.ibase[d.ioff[k] + col]);
            const uint64_t p = (uint64_t)i * L + col;
            if (p < CS)
                d.obase[p] = (uint8_t)z;
            else
                tail_note(s_tail, p, z, marker);
        }
        lds_barrier();
        tail_scan_decoded(s_tail, lds + LDS_BYTES, d.ibase, d.ioff, marker);
        tail_finish(s_tail, c, status, info);
    }
    // 2. the sweep (tiles in runs per XCD, each XCD with its own counter — rlnc_decode_kernel's
    // DEC_XCD_RUN — measured 1-2 % slower here at runs of 4, 8 and 16, r05q)
    const uint32_t total = (uint32_t)((uint64_t)n * T), G = gridDim.x;
    uint32_t k = blockIdx.x;  // this workgroup's tile
    if (k >= total) return;
    auto col_of = [&](uint32_t tt) { return tile_col<DW, false>(tt % T, T, phase); };
    auto grab_next = [&]() -> uint32_t {  // inline asm for the reason given in rlnc_encode_sweep_kernel
        uint32_t r = 0;
        if (counter && threadIdx.x == 0)
            asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(r) : "v"(counter), "v"(1u) : "memory");
        return r;
    };
    uint32_t &s_next = *reinterpret_cast<uint32_t *>(lds + 2 * LDS_BYTES);
    uint32_t cs = k / T;
    DecodeDesc cur, nxt;
    cur.load(plan, in_bases, out_bases, cs);
    uint32_t cw = table_coeffs_imaj<K, K>(plan[cs].inv);
    cur.resolve(coded, dst, pitch, in_bases, cs);
    uint32_t colt = cur.ready ? col_of(k) : OOB_COL;
    Vec<DW> x[K];
    load_block<K, DW>(x, cur.ibase, cur.ioff, colt);
#if DECDS_STATIC_SECOND
    uint32_t grab = 0;  // the second tile is static (k + G): the first grab goes out in the loop
    lds_barrier();      // the edge pass's table readers are done
    uint32_t kn = k + G;
#else
    uint32_t grab = grab_next();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) s_next = counter ? G + grab : k + G;
    lds_barrier();  // also: the edge pass's table readers are done
    uint32_t kn = __builtin_amdgcn_readfirstlane(s_next);
#endif
    sweep_guard(kn, k);
    uint32_t more;
#pragma unroll 1
    do {
        more = kn < total;
        const uint32_t csn = more ? kn / T : cs;
        nxt.load(plan, in_bases, out_bases, csn);
        const uint32_t cwn = table_coeffs_imaj<K, K>(plan[csn].inv);
        build_tables<K, K, DECDS_DEC_REMAT>(lds, cw, poly);
        lds_barrier();
        grab = grab_next();  // -> the tile after the next
        asm volatile("" ::: "memory");
        nxt.resolve(coded, dst, pitch, in_bases, csn);
        const uint32_t coln = more && nxt.ready ? col_of(kn) : OOB_COL;
        combine_block<K, K, DW, 0, NoSink, 0, true, HB>(x, cur.obase, ooff, colt, nxt.ibase, nxt.ioff, coln);
        // the counter's answer: everything but this tile's 2K prefetch loads and stores has landed
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * K) : "memory");
        if (threadIdx.x == 0) s_next = counter ? (DECDS_STATIC_SECOND ? 2 * G : G) + grab : kn + G;
        lds_barrier();
        k = kn;
        kn = __builtin_amdgcn_readfirstlane(s_next);
        sweep_guard(kn, k);
        cs = csn;
        cur = nxt;
        cw = cwn;
        colt = coln;
    } while (more);
    if (counter && threadIdx.x == 0) {  // the last workgroup out resets the counter pair
        if (atomicAdd(counter + 1, 1u) == G - 1) {
            __atomic_store_n(counter, 0u, __ATOMIC_RELAXED);
            __atomic_store_n(counter + 1, 0u, __ATOMIC_RELAXED);
        }
    }
}

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
// Products are log-domain: x * f = exp[log x + log f], with log 0 = PLAN_LOG0 and exp zero from
// index 765 on, so a product with a zero factor reads a zero and no term needs a mask. The basis
// is kept with its logs and every candidate's log is read up front, so a step is four dependent
// LDS reads (projection, log of the reduced row, normalised row + basis update, basis logs); the
// exp table comes from the host as a kernel argument. Most chunksets never get
// here: plan_fast inverts the first ten candidates directly when they are valid and independent.
struct GfExpTable {
    uint32_t w[64];  // byte i = gen^i (i < 255), byte 255 = 0
};
// exp[i] = gen^(i mod 255) for i < 765 (three periods: a sum of up to three logs needs no reduction), zero
// from 765 to the largest index, log0 + 255 + log0 (plan_fast's unreduced pivot-row products)
constexpr uint32_t PLAN_LOG0 = 1024;
constexpr uint32_t PLAN_EXP_VALID = 3 * 255;
constexpr uint32_t PLAN_EXP_BYTES = 2 * PLAN_LOG0 + 256;
// the plan's LDS scratch: exp / log tables and the logs of every coded row's coding vector
struct PlanLds {
    uint8_t exp[PLAN_EXP_BYTES];
    uint16_t log[256];
    uint16_t lcv[N * 16];  // log of byte c of row r's coding vector at r * 16 + c
    uint8_t cv[N * 16];    // byte c of row r's coding vector at r * 16 + c
};

// LDS visibility among the lanes of one wave: its LDS operations complete in order, so waiting for
// them is enough (the fused kernel's plan runs on one wave while the others wait at a barrier)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
}

// The plan of chunkset cs on one wave (lane = threadIdx.x & 63): writes *pl (rank always; sel and the
// input-major inverse when ready) and, when status is given, status[cs]; returns lane a's verdict for
// candidate a (< 16). WAVE_SYNC: the caller's other waves do not take part (wave-level LDS syncs).
#ifndef DECDS_STUDY_PLAN
#define DECDS_STUDY_PLAN 0  // timing studies of the plan (1: no elimination, 2: no coding-vector loads)
#endif
#ifndef DECDS_PLAN_FAST
#define DECDS_PLAN_FAST 1  // 0: the incremental elimination for every chunkset (A/B builds)
#endif
// The plan's fast path, for the common case: the first ten candidates in arrival order are valid and
// independent, so the rank test accepts exactly them (chunkset.rs:177-183) and every later candidate
// is "ready to repair". Their inverse is then found by Gauss-Jordan elimination on the augmented
// matrix [R | I] column by column — row s (after a swap when its entry is zero) is the pivot of column
// s and column s is cleared from all nine other rows at once — so a column costs two dependent LDS
// round trips (the products exp[log row + log factor], then the logs of the updated rows) where the
// incremental form needs five per accepted row. A column without a pivot means the ten rows are
// dependent: false, and the caller runs the incremental form, which decides which rows are accepted.
// Lane c < 20 holds column c of every row; the factors are the rows' logs at lane s (readlane).
__device__ __forceinline__ bool plan_fast(uint32_t lane, uint32_t my_cand, const PlanLds &sl, RepairPlan *pl,
                                          int32_t *__restrict__ status, size_t cs, int32_t *verdict) {
    const uint8_t *s_exp = sl.exp;
    const uint16_t *s_log = sl.log;
    const bool col = lane < K;
    uint32_t M[K], LM[K];
    const uint32_t c = col ? lane : 0u;
#pragma unroll
    for (int i = 0; i < (int)K; i++) {
        const uint32_t r = __builtin_amdgcn_readlane(my_cand, i);  // < N (checked by the caller)
        const uint32_t v = sl.cv[r * 16 + c];
        M[i] = col ? v : (lane == K + i ? 1u : 0u);
    }
#pragma unroll
    for (int i = 0; i < (int)K; i++) LM[i] = s_log[M[i]];
#pragma unroll
    for (int s = 0; s < (int)K; s++) {
        uint32_t f[K];
#pragma unroll
        for (int i = 0; i < (int)K; i++) f[i] = __builtin_amdgcn_readlane(LM[i], s);
        if (f[s] == PLAN_LOG0) {  // zero pivot: swap in the first later row with a nonzero entry
            int q = -1;
#pragma unroll
            for (int j = s + 1; j < (int)K; j++)
                if (q < 0 && f[j] != PLAN_LOG0) q = j;
            if (q < 0) return false;  // no pivot: the ten rows are dependent
#pragma unroll
            for (int j = s + 1; j < (int)K; j++)
                if (j == q) {
                    const uint32_t m = M[s], lm = LM[s], ff = f[s];
                    M[s] = M[j], LM[s] = LM[j], f[s] = f[j];
                    M[j] = m, LM[j] = lm, f[j] = ff;
                }
        }
        // row i -= (row i's entry / pivot) * pivot row, row s /= pivot: log row s + (255 - log pivot)
        // [+ log of row i's entry], the uniform part summed on the scalar unit; unreduced, every index
        // stays below PLAN_EXP_BYTES (a nonzero product below 765, one with a zero entry or factor at
        // log0 or above, where the table reads zero), so no term needs a mask or a reduction
        const uint32_t u = 255u - f[s];
#pragma unroll
        for (int i = 0; i < (int)K; i++) M[i] = i == s ? (uint32_t)s_exp[LM[s] + u] : M[i] ^ (uint32_t)s_exp[LM[s] + (u + f[i])];
        if (s + 1 < (int)K) {
#pragma unroll
            for (int i = 0; i < (int)K; i++) LM[i] = s_log[M[i]];
        }
    }
    // row s is now [e_s | row s of the inverse]: lane 10 + k writes inverse entry (s, k), input-major
    if (lane >= K && lane < 2 * K) {
#pragma unroll
        for (int s = 0; s < (int)K; s++) pl->inv[(lane - K) * K + s] = (uint8_t)M[s];
    }
    if (lane < K) pl->sel[lane] = (uint8_t)my_cand;
    if (lane == 0) {
        pl->rank = (uint8_t)K;
        if (status) status[cs] = 0;
    }
    // verdicts: accepted (0) for the ten, "ready to repair" (3) for the later ones up to the list's end
    const uint64_t ends = __ballot(lane < N && my_cand >= N) | (1ull << N);
    const uint32_t end = (uint32_t)__builtin_ctzll(ends & ~((1ull << K) - 1));
    *verdict = lane < K ? 0 : (lane < end ? 3 : -1);
    return true;
}
struct NoHook {
    __device__ __forceinline__ void operator()() const {}
};
template <bool WAVE_SYNC, class AfterLoads = NoHook>
__device__ __forceinline__ int32_t plan_wave(const uint8_t *__restrict__ coded, size_t pitch, size_t cs,
                                             const uint8_t *__restrict__ cand, PlanLds &sl, const GfExpTable &tab,
                                             RepairPlan *pl, int32_t *__restrict__ status,
                                             AfterLoads after_loads = AfterLoads()) {
    const uint32_t lane = threadIdx.x & 63u;
    const bool col = lane < K;
    // the arrival order and the coding vector of every coded row of the chunkset (lane c < 10
    // loads byte c of rows 0..15): all in flight while the tables below are built
    const uint32_t my_cand = lane < N ? cand[cs * N + lane] : (uint32_t)DECDS_NO_CANDIDATE_U8;
    uint32_t rowcv[N];
#pragma unroll
#if DECDS_STUDY_PLAN == 2  // timing study: no coding-vector loads (a fixed full-rank pattern instead)
    for (int r = 0; r < (int)N; r++) rowcv[r] = col ? ((uint32_t)(r * 37 + lane * 11 + cs) & 0xFFu) | 1u : 0u;
#else
    for (int r = 0; r < (int)N; r++) rowcv[r] = col ? coded[(cs * N + r) * pitch + lane] : 0u;
#endif
    after_loads();  // (the fused kernel issues its speculative tile loads here, behind the plan's own)
    uint8_t *s_exp = sl.exp;
    uint16_t *s_log = sl.log, *s_lcv = sl.lcv;
    {
        // exp[i] = gen^(i mod 255) for i < 765, zeros after (PLAN_EXP_BYTES)
        const uint32_t e4 = tab.w[lane];  // exp[4 lane .. 4 lane + 3]
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
            const uint32_t i = 4 * lane + q, v = (e4 >> (8 * q)) & 0xFFu;
            if (i < 255) {
                s_exp[i] = (uint8_t)v;
                s_exp[i + 255] = (uint8_t)v;
                s_exp[i + 510] = (uint8_t)v;
                s_log[v] = (uint16_t)i;
            }
        }
        for (uint32_t w = 768 / 4 + lane; w < PLAN_EXP_BYTES / 4; w += 64) reinterpret_cast<uint32_t *>(s_exp)[w] = 0;
        if (lane < 3) s_exp[PLAN_EXP_VALID + lane] = 0;
        if (lane == 0) s_log[0] = PLAN_LOG0;
        if (col) {
#pragma unroll
            for (int r = 0; r < (int)N; r++) sl.cv[r * 16 + lane] = (uint8_t)rowcv[r];
        }
    }
    if constexpr (WAVE_SYNC) wave_lds_sync(); else __syncthreads();
    PT_STAMP(1);
#if DECDS_PLAN_FAST && DECDS_STUDY_PLAN == 0
    if (!__ballot(lane < K && my_cand >= N)) {  // the first ten candidates exist
        int32_t v = -1;
        if (plan_fast(lane, my_cand, sl, pl, status, cs, &v)) {
            PT_STAMP(2);
            return v;
        }
    }
#endif
    // the incremental form: every coded row's logs
    if (col) {
#pragma unroll
        for (int r = 0; r < (int)N; r++) s_lcv[r * 16 + lane] = s_log[rowcv[r]];
    }
    if constexpr (WAVE_SYNC) wave_lds_sync(); else __syncthreads();
#if DECDS_STUDY_PLAN == 1  // timing study: loads and tables only, no elimination
    if (lane == 0) pl->rank = (uint8_t)(s_lcv[lane] & 1u);
    if (lane == 0 && status) status[cs] = 5;
    return -1;
#endif
    // Basis slot k is filled by the k-th accepted candidate, so the slot loop is unrolled with k a
    // constant: step k reduces against k basis rows only, and the pivots stay in SGPRs. Candidates
    // are taken in arrival order by a uniform inner loop until one raises the rank.
    uint32_t basis[K], lgb[K], piv[K], sel[K];  // lgb[e] = log basis[e] (PLAN_LOG0 where 0)
    uint32_t a = 0, rank = 0;                     // next candidate; rank = accepted so far
    bool stop = false;                            // the arrival list ended (no candidate / id >= 16)
    int32_t my_verdict = -1;                      // lane a < 16 keeps candidate a's verdict
#pragma unroll
    for (int k = 0; k < (int)K; k++) {
        basis[k] = 0;
        lgb[k] = PLAN_LOG0;
        piv[k] = sel[k] = 0;
        if (stop || rank < (uint32_t)k) continue;
        while (true) {
            const uint32_t r = a < N ? __builtin_amdgcn_readlane(my_cand, a) : N;
            if (r >= N) {
                stop = true;
                break;
            }
            const uint32_t lcv = col ? (uint32_t)s_lcv[r * 16 + lane] : PLAN_LOG0;
            // augmented row [cv | unit(k)] minus its projection on the basis: the factor of basis row
            // e is the row's entry at pivot e
            uint32_t row = col ? (uint32_t)s_exp[lcv] : (lane == K + k ? 1u : 0u);
#pragma unroll
            for (int e = 0; e < k; e++) row ^= s_exp[lgb[e] + __builtin_amdgcn_readlane(lcv, piv[e])];
            const uint64_t nz = __ballot(col && row != 0);
            if (!nz) {
                if (lane == a) my_verdict = 4;  // DECDS_ERR_CHUNK_DECODING_FAILED: piece not useful
                a++;
                continue;
            }
            const uint32_t p = __builtin_ctzll(nz);
            // row /= row[p] in logs: lrow = log row - log row[p] (mod 255), log0 kept
            const uint32_t lrow0 = s_log[row];
            const uint32_t linv = 255u - __builtin_amdgcn_readlane(lrow0, p);
            const uint32_t ls = lrow0 + linv;
            const uint32_t lrow = lrow0 >= PLAN_LOG0 ? PLAN_LOG0 : (ls >= 255u ? ls - 255u : ls);
            // clear column p from the basis: basis[e] -= basis[e][p] * row
#pragma unroll
            for (int e = 0; e < k; e++) basis[e] ^= s_exp[lrow + __builtin_amdgcn_readlane(lgb[e], p)];
#pragma unroll
            for (int e = 0; e < k; e++) lgb[e] = s_log[basis[e]];
            basis[k] = s_exp[lrow];
            lgb[k] = lrow;
            piv[k] = p;
            sel[k] = r;
            if (lane == a) my_verdict = 0;
            a++;
            rank++;
            break;
        }
    }
    // after rank 10 every further candidate is "ready to repair", up to the end of the list
    if (rank == K) {
        while (a < N && __builtin_amdgcn_readlane(my_cand, a) < N) {
            if (lane == a) my_verdict = 3;  // DECDS_ERR_CHUNKSET_READY_TO_REPAIR
            a++;
        }
    }
    if (lane == 0) pl->rank = (uint8_t)rank;
    if (rank < K) {
        if (lane == 0 && status) status[cs] = 5;  // DECDS_ERR_CHUNKSET_NOT_YET_READY
        return my_verdict;
    }
    // inverse row piv[e] = combination part of basis row e: lane 10 + k writes inverse entry
    // (piv[e], k), stored input-major at k * K + piv[e] (so a table build reads 4 outputs' coefficients
    // of one input as one dword, table_coeffs_imaj)
    if (lane >= K && lane < 2 * K) {
#pragma unroll
        for (int e = 0; e < (int)K; e++) pl->inv[(lane - K) * K + piv[e]] = (uint8_t)basis[e];
    }
    if (lane == 0) {
#pragma unroll
        for (int e = 0; e < (int)K; e++) pl->sel[e] = (uint8_t)sel[e];
        if (status) status[cs] = 0;
    }
    return my_verdict;
}

__global__ __launch_bounds__(64) void rlnc_plan_kernel(const uint8_t *__restrict__ coded, size_t pitch, size_t n,
                                                       const uint8_t *__restrict__ cand,
                                                       RepairPlan *__restrict__ plan,
                                                       int8_t *__restrict__ verdicts,
                                                       int32_t *__restrict__ status, GfExpTable tab) {
    __shared__ __attribute__((aligned(16))) PlanLds sl;
    const size_t cs = blockIdx.x;
    const int32_t v = plan_wave<false>(coded, pitch, cs, cand, sl, tab, plan + cs, status);
    if (threadIdx.x < N) verdicts[cs * N + threadIdx.x] = (int8_t)v;
}

// table_coeffs_imaj from an input-major inverse held in LDS (the fused plan + decode's own plan)
template <int NIN, int NOUT>
__device__ __forceinline__ uint32_t table_coeffs_imaj_lds(const uint8_t *M) {
    const uint32_t p0 = threadIdx.x;
    const bool live = p0 < NIN * 8;
    const uint32_t p = live ? p0 : 0u, q = p & 3u, i = p >> 3;
    uint32_t w = 0;
#pragma unroll
    for (uint32_t jj = 0; jj < 4; jj++)
        if (4 * q + jj < (uint32_t)NOUT) w |= (uint32_t)M[i * NOUT + 4 * q + jj] << (8 * jj);
    return live ? w : 0u;
}

// Repair of a small batch as ONE launch (decds_repair_batch for n <= DECDS_PLAN_DECODE_MAX_N): the
// one-tile decode (rlnc_decode_kernel) whose workgroups first run their chunkset's plan themselves —
// wave 0 replays the rank test and inverts the accepted coding vectors (plan_wave, into LDS) while
// the other waves wait at the barrier; the workgroup of tile 0 also writes the plan, the verdicts and
// the status to memory, as rlnc_plan_kernel would. Every workgroup of a chunkset computes the same
// plan (256 per chunkset, 512 with 8-column tiles: the plan's few microseconds of one wave, in
// parallel, against a second launch and its plan round trip through memory). Same bytes as plan +
// decode.
template <int SAUX = 0, int DW = DECDS_DEC_DW>
__global__ __launch_bounds__(WG, DECDS_DEC_WAVES) __attribute__((amdgpu_waves_per_eu(DECDS_DEC_WAVES, DECDS_DEC_WAVES)))
void rlnc_plan_decode_kernel(const uint8_t *__restrict__ coded, size_t pitch, size_t n, const uint8_t *__restrict__ cand,
                             RepairPlan *__restrict__ plan, int8_t *__restrict__ verdicts, uint8_t *__restrict__ dst,
                             int32_t *__restrict__ status, uint32_t poly, uint32_t marker, uint32_t *__restrict__ info,
                             GfExpTable tab) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    tables_at_lds_zero();
    TailLds &s_tail = *reinterpret_cast<TailLds *>(lds + LDS_BYTES);
    PlanLds &s_plan = *reinterpret_cast<PlanLds *>(lds + LDS_BYTES + TAIL_LDS);
    RepairPlan &s_rp = *reinterpret_cast<RepairPlan *>(lds + LDS_BYTES + TAIL_LDS + sizeof(PlanLds));
    constexpr uint32_t T = TILES<DW>;
    constexpr uint32_t phase = 0;
    uint32_t u = blockIdx.x;
    if constexpr (DEC_XCD_RUN > 1) {  // runs of consecutive tiles per XCD, as rlnc_decode_kernel
        constexpr uint32_t R = DEC_XCD_RUN;
        if (gridDim.x % (8 * R) == 0) u = (u / (8 * R)) * 8 * R + (u % 8) * R + (u / 8) % R;
    }
    const uint32_t cs = u / T, tile0 = u % T;
    PT_STAMP(0);
    if (cs >= n) return;
    const bool first = tile0 == 0;
    const uint8_t *ibase = coded + (size_t)cs * N * pitch;
    // Speculative first loads: the first ten candidates in arrival order are the accepted rows in the
    // common case (exactly ten survivors, or the first ten of more: independent with probability 0.996),
    // so every wave issues its tile's loads from those rows before (wave 0: behind the plan's own loads)
    // the plan is known; a plan that accepted other rows reloads below.
    const uint32_t *cw = reinterpret_cast<const uint32_t *>(cand + (size_t)cs * N);
    const uint32_t c0 = __builtin_amdgcn_readfirstlane(cw[0]), c1 = __builtin_amdgcn_readfirstlane(cw[1]),
                   c2 = __builtin_amdgcn_readfirstlane(cw[2]) & 0xFFFFu;
    const uint32_t spec_sel[K] = {c0 & 0xFFu, (c0 >> 8) & 0xFFu, (c0 >> 16) & 0xFFu, c0 >> 24,
                                  c1 & 0xFFu, (c1 >> 8) & 0xFFu, (c1 >> 16) & 0xFFu, c1 >> 24,
                                  c2 & 0xFFu, c2 >> 8};
    bool spec_ok = true;
#pragma unroll
    for (int k = 0; k < (int)K; k++) spec_ok &= spec_sel[k] < N;
    uint32_t soff[K];
#pragma unroll
    for (int k = 0; k < (int)K; k++) soff[k] = (uint32_t)((spec_sel[k] & 15u) * pitch + K);
    Vec<DW> x[K];
    const uint32_t col0 = tile_col<DW, false>(tile0, tile0 + 1, 0);
    auto speculate = [&]() {
        if (spec_ok) load_block<K, DW>(x, ibase, soff, col0);
    };
    if (threadIdx.x < 64) {
        const int32_t v = plan_wave<true>(coded, pitch, cs, cand, s_plan, tab, &s_rp, first ? status : nullptr, speculate);
        if (first && threadIdx.x < N) verdicts[(size_t)cs * N + threadIdx.x] = (int8_t)v;
    } else {
        speculate();
    }
    if (first) tail_reset(s_tail);
    lds_barrier();
    PT_STAMP(3);
    const uint32_t *pw = reinterpret_cast<const uint32_t *>(&s_rp);
    if (first && threadIdx.x < sizeof(RepairPlan) / 4)  // the plan, as rlnc_plan_kernel leaves it
        reinterpret_cast<uint32_t *>(plan + cs)[threadIdx.x] = pw[threadIdx.x];
    const uint32_t w0 = __builtin_amdgcn_readfirstlane(pw[0]);
    const uint32_t w1 = __builtin_amdgcn_readfirstlane(pw[1]);
    const uint32_t w2 = __builtin_amdgcn_readfirstlane(pw[2]);
    if (((w2 >> 16) & 0xFFu) != K) return;  // RepairPlan::rank at byte 10: not ready
    const uint32_t sel[K] = {w0 & 0xFFu, (w0 >> 8) & 0xFFu, (w0 >> 16) & 0xFFu, w0 >> 24,
                             w1 & 0xFFu, (w1 >> 8) & 0xFFu, (w1 >> 16) & 0xFFu, w1 >> 24,
                             w2 & 0xFFu, (w2 >> 8) & 0xFFu};
    uint32_t ioff[K], ooff[K];
#pragma unroll
    for (int k = 0; k < (int)K; k++) ioff[k] = (uint32_t)(sel[k] * pitch + K);
#pragma unroll
    for (int i = 0; i < (int)K; i++) ooff[i] = piece_off(i);
    uint8_t *obase = dst + (size_t)cs * CS;
    const uint32_t tcw = table_coeffs_imaj_lds<K, K>(s_rp.inv);
    if (!spec_ok || w0 != c0 || w1 != c1 || (w2 & 0xFFFFu) != c2) load_block<K, DW>(x, ibase, ioff, col0);  // misspeculated
    build_tables<K, K>(lds, tcw, poly);
    lds_barrier();
    PT_STAMP(4);
    stream_range<K, K, DW, true, false, DECDS_DEC_HB, SAUX>(tile0, tile0 + 1, phase, ibase, ioff, obase, ooff, x);
    PT_STAMP(5);
    if (first) {
        // the edge columns and get_decoded_data's cut, as rlnc_decode_kernel's edge pass
        for (uint32_t idx = threadIdx.x; idx < edge_cols<DW, false>(phase) * K; idx += WG) {
            const uint32_t i = idx % K, col = edge_col<DW, false>(idx / K, phase);
            uint32_t z = 0;
#pragma unroll
            for (uint32_t k = 0; k < K; k++) z ^= tbl_mul(lds, k, i, ibase[ioff[k] + col]);
            const uint64_t p = (uint64_t)i * L + col;
            if (p < CS)
                obase[p] = (uint8_t)z;
            else
                tail_note(s_tail, p, z, marker);
        }
        lds_barrier();
        tail_scan_decoded(s_tail, lds, ibase, ioff, marker);
        tail_finish(s_tail, cs, status, info);
    }
#ifdef DECDS_PHASE_TRACE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    PT_STAMP(6);
#endif
}
constexpr uint32_t PLAN_DEC_LDS = DEC_LDS + sizeof(PlanLds) + sizeof(RepairPlan);

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
// Column phase of the coded rows' payloads (edge_col): with a pitch that is a multiple of the
// lane-block width every row's payload (row + 10) has the same alignment, and encode blocks starting
// `phase` columns in store aligned. Other pitches keep phase 0.
template <int DW>
static uint32_t row_phase(const uint8_t *rows, size_t pitch) {
    constexpr uint32_t C = 4 * DW;
    if (pitch % C) return 0;
    return (uint32_t)((C - ((uintptr_t)rows + K) % C) % C);
}

// encode lane-block width and waves per SIMD: 16-column blocks, 2 waves (254 VGPRs). 8-column
// blocks at 3 waves per SIMD (168 VGPRs) measured no faster (r02g).
#ifndef DECDS_ENC_DW
#define DECDS_ENC_DW 4
#endif
#ifndef DECDS_ENC_WAVES
#define DECDS_ENC_WAVES 2
#endif
// fused ChunkSet::new (rlnc_encode_hash_kernel): 8-column blocks (128-byte steps) at 3 waves per SIMD;
// 16-column blocks (256-byte steps) at 2 waves per SIMD measured 9 % slower (r03d)
#ifndef DECDS_FH_DW
#define DECDS_FH_DW 2
#endif
#ifndef DECDS_FH_WAVES
#define DECDS_FH_WAVES 3
#endif
#define ENC_HASH rlnc_encode_hash_kernel<DECDS_FH_DW, DECDS_FH_WAVES>
// 16-byte-aligned rows (phase MSG_PHASE with 16-column blocks) take the message-tiled kernels
constexpr bool MSG_OK = DECDS_ENC_DW == 4;
#ifndef DECDS_ENC_QUEUE
#define DECDS_ENC_QUEUE 1
#endif
#define DEC_SWEEP rlnc_decode_sweep_kernel<DECDS_DEC_DW, DECDS_DEC_SWEEP_WAVES, DECDS_DEC_HB>
#define ENC_SWEEP(MSG, SAUX) rlnc_encode_sweep_kernel<DECDS_ENC_DW, DECDS_ENC_WAVES, MSG, (DECDS_ENC_QUEUE != 0), false, SAUX>
// small batches (DECDS_ENC_SMALL_MAX_N): 8-column lane blocks, 512 tiles per chunkset, 4 waves per SIMD
// (118 VGPRs) — one chunkset fills 512 workgroups (16-column tiles give 256 at n = 1); slower per byte
// from 4 chunksets on, where the 16-column form fills the grid too (r06c / r06j, profiles/HISTORY.md §8): threshold 2
#ifndef DECDS_ENC_SMALL_WAVES
#define DECDS_ENC_SMALL_WAVES 4
#endif
#ifndef DECDS_ENC_SMALL_EDGE
#define DECDS_ENC_SMALL_EDGE 1  // the small form's edge columns on their own workgroups (EDGE_SPLIT)
#endif
#define ENC_SMALL rlnc_encode_sweep_kernel<2, DECDS_ENC_SMALL_WAVES, false, (DECDS_ENC_QUEUE != 0), (DECDS_ENC_SMALL_EDGE != 0), STORE_SC1>

hipError_t configure_kernels() {
    const void *fns[] = {reinterpret_cast<const void *>(ENC_SWEEP(false, STORE_SC1)), reinterpret_cast<const void *>(ENC_SWEEP(MSG_OK, STORE_SC1)),
                         reinterpret_cast<const void *>(ENC_SWEEP(false, STORE_NT)), reinterpret_cast<const void *>(ENC_SWEEP(MSG_OK, STORE_NT)),
                         reinterpret_cast<const void *>(ENC_HASH), reinterpret_cast<const void *>(rlnc_decode_kernel<DEC_UNIT>),
                         reinterpret_cast<const void *>(rlnc_decode_kernel<DEC_UNIT, STORE_SC1>),
                         reinterpret_cast<const void *>(DEC_SWEEP), reinterpret_cast<const void *>(ENC_SMALL)};
    for (const void *f : fns) {
        hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, std::max(SWEEP_LDS, FH_LDS<DECDS_FH_DW>));
        if (e != hipSuccess) return e;
    }
    // every other kernel's code object resolved now, on the creating thread, not lazily by the first
    // launch — which may come from several caller threads at once (the coalesced ChunkSet::new)
    const void *rest[] = {reinterpret_cast<const void *>(rlnc_plan_kernel), reinterpret_cast<const void *>(rlnc_plan_decode_kernel<0>),
                          reinterpret_cast<const void *>(rlnc_plan_decode_kernel<STORE_SC1>),
                          reinterpret_cast<const void *>(rlnc_plan_decode_kernel<0, 2>),
                          reinterpret_cast<const void *>(rlnc_plan_decode_kernel<STORE_SC1, 2>),
                          reinterpret_cast<const void *>(rlnc_decode_kernel<DEC_UNIT, 0, 2>),
                          reinterpret_cast<const void *>(rlnc_decode_kernel<DEC_UNIT, STORE_SC1, 2>),
                          reinterpret_cast<const void *>(fill_random_words_kernel),
                          reinterpret_cast<const void *>(fill_random_bytes_kernel)};
    for (const void *f : rest) {
        hipFuncAttributes a;
        hipError_t e = hipFuncGetAttributes(&a, f);
        if (e != hipSuccess) return e;
    }
    return configure_commit_kernels();
}

#ifndef DECDS_DEC_SWEEP_MIN_N
#define DECDS_DEC_SWEEP_MIN_N 1536
#endif
#ifndef DECDS_ENC_SMALL_MAX_N
#define DECDS_ENC_SMALL_MAX_N 2
#endif
#ifndef DECDS_ENC_NT_MIN_N
#define DECDS_ENC_NT_MIN_N 256
#endif
#ifndef DECDS_DEC_NARROW_MAX_N
// the one-tile decode (and the fused plan + decode) with 8-column lane blocks up to this many chunksets
#define DECDS_DEC_NARROW_MAX_N 2
#endif
#ifndef DECDS_PLAN_DECODE_MAX_N
// decds_repair_batch: plan + decode as one launch up to this many chunksets. Every workgroup of the fused
// kernel runs its chunkset's plan first (~6 us of one wave). Against the plan kernel and the decode back
// to back on one stream (no event between them, as decds_repair_batch launches them) it saves the second
// launch: 17.6 / 20.2 against 18.2 / 21.0 us at 1 / 2 chunksets; from 4 on the redundant plans cost more
// than that (30.9 against 29.7 us at 4, 54.9 against 44.7 at 8; r09h, tools/kbench.py --repair)
#define DECDS_PLAN_DECODE_MAX_N 2
#endif
// Launch-shape thresholds (process-wide): the environment variable of the same name read once (at
// first use), else the build's default; decds_set_tuning changes one for the process (tests force
// either form of a kernel pair, tools A/B them). Every form gives identical bytes.
struct Tunable {
    const char *name;
    uint64_t build_default;
    uint64_t initial() const {
        const char *e = std::getenv(name);
        return e && *e ? (uint64_t)std::strtoull(e, nullptr, 10) : build_default;
    }
};
static const Tunable TUNABLES[] = {{"DECDS_DEC_SWEEP_MIN_N", DECDS_DEC_SWEEP_MIN_N},
                                   {"DECDS_ENC_SMALL_MAX_N", DECDS_ENC_SMALL_MAX_N},
                                   {"DECDS_ENC_NT_MIN_N", DECDS_ENC_NT_MIN_N},
                                   {"DECDS_PLAN_DECODE_MAX_N", DECDS_PLAN_DECODE_MAX_N},
                                   {"DECDS_DEC_NARROW_MAX_N", DECDS_DEC_NARROW_MAX_N}};
constexpr int TUNE_DEC_SWEEP_MIN_N = 0, TUNE_ENC_SMALL_MAX_N = 1, TUNE_ENC_NT_MIN_N = 2, TUNE_PLAN_DECODE_MAX_N = 3,
              TUNE_DEC_NARROW_MAX_N = 4, N_TUNABLES = 5;
static uint64_t tune_default(int k) {
    static const uint64_t d[N_TUNABLES] = {TUNABLES[0].initial(), TUNABLES[1].initial(), TUNABLES[2].initial(),
                                           TUNABLES[3].initial(), TUNABLES[4].initial()};
    return d[k];
}
static std::atomic<uint64_t> &tune(int k) {
    static std::atomic<uint64_t> v[N_TUNABLES] = {{tune_default(0)}, {tune_default(1)}, {tune_default(2)}, {tune_default(3)},
                                                  {tune_default(4)}};
    return v[k];
}
uint64_t set_tuning(const char *name, uint64_t value, bool set) {
    for (int k = 0; k < N_TUNABLES; k++) {
        if (std::strcmp(name, TUNABLES[k].name) != 0 && std::strcmp(name, TUNABLES[k].name + 6) != 0) continue;
        if (set) tune(k).store(value == UINT64_MAX ? tune_default(k) : value);
        return tune(k).load();
    }
    return UINT64_MAX;
}
static bool decode_sweeps(size_t n) { return n >= tune(TUNE_DEC_SWEEP_MIN_N).load(std::memory_order_relaxed); }
static bool encode_small(size_t n) { return n <= tune(TUNE_ENC_SMALL_MAX_N).load(std::memory_order_relaxed); }
static bool encode_nt(size_t n) { return n >= tune(TUNE_ENC_NT_MIN_N).load(std::memory_order_relaxed); }
static bool decode_narrow(size_t n) { return n <= tune(TUNE_DEC_NARROW_MAX_N).load(std::memory_order_relaxed); }
static bool plan_decode_fused(size_t n) {
    return n <= tune(TUNE_PLAN_DECODE_MAX_N).load(std::memory_order_relaxed) && !decode_sweeps(n);
}

// resident workgroups of a persistent kernel on this device (occupancy x CUs)
static uint32_t resident_grid(const void *fn, uint32_t lds, int fallback_per_cu, int num_cus) {
    int per_cu = 0;
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, WG, lds);
    if (e != hipSuccess || per_cu < 1) {
        hip_tolerate(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor (the kernel's own occupancy used instead)");
        per_cu = fallback_per_cu;
    }
    return (uint32_t)per_cu * (uint32_t)(num_cus > 0 ? num_cus : 256);
}

// the persistent sweeps' grids, once per context at creation (not lazily by concurrent launches)
void configure_geom(LaunchGeom &g) {
    g.enc_grid = resident_grid(reinterpret_cast<const void *>(ENC_SWEEP(false, STORE_NT)), SWEEP_LDS, DECDS_ENC_WAVES, g.num_cus);
#ifdef DECDS_SWEEP_GRID_PCT
    g.enc_grid = g.enc_grid * DECDS_SWEEP_GRID_PCT / 100;  // study builds: fewer resident workgroups than fit
#endif
    g.dec_grid = resident_grid(reinterpret_cast<const void *>(DEC_SWEEP), SWEEP_LDS, DECDS_DEC_SWEEP_WAVES, g.num_cus);
    g.enc_small_grid = resident_grid(reinterpret_cast<const void *>(ENC_SMALL), SWEEP_LDS, DECDS_ENC_SMALL_WAVES, g.num_cus);
}
static uint32_t sweep_grid(const LaunchGeom &g) { return g.enc_grid; }

hipError_t launch_encode(const LaunchGeom &geom, const uint8_t *src, size_t n, const uint8_t *coeffs, uint8_t *dst,
                         size_t pitch, uint32_t poly, uint32_t marker, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const bool small = encode_small(n);
    const uint32_t phase = small ? row_phase<2>(dst, pitch) : row_phase<DECDS_ENC_DW>(dst, pitch);
    const bool msg = !small && MSG_OK && phase == MSG_PHASE;
    const uint64_t T = small ? TILES<2> : TILES<DECDS_ENC_DW>;
    // small batches too: with fewer tiles than resident slots it is one tile each. The small form's edge
    // workgroups (EDGE_SPLIT) come on top only when every tile has its own workgroup and the whole grid
    // stays resident — taking slots from the tiles instead left a straggler round (n = 2: 1024 tiles on
    // 1022 workgroups, 2.4x the time, r06j)
    const uint32_t cap = small ? geom.enc_small_grid : sweep_grid(geom);
    const uint32_t tile_grid = (uint32_t)std::min<uint64_t>((uint64_t)n * T, cap);
    const uint32_t ne_want = small && DECDS_ENC_SMALL_EDGE ? (uint32_t)std::min<size_t>(n, EDGE_WGS) : 0u;
    const uint32_t ne = (uint64_t)n * T + ne_want <= cap ? ne_want : 0u;
    const uint32_t grid = tile_grid + ne;
    const bool nt = encode_nt(n);
    const void *fn = small ? reinterpret_cast<const void *>(ENC_SMALL)
                     : msg ? (nt ? reinterpret_cast<const void *>(ENC_SWEEP(MSG_OK, STORE_NT)) : reinterpret_cast<const void *>(ENC_SWEEP(MSG_OK, STORE_SC1)))
                           : (nt ? reinterpret_cast<const void *>(ENC_SWEEP(false, STORE_NT)) : reinterpret_cast<const void *>(ENC_SWEEP(false, STORE_SC1)));
    uint32_t *counter = nullptr;  // none when every workgroup has one tile: no counter reset to launch
    if (DECDS_ENC_QUEUE && (uint64_t)n * T > tile_grid) {
        if (!geom.counters) return hipErrorInvalidValue;
        counter = geom.counters + (geom.counter_next.fetch_add(1) % LaunchGeom::N_COUNTERS) * LaunchGeom::COUNTER_STRIDE;
    }
    void *args[] = {&src, &n, &coeffs, &dst, &pitch, const_cast<uint32_t *>(&phase), &poly, &marker, &counter};
    if (hipError_t p_ = hip_launch_begin("rlnc_encode_sweep_kernel")) return p_;
    return hipLaunchKernel(fn, dim3(grid), dim3(WG), args, SWEEP_LDS, stream);
}

// The decode's two forms: batches of DECDS_DEC_SWEEP_MIN_N chunksets or more run the
// persistent sweep, smaller ones one-tile workgroups. Round 3 measured the sweep -1.5...-3.3 % from 256
// chunksets on (r05p-r05s); on round 5's kernels the one-tile form is 1-2 % faster at 256-512 and even to
// 1280, the sweep 0.4-0.9 % faster at 1639 (r08w / r08za / r08zb), hence 1536. The environment variable of
// that name overrides the threshold per launch (tests force either form at any size).
const char *decode_kernel_name(size_t n) { return decode_sweeps(n) ? "rlnc_decode_sweep_kernel" : "rlnc_decode_kernel"; }

const char *encode_kernel_name(size_t) { return "rlnc_encode_sweep_kernel"; }

bool encode_commit_fusable(const uint8_t *dst, size_t pitch) { return row_phase<4>(dst, pitch) == MSG_PHASE; }
static_assert(MSG_PHASE < COLS<2>, "16-byte-aligned rows have the message phase for both block widths");

uint32_t encode_commit_subtrees() { return FH_WAVE_UNITS; }

hipError_t launch_encode_commit(const uint8_t *src, size_t n, const uint8_t *coeffs, uint8_t *dst, size_t pitch,
                                uint32_t poly, uint32_t marker, uint64_t first_id, const uint64_t *ids, uint32_t *sub,
                                hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (!encode_commit_fusable(dst, pitch)) return hipErrorInvalidValue;
    if (hipError_t p_ = hip_launch_begin("rlnc_encode_hash_kernel")) return p_;
    hipLaunchKernelGGL((ENC_HASH), dim3((uint32_t)(n * FH_WG_UNITS)), dim3(WG), FH_LDS<DECDS_FH_DW>, stream, src, n,
                       coeffs, dst, pitch, poly, marker, first_id, ids, sub);
    return hipGetLastError();
}

// exp table of gen under poly (the plan's log/exp tables), kept for the last (poly, gen) asked for
static const GfExpTable &exp_table(uint32_t poly, uint32_t gen) {
    static thread_local uint32_t last_poly = 0, last_gen = 0;
    static thread_local GfExpTable tab;
    if (poly != last_poly || gen != last_gen) {
        uint32_t v = 1;
        for (uint32_t i = 0; i < 256; i++) {
            if (i % 4 == 0) tab.w[i / 4] = 0;
            tab.w[i / 4] |= (i < 255 ? v : 0u) << (8 * (i % 4));
            uint32_t acc = 0, a = v;  // v *= gen
            for (int b = 0; b < 8; b++) {
                acc ^= ((gen >> b) & 1u) ? a : 0u;
                a = (a << 1) ^ ((a & 0x80u) ? (poly & 0x1FFu) : 0u);
            }
            v = acc & 0xFFu;
        }
        last_poly = poly;
        last_gen = gen;
    }
    return tab;
}

hipError_t launch_repair_plan(const uint8_t *coded, size_t pitch, size_t n, const uint8_t *cand, uint8_t *plan,
                              int8_t *verdicts, int32_t *status, uint32_t poly, uint32_t gen, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const GfExpTable &tab = exp_table(poly, gen);
    if (hipError_t p_ = hip_launch_begin("rlnc_plan_kernel")) return p_;
    hipLaunchKernelGGL(rlnc_plan_kernel, dim3((uint32_t)n), dim3(64), 0, stream, coded, pitch, n, cand,
                       reinterpret_cast<RepairPlan *>(plan), verdicts, status, tab);
    return hipGetLastError();
}

static hipError_t launch_decode_kernel(const LaunchGeom &geom, const uint8_t *coded, size_t pitch, size_t n,
                                       const uint8_t *plan, uint8_t *dst, int32_t *status, const uint64_t *in_bases,
                                       const uint64_t *out_bases, uint32_t poly, uint32_t marker, uint32_t *info,
                                       hipStream_t stream) {
    const RepairPlan *pl = reinterpret_cast<const RepairPlan *>(plan);
    if (decode_sweeps(n)) {
        const uint32_t resident = geom.dec_grid;
        const uint64_t tiles = (uint64_t)n * TILES<DECDS_DEC_DW>;
        if (tiles >= (1ull << 31)) return hipErrorInvalidValue;  // tile indices are 32-bit
        const uint32_t grid = (uint32_t)std::min<uint64_t>(tiles, resident);
        uint32_t *counter = nullptr;
        if (tiles > grid) {
            if (!geom.counters) return hipErrorInvalidValue;
            counter = geom.counters + (geom.counter_next.fetch_add(1) % LaunchGeom::N_COUNTERS) * LaunchGeom::COUNTER_STRIDE;
        }
        void *args[] = {&coded, &pitch, &n, &pl, &dst, &status, &in_bases, &out_bases, &poly, &marker, &counter, &info};
        if (hipError_t p_ = hip_launch_begin("rlnc_decode_sweep_kernel")) return p_;
        return hipLaunchKernel(reinterpret_cast<const void *>(DEC_SWEEP), dim3(grid), dim3(WG), args, SWEEP_LDS, stream);
    }
    constexpr uint32_t U = DEC_UNIT;
    if (hipError_t p_ = hip_launch_begin("rlnc_decode_kernel")) return p_;
    const bool narrow = decode_narrow(n), wt = n <= DEC_WT_MAX_N;
    const dim3 grid((uint32_t)(n * ((narrow ? TILES<2> : TILES<DECDS_DEC_DW>) / U)));
    const void *fn = narrow ? (wt ? reinterpret_cast<const void *>(rlnc_decode_kernel<U, STORE_SC1, 2>)
                                  : reinterpret_cast<const void *>(rlnc_decode_kernel<U, 0, 2>))
                            : (wt ? reinterpret_cast<const void *>(rlnc_decode_kernel<U, STORE_SC1>)
                                  : reinterpret_cast<const void *>(rlnc_decode_kernel<U>));
    void *args[] = {&coded, &pitch, &n, &pl, &dst, &status, &in_bases, &out_bases, &poly, &marker, &info};
    return hipLaunchKernel(fn, grid, dim3(WG), args, DEC_LDS, stream);
}

hipError_t launch_decode(const LaunchGeom &geom, const uint8_t *coded, size_t pitch, size_t n, const uint8_t *plan,
                         uint8_t *dst, int32_t *status, const uint64_t *in_bases, const uint64_t *out_bases,
                         uint32_t poly, uint32_t marker, uint8_t *info, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    uint32_t *inf = reinterpret_cast<uint32_t *>(info);
    // get_decoded_data's cut, the repair info and the status come from the decode kernels' edge pass
    // (tail_scan_decoded for the chunksets whose tail bytes hold no marker): one launch
    return launch_decode_kernel(geom, coded, pitch, n, plan, dst, status, in_bases, out_bases, poly, marker, inf, stream);
}

hipError_t launch_repair(const LaunchGeom &geom, const uint8_t *coded, size_t pitch, size_t n, const uint8_t *cand,
                         uint8_t *plan, int8_t *verdicts, uint8_t *dst, int32_t *status, uint32_t poly, uint32_t gen,
                         uint32_t marker, uint8_t *info, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    // the fused kernel reads each chunkset's first ten candidates as three dwords: 4-byte aligned lists only
    if (!plan_decode_fused(n) || (reinterpret_cast<uintptr_t>(cand) & 3u)) {
        if (hipError_t e = launch_repair_plan(coded, pitch, n, cand, plan, verdicts, status, poly, gen, stream)) return e;
        return launch_decode(geom, coded, pitch, n, plan, dst, status, nullptr, nullptr, poly, marker, info, stream);
    }
    const GfExpTable &tab = exp_table(poly, gen);
    RepairPlan *pl = reinterpret_cast<RepairPlan *>(plan);
    uint32_t *inf = reinterpret_cast<uint32_t *>(info);
    if (hipError_t p_ = hip_launch_begin("rlnc_plan_decode_kernel")) return p_;
    const bool narrow = decode_narrow(n), wt = n <= DEC_WT_MAX_N;
    const dim3 grid((uint32_t)(n * (narrow ? TILES<2> : TILES<DECDS_DEC_DW>)));
    const void *fn = narrow ? (wt ? reinterpret_cast<const void *>(rlnc_plan_decode_kernel<STORE_SC1, 2>)
                                  : reinterpret_cast<const void *>(rlnc_plan_decode_kernel<0, 2>))
                            : (wt ? reinterpret_cast<const void *>(rlnc_plan_decode_kernel<STORE_SC1>)
                                  : reinterpret_cast<const void *>(rlnc_plan_decode_kernel<0>));
    GfExpTable targ = tab;
    void *args[] = {&coded, &pitch, &n, &cand, &pl, &verdicts, &dst, &status, &poly, &marker, &inf, &targ};
    return hipLaunchKernel(fn, grid, dim3(WG), args, PLAN_DEC_LDS, stream);
}

const char *repair_kernel_name(size_t n) { return plan_decode_fused(n) ? "rlnc_plan_decode_kernel" : "rlnc_plan_kernel"; }

hipError_t launch_fill_random(uint64_t seed, uint64_t byte_offset, uint8_t *dst, size_t nbytes,
                              hipStream_t stream) {
    if (nbytes == 0) return hipSuccess;
    if ((byte_offset & 7u) == 0 && (reinterpret_cast<uintptr_t>(dst) & 7u) == 0 && (nbytes & 7u) == 0) {
        const size_t nw = nbytes / 8;
        const uint32_t grid = (uint32_t)((nw + 255) / 256 < 8192 ? (nw + 255) / 256 : 8192);
        if (hipError_t p_ = hip_launch_begin("fill_random_words_kernel")) return p_;
        hipLaunchKernelGGL(fill_random_words_kernel, dim3(grid), dim3(256), 0, stream, seed, byte_offset / 8,
                           reinterpret_cast<uint64_t *>(dst), nw);
    } else {
        const uint32_t grid = (uint32_t)((nbytes + 255) / 256 < 8192 ? (nbytes + 255) / 256 : 8192);
        if (hipError_t p_ = hip_launch_begin("fill_random_bytes_kernel")) return p_;
        hipLaunchKernelGGL(fill_random_bytes_kernel, dim3(grid), dim3(256), 0, stream, seed, byte_offset, dst,
                           nbytes);
    }
    return hipGetLastError();
}

}  // namespace decds

#ifdef DECDS_PHASE_TRACE
// study builds: copy out (and clear) the encode sweep's per-workgroup phase stamps
extern "C" int decds_debug_phase_trace(uint64_t *out, int clear) {
    using namespace decds;
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess && out) e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase_trace), sizeof(g_phase_trace), 0, hipMemcpyDeviceToHost);
    if (e == hipSuccess && clear) {
        static uint64_t zero[PT_WGS * PT_SLOTS];
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_phase_trace), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
    }
    return (int)e;
}
#endif

// decode_lines_r03.hip — STUDY CODE, not built: round 3's decode with line-aligned piece stores
// (rlnc_decode_lines_kernel), taken out of decds_amd/csrc/rlnc_kernels.hip after in-process A/B on four
// boxes came out mixed (-2.2 ... +2.9 %); it uses that file's helpers (combine_block with
// a sink and GSTORE = false, strow, build_tables, tbl_mul, RepairPlan). Launch:
//   rlnc_decode_lines_kernel<U><<<n * ceil(DL_TILES / U), 256, LDS_BYTES>>>(coded, pitch, n, plan, dst, status,
//                                                                      in_bases, out_bases, poly, marker)
#ifndef DECDS_DEC_WAVES
#define DECDS_DEC_WAVES 2  // waves per SIMD (3 measured no faster, r02f)
#endif
// tiles per workgroup of the line-aligned decode: 1 up to DECDS_DL_SMALL_N chunksets, DECDS_DL_UNIT
// above (r03o, one box: units of 1 / 2 / 4 at 103 chunksets 0.417 / 0.417 / 0.427 ms, at 1639 6.80 /
// 6.67 / 6.54 ms; the plain decode 0.422 / 6.78)
#ifndef DECDS_DL_UNIT
#define DECDS_DL_UNIT 4
#endif
#ifndef DECDS_DL_SMALL_N
#define DECDS_DL_SMALL_N 256
#endif
// Decode with line-aligned piece stores (round 3). Piece i of the repaired chunkset starts at i*L =
// i*2^20 + i, so the plain decode's wave stores are 1 KiB runs i bytes past line boundaries; runs that
// fill whole 128-byte lines measured 7-8 % faster as a pattern (tools/layoutbench --only declines, r03m).
// Here a wave computes 57 consecutive lane blocks — lane 0 the block before its run, lanes 57..63
// idle — and lanes 1..56 each store the ALIGNED 16-byte granule g of every piece: bytes [16 - i, 32 - i)
// of (previous lane's block || own block), the previous lane's bytes moved over by a DPP wave shift
// (v_mov_b32_dpp wave_shr:1) and joined with v_alignbyte. A wave stores 56 granules = 7 whole lines per
// piece; a workgroup 224 blocks (DL_TILES = 293 workgroups per chunkset). Granule 0 of piece i > 0 also
// covers piece i-1's last i columns (edge columns, zeros here): the chunkset's first workgroup writes
// the edge columns only after its own stores (barrier). The last block's last i columns fall in no
// granule: the edge pass covers columns [16 * BLOCKS - 9, L) (the lanes of the last workgroup write
// some of the same bytes with the same values).
constexpr uint32_t DL_RUN = 56;                                          // granules per wave: 7 lines
constexpr uint32_t DL_TILE = (WG / 64) * DL_RUN;                         // 224 blocks per workgroup
constexpr uint32_t DL_TILES = (BLOCKS<4> + DL_TILE - 1) / DL_TILE;       // 293 per chunkset
constexpr uint32_t DL_EDGE0 = BLOCKS<4> * COLS<4> - (K - 1);             // first edge column
constexpr uint32_t DL_EDGE = (uint32_t)L - DL_EDGE0;                     // 26 edge columns
static_assert(DL_TILE % 8 == 0 && DL_RUN % 8 == 0, "wave runs start on 128-byte lines");

// piece I's aligned granule from this lane's 16 columns (cur) and the previous lane's (DPP)
__device__ __forceinline__ u32x4 realign(int I, const u32x4 &cur) {
    if (I == 0) return cur;
    const int q = (16 - I) / 4, b = (16 - I) % 4;
    uint32_t z[8];
#pragma unroll
    for (int w = 0; w < 4; w++) z[4 + w] = cur[w];
#pragma unroll
    for (int w = 0; w < 4; w++)
        if (w >= q) z[w] = __builtin_amdgcn_update_dpp(0u, cur[w], 0x138 /* wave_shr:1 */, 0xf, 0xf, false);
    u32x4 r;
#pragma unroll
    for (int w = 0; w < 4; w++) r[w] = b == 0 ? z[q + w] : __builtin_amdgcn_alignbyte(z[q + w + 1], z[q + w], b);
    return r;
}

template <uint32_t UNIT>
__global__ __launch_bounds__(WG, DECDS_DEC_WAVES) __attribute__((amdgpu_waves_per_eu(DECDS_DEC_WAVES, DECDS_DEC_WAVES)))
void rlnc_decode_lines_kernel(const uint8_t *__restrict__ coded, size_t pitch, size_t n,
                              const RepairPlan *__restrict__ plan, uint8_t *__restrict__ dst,
                              int32_t *__restrict__ status, const uint64_t *__restrict__ in_bases,
                              const uint64_t *__restrict__ out_bases, uint32_t poly, uint32_t marker) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int DW = 4;
    constexpr uint32_t UPC = (DL_TILES + UNIT - 1) / UNIT;  // units per chunkset
    const uint32_t cs = blockIdx.x / UPC, t0 = (blockIdx.x % UPC) * UNIT;
    const uint32_t te = t0 + UNIT < DL_TILES ? t0 + UNIT : DL_TILES;
    if (cs >= n) return;
    const uint32_t *pw = reinterpret_cast<const uint32_t *>(plan + cs);
    const uint32_t w0 = __builtin_amdgcn_readfirstlane(pw[0]);
    const uint32_t w1 = __builtin_amdgcn_readfirstlane(pw[1]);
    const uint32_t w2 = __builtin_amdgcn_readfirstlane(pw[2]);
    if (((w2 >> 16) & 0xFFu) != K) return;  // RepairPlan::rank at byte 10: not ready
    const uint32_t cw = table_coeffs<K, K>(plan[cs].inv, K);
    const uint32_t sel[K] = {w0 & 0xFFu, (w0 >> 8) & 0xFFu, (w0 >> 16) & 0xFFu, w0 >> 24,
                             w1 & 0xFFu, (w1 >> 8) & 0xFFu, (w1 >> 16) & 0xFFu, w1 >> 24,
                             w2 & 0xFFu, (w2 >> 8) & 0xFFu};
    uint32_t ioff[K], ooff[K];
#pragma unroll
    for (int k = 0; k < (int)K; k++) ioff[k] = (uint32_t)(sel[k] * pitch + K);
#pragma unroll
    for (int i = 0; i < (int)K; i++) ooff[i] = (uint32_t)(i * L);
    const uint8_t *ibase;
    uint8_t *obase;
    if (in_bases) {
        ibase = reinterpret_cast<const uint8_t *>(uniform_u64(in_bases[cs]));
        obase = reinterpret_cast<uint8_t *>(uniform_u64(out_bases[cs]));
    } else {
        ibase = coded + (size_t)cs * N * pitch;
        obase = dst + (size_t)cs * CS;
    }
    const uint32_t l = threadIdx.x & 63u;
    // this lane's block of tile t (lanes 1..56 also store its aligned granule), or out of range
    auto blk = [&](uint32_t t) { return t * DL_TILE + (threadIdx.x >> 6) * DL_RUN + l - 1; };  // wraps for lane 0 of tile 0
    auto col = [&](uint32_t t) {
        const uint32_t g = blk(t);
        return t < te && l <= DL_RUN && g < BLOCKS<DW> ? g * COLS<DW> : OOB_COL;
    };
    Vec<DW> x[K];
    load_block<K, DW>(x, ibase, ioff, col(t0));
    build_tables<K, K>(lds, cw, poly);
    lds_barrier();
    uint32_t gcol = 0;
    auto sink = [&](int i, const Vec<DW> &v) { strow<DW>(obase, ((uint32_t)i << 20) + gcol, realign(i, v)); };
    asm volatile("" ::: "memory");  // the loop's memory-counter picture: inputs, then 10 dropped stores
#pragma unroll
    for (int i = 0; i < (int)K; i++) strow<DW>(obase, OOB_COL + ooff[i], Vec<DW>{});
    uint32_t t = t0;
#pragma unroll 1
    do {
        const uint32_t c = col(t);
        gcol = l >= 1 ? c : OOB_COL;  // aligned granule of each piece
        combine_block<K, K, DW, 0, decltype(sink), 0, false>(x, obase, ooff, c, ibase, ioff, col(t + 1), sink);
    } while (++t < te);
    if (t0 == 0) {  // the edge columns, after this workgroup's own stores (granule 0 overlaps them)
        __syncthreads();
        // piece 9's must decode to marker || zeros (rlnc get_decoded_data strips them; a mismatch is a
        // repairing failure, chunkset.rs:202-204)
        bool ok = true;
        for (uint32_t idx = threadIdx.x; idx < DL_EDGE * K; idx += WG) {
            const uint32_t i = idx % K, c = DL_EDGE0 + idx / K;
            uint32_t z = 0;
#pragma unroll
            for (uint32_t k = 0; k < K; k++) z ^= tbl_mul(lds, k, i, ibase[ioff[k] + c]);
            const uint64_t p = (uint64_t)i * L + c;
            if (p < CS)
                obase[p] = (uint8_t)z;
            else
                ok &= z == (p == CS ? marker : 0u);
        }
        if (__any(!ok) && (threadIdx.x & 63u) == 0) status[cs] = 6;  // DECDS_ERR_CHUNKSET_REPAIRING_FAILED
    }
}


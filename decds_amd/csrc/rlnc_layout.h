// rlnc_layout.h — constants and device-side data layout shared by the kernels, the C-ABI and the
// host mirror. Every constant cites the reference line it reproduces.
#pragma once
#include <stdint.h>

namespace decds {

constexpr uint32_t K = 10;                   // ChunkSet::NUM_ORIGINAL_CHUNKS (chunkset.rs:19)
constexpr uint32_t N = 16;                   // NUM_ERASURE_CODED_CHUNKS = DECDS_NUM_ERASURE_CODED_SHARES
                                             // (chunkset.rs:21, consts.rs:5)
constexpr uint64_t CS = 10ull * (1ull << 20);  // ChunkSet::BYTE_LENGTH (chunkset.rs:20, chunk.rs:14)
constexpr uint64_t L = (CS + 1 + K - 1) / K;   // PADDED_CHUNK_BYTE_LEN (chunkset.rs:117) = 1,048,577
constexpr uint64_t F = L + K;                  // full coded piece: coding vector || payload
constexpr uint32_t PROOF_SIZE = 4;           // ChunkSet::PROOF_SIZE = log2(16) chunkset-level proof hashes (chunkset.rs:22)
static_assert(L == 1048577ull, "piece length pinned by chunkset.rs:117");

constexpr uint32_t POLY_DEFAULT = 0x11D;     // rlnc 0.4.0 GF(2^8) polynomial [recalled, run-time parameter]
constexpr uint32_t MARKER_DEFAULT = 0x81;    // rlnc 0.4.0 boundary marker [recalled, run-time parameter]

// Column tiling of one L-byte piece for the streaming kernels: each lane owns 16 consecutive
// columns (one 16-byte vector per piece); columns [0, MAIN_COLS) go through the vector loop,
// the last TAIL_COLS columns (which hold piece 9's boundary marker) through a byte-wise path.
constexpr uint32_t COLS_PER_LANE = 16;
constexpr uint32_t MAIN_BLOCKS = 65535;                    // 16-column lane blocks in the main loop
constexpr uint32_t MAIN_COLS = MAIN_BLOCKS * COLS_PER_LANE;  // 1,048,560
constexpr uint32_t TAIL_COLS = (uint32_t)L - MAIN_COLS;     // 17
static_assert(MAIN_COLS + TAIL_COLS == L, "tiling covers the piece");
static_assert((K - 1) * L + MAIN_COLS <= CS, "main loop never reads piece 9's marker/padding");

// Decode plan, one per chunkset (written by the plan kernel, read by the decode kernel).
struct alignas(16) RepairPlan {
    uint8_t sel[K];      // coded-row index (0..15) of the k-th accepted chunk, acceptance order
    uint8_t rank;        // decoder rank after all candidates (== K -> ready to repair)
    uint8_t pad0[5];
    uint8_t inv[K * K];  // inverse of the accepted coding vectors, input-major: piece_i = sum_k inv[k * K + i] * y_k
    uint8_t pad1[12];
};
static_assert(sizeof(RepairPlan) == 128, "plan is 128 B");

}  // namespace decds

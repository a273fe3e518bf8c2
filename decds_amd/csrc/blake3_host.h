// blake3_host.h — host BLAKE3 with 8 chunks (or parents) per AVX2 compression (blake3_host.cpp)
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <functional>

namespace decds {
namespace b3h {
constexpr size_t MAX_SIMD_SUBTREE = 1024;  // chunks per simd_subtree call (32 KiB of chaining values)
bool simd_available();                      // AVX2 on this CPU
// chaining value (not finalised) of the complete subtree of nchunks full chunks at p, chunk counter
// `first`; nchunks a power of two in [8, MAX_SIMD_SUBTREE]; requires simd_available()
void simd_subtree(const uint8_t *p, size_t nchunks, uint64_t first, uint32_t cv[8]);
}  // namespace b3h
// Chunk::digest of a full 1,048,587-byte coded piece on the host pool, side(0 .. side_tasks - 1) (if
// any) beside it (commit.cpp); requires b3h::simd_available()
void full_piece_digest(uint64_t chunkset_id, uint64_t chunk_id, const uint8_t *data, uint8_t out[32],
                       const std::function<void(size_t)> *side, size_t side_tasks);
// chaining value (not finalised) of the BLAKE3 subtree of [p, p + len) from chunk `first` (commit.cpp)
void blake3_subtree_cv(const uint8_t *p, size_t len, uint64_t first, uint32_t cv[8], int threads);
// blake3::hash of a message from the chaining values of its n >= 2 consecutive aligned 2^k-chunk subtrees
// (the last possibly smaller): the left-balanced tree over them with ROOT at the top (commit.cpp)
void blake3_fold_root(const uint32_t (*cvs)[8], size_t n, uint8_t out[32]);
}  // namespace decds

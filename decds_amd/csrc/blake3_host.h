// blake3_host.h — host BLAKE3 with 8 chunks (or parents) per AVX2 compression (blake3_host.cpp)
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace decds {
namespace b3h {
constexpr size_t MAX_SIMD_SUBTREE = 1024;  // chunks per simd_subtree call (32 KiB of chaining values)
bool simd_available();                      // AVX2 on this CPU
// chaining value (not finalised) of the complete subtree of nchunks full chunks at p, chunk counter
// `first`; nchunks a power of two in [8, MAX_SIMD_SUBTREE]; requires simd_available()
void simd_subtree(const uint8_t *p, size_t nchunks, uint64_t first, uint32_t cv[8]);
}  // namespace b3h
}  // namespace decds

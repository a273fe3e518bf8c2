// commit_kernels.h — launcher of the commitment kernels (commit_kernels.hip)
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace decds {
hipError_t launch_commit(const uint8_t *coded, size_t pitch, size_t n, uint64_t first_chunkset_id, uint8_t *digests,
                         uint8_t *roots, uint8_t *proofs, hipStream_t stream);
}

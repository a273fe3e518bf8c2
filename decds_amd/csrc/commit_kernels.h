// commit_kernels.h — launcher of the commitment kernels (commit_kernels.hip)
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace decds {
hipError_t configure_commit_kernels();  // resolve the commitment kernels eagerly (configure_kernels)
hipError_t launch_commit(const uint8_t *coded, size_t pitch, size_t n, uint64_t first_chunkset_id, uint8_t *digests,
                         uint8_t *roots, uint8_t *proofs, hipStream_t stream);
// digests of rows encoded by launch_encode_commit (sub: its subtree values), then the Merkle trees
hipError_t launch_commit_fold(const uint8_t *coded, size_t pitch, size_t n, const uint32_t *sub, uint32_t per_row,
                              uint8_t *digests, uint8_t *roots, uint8_t *proofs, hipStream_t stream);
// Blob::new's whole-blob digest, device part: the 1024-chunk subtree value of each of n_groups full
// 1 MiB groups at data (chunk counters from first_chunk) into cvs (32 B per group)
hipError_t launch_blob_groups(const uint8_t *data, size_t n_groups, uint64_t first_chunk, uint8_t *cvs,
                              hipStream_t stream);
hipError_t launch_validate(const uint8_t *coded, size_t pitch, size_t n_rows, const uint64_t *ids,
                           const uint8_t *proofs, size_t proof_len, const uint8_t *chunkset_roots,
                           size_t num_chunksets, const uint8_t *blob_root, uint8_t *digests, uint8_t *valid,
                           hipStream_t stream);
}

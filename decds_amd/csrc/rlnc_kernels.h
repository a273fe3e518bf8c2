// rlnc_kernels.h — host-side launchers for the gfx950 RLNC kernels (rlnc_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <atomic>

namespace decds {

struct LaunchGeom {
    int num_cus;  // CUs on the device (256 on MI355X)
    // tile counters of the queue-fed encode sweep: one 128-byte line each (tile counter, exit count),
    // zeroed at context creation; a launch takes the next one round robin (concurrent launches on
    // other streams never share one) and its last workgroup zeroes it again
    uint32_t *counters = nullptr;
    mutable std::atomic<uint32_t> counter_next{0};
    static constexpr uint32_t N_COUNTERS = 256, COUNTER_STRIDE = 32;  // in uint32_t
    // resident workgroups of the persistent encode / decode sweeps (configure_geom, at context creation)
    uint32_t enc_grid = 0, enc_small_grid = 0, dec_grid = 0;
};
void configure_geom(LaunchGeom &g);
// launch-shape thresholds by name (DECDS_DEC_SWEEP_MIN_N, DECDS_ENC_SMALL_MAX_N, DECDS_ENC_NT_MIN_N,
// DECDS_PLAN_DECODE_MAX_N, with or without the
// DECDS_ prefix): set (set = true; UINT64_MAX = the default again) and/or read; UINT64_MAX if unknown
uint64_t set_tuning(const char *name, uint64_t value, bool set);

hipError_t launch_encode(const LaunchGeom &g, const uint8_t *src, size_t n, const uint8_t *coeffs,
                         uint8_t *dst, size_t pitch, uint32_t poly, uint32_t marker,
                         hipStream_t stream);
// ChunkSet::new's encode with the commitment's chunk hashing fused (rows at a 16-byte-aligned pitch
// and base only: encode_commit_fusable). sub: n x 16 x encode_commit_subtrees() x 32 B of aligned
// subtree values (256 of 4 chunks per row, or 64 of 16 with the unit-hash form), completed into
// digests / roots / proofs by launch_commit_fold.
bool encode_commit_fusable(const uint8_t *dst, size_t pitch);
uint32_t encode_commit_subtrees();
hipError_t launch_encode_commit(const uint8_t *src, size_t n, const uint8_t *coeffs, uint8_t *dst, size_t pitch,
                                uint32_t poly, uint32_t marker, uint64_t first_id, const uint64_t *ids, uint32_t *sub,
                                hipStream_t stream);
hipError_t launch_repair_plan(const uint8_t *coded, size_t pitch, size_t n, const uint8_t *cand,
                              uint8_t *plan, int8_t *verdicts, int32_t *status, uint32_t poly,
                              uint32_t gen, hipStream_t stream);
// in_bases / out_bases (device arrays of n addresses, or NULL): the gather form — chunkset c's
// accepted rows at in_bases[c] + plan.sel[k]*pitch, its output at out_bases[c]. info (n x 16 B,
// decds_repair_info, or NULL): get_decoded_data's length and the 10 decoded tail bytes of every
// chunkset that decodes (the decode kernels' edge pass finds the cut, tail_scan_decoded when no tail
// byte is the marker).
hipError_t launch_decode(const LaunchGeom &g, const uint8_t *coded, size_t pitch, size_t n,
                         const uint8_t *plan, uint8_t *dst, int32_t *status, const uint64_t *in_bases,
                         const uint64_t *out_bases, uint32_t poly, uint32_t marker, uint8_t *info,
                         hipStream_t stream);
// RepairingChunkSet's rank step + repair for n chunksets (decds_repair_batch): the plan kernel then
// the decode, or — up to DECDS_PLAN_DECODE_MAX_N chunksets (one-tile decode form) — both as one launch
// (rlnc_plan_decode_kernel), with the same outputs
hipError_t launch_repair(const LaunchGeom &g, const uint8_t *coded, size_t pitch, size_t n, const uint8_t *cand,
                         uint8_t *plan, int8_t *verdicts, uint8_t *dst, int32_t *status, uint32_t poly, uint32_t gen,
                         uint32_t marker, uint8_t *info, hipStream_t stream);
const char *repair_kernel_name(size_t n);  // the first kernel launch_repair runs for n chunksets
hipError_t launch_fill_random(uint64_t seed, uint64_t byte_offset, uint8_t *dst, size_t nbytes,
                              hipStream_t stream);
const char *encode_kernel_name(size_t n);  // the kernel launch_encode runs for n chunksets
const char *decode_kernel_name(size_t n);  // ... launch_decode
hipError_t configure_kernels();  // raise the dynamic-LDS limit once per process

}  // namespace decds

// capi_internal.h — state shared by the C-ABI translation units (not part of the public ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <condition_variable>
#include <mutex>
#include <vector>

#include "hip_status.h"
#include "host_mem.h"
#include "rlnc_kernels.h"

namespace decds {
struct Lane;       // chunkset.cpp: the buffers and stream of one in-flight chunkset-mirror call
struct Coalescer;  // chunkset.cpp: concurrent ChunkSet::new calls gathered into shared launches
struct Pipe;       // blob.cpp: the host paths' H2D / kernel / D2H streams and slot events
void pipe_destroy(Pipe *p);
}

struct decds_ctx {
    int device;
    uint32_t poly;     // GF(2^8) polynomial incl. x^8 (rlnc 0.4.0: 0x11D [recalled])
    uint8_t marker;    // boundary marker appended by rlnc Encoder::new (0x81 [recalled])
    uint32_t gen;      // smallest generator of GF(2^8)* under poly (the plan kernel's log/exp tables)
    decds::LaunchGeom geom;
    // host blob paths (decds_blob_*_host, Blob, RepairingBlob): device slot buffers kept across
    // calls (grow-only) and the pinned bounce rings for caller memory that is not page-locked;
    // host_mu serialises those calls on one context
    std::mutex host_mu;
    uint8_t *host_scratch = nullptr;
    size_t host_scratch_cap = 0;
    uint8_t *host_small = nullptr;  // page-locked, grow-only: plans, statuses, commitment outputs of a call
    size_t host_small_cap = 0;
    decds::BounceRing in_ring, out_ring;
    decds::Pipe *pipe = nullptr;  // created by the first host-path call, kept for the context's life
    // chunkset mirror (decds_chunkset_new, decds_repairing_chunkset_repair): a pool of lanes, one
    // per concurrent caller (the reference calls ChunkSet::new from rayon workers, blob.rs:256-264)
    std::mutex lane_mu;
    std::condition_variable lane_cv;
    std::vector<decds::Lane *> lanes_all, lanes_free;
    decds::Coalescer *coalescer = nullptr;  // created by the first decds_chunkset_new (under lane_mu)
};

// at least `bytes` of the context's host-path scratch (caller holds ctx->host_mu)
hipError_t decds_ctx_scratch(decds_ctx *ctx, size_t bytes, uint8_t **out);
// at least `bytes` of the context's small page-locked host area (caller holds ctx->host_mu)
hipError_t decds_ctx_host_small(decds_ctx *ctx, size_t bytes, uint8_t **out);
void decds_lanes_destroy(decds_ctx *ctx);  // chunkset.cpp

int decds_set_error(int code, const char *fmt, ...);
int decds_hip_error(hipError_t e, const char *what);
int decds_ctx_bind(const decds_ctx *ctx);  // hipSetDevice(ctx->device)
// decds_encode_commit_batch with per-chunkset ids (commit.cpp)
int encode_commit_ids(decds_ctx *ctx, const uint8_t *src, size_t n, const uint8_t *coeffs, uint8_t *dst, size_t pitch,
                      uint64_t first_chunkset_id, const uint64_t *ids, uint8_t *digests, uint8_t *roots, uint8_t *proofs,
                      void *workspace, void *stream);

namespace decds {
// host-side GF(2^8) helpers for the 10-byte coding vectors (control path, not the hot path)
uint8_t host_gf_mul(uint8_t a, uint8_t b, uint32_t poly);
uint8_t host_gf_inv(uint8_t a, uint32_t poly);
// smallest element of multiplicative order 255, or 0 when poly is reducible (no field)
uint32_t host_gf_generator(uint32_t poly);
// inverse of a 10x10 matrix over GF(2^8) (row-major); false if singular
bool host_gf_invert(const uint8_t *m, uint8_t *inv, uint32_t poly);
}  // namespace decds

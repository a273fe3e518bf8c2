// host_mem.h — host memory the DMA engines read and write (internal, not part of the public ABI).
//
// The library never page-locks caller memory behind the caller's back. A host buffer is DMA'd
// directly only if it lies inside a range this library knows to be page-locked — one the caller
// locked with decds_host_register or allocated with decds_host_alloc (a refcounted process-wide
// registry). Any other host buffer goes through a ring of the context's own page-locked staging
// pieces (bounce copies, parallel memcpy on a small host thread pool). Round 1 locked and unlocked
// every caller buffer per call (hipHostRegister on arbitrary sub-page ranges of the Python heap,
// failures swallowed): the suspected cause of the illegal-address fault in GPUTEST_r01.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <functional>

// Page-locked memory of the library (rings, lane staging, statuses, plans): non-coherent
// (coarse-grained) hipHostMalloc memory.
#ifndef DECDS_HOST_MALLOC_FLAGS
#define DECDS_HOST_MALLOC_FLAGS hipHostMallocNonCoherent
#endif

namespace decds {

// Large page-locked buffers (staging rings, lane staging, decds_host_alloc). Huge-page anonymous
// memory + hipHostRegister was measured against hipHostMalloc here and moved data at the same rate
// (blob host paths 28.7 / 35 GiB/s either way, r02zd-ze), so these stay hipHostMalloc memory.
hipError_t host_pinned_alloc(size_t n, void **out);
void host_pinned_free(void *p, size_t n);  // blocks >= 64 MiB are cached for reuse (host_mem.cpp)
size_t host_cache_trim();                   // frees the cached blocks; returns their bytes

// A use of [p, p+n) by one call: pinned() is true iff the whole range lies in one registered
// range, which then stays locked until the use ends (an unregister meanwhile is deferred).
class HostUse {
   public:
    HostUse(const void *p, size_t n);
    ~HostUse();
    HostUse(const HostUse &) = delete;
    HostUse &operator=(const HostUse &) = delete;
    bool pinned() const { return key_ != 0; }

   private:
    uintptr_t key_ = 0;
};

// parallel_for over [0, n) on the library's host pool (the caller's thread takes part)
void host_parallel(size_t n, const std::function<void(size_t)> &fn);
// memcpy split over the host pool above a few MiB
void par_memcpy(void *dst, const void *src, size_t n);

// Ring of page-locked staging pieces for one direction of one stream.
//   h2d: each piece is filled by the host, then copied to the device on `s`; a piece is refilled
//        only once its previous copy has completed (the host is paced by the DMA).
//   d2h: each piece is copied from the device on `s`; its copy-out into the caller's buffer is
//        deferred until the piece is needed again or flush() runs.
struct BounceRing {
    static constexpr int R = 4;
    static constexpr size_t PIECE = (size_t)8 << 20;
    uint8_t *buf[R] = {};
    hipEvent_t ev[R] = {};
    bool used[R] = {};
    uint8_t *pend_dst[R] = {};
    size_t pend_len[R] = {};
    int next = 0;

    hipError_t init();  // lazily; idempotent
    hipError_t h2d(uint8_t *ddst, const uint8_t *hsrc, size_t n, hipStream_t s);
    hipError_t d2h(uint8_t *hdst, const uint8_t *dsrc, size_t n, hipStream_t s);
    hipError_t flush();
    void abandon();  // after a failed call: wait for the pieces' copies, drop pending copy-outs
    // after the streams this call's copies were queued on have been drained, before they are destroyed:
    // every piece is free. (A piece left "used" had its event waited for by the NEXT call, after the
    // stream the event was recorded on had been destroyed; that wait failed now and then with
    // hipErrorCapturedEvent (907), r09f.) Pending copy-outs must have been flushed.
    void retire();
    // h2d in two steps, so the host fill of a piece can overlap other host work: stage() settles the
    // next piece and returns it (*idx), commit() queues its copy to the device; an uncommitted piece is
    // simply reused later
    hipError_t stage(int *idx, uint8_t **piece);
    hipError_t commit(int idx, uint8_t *ddst, size_t n, hipStream_t s);
    ~BounceRing();

   private:
    hipError_t settle(int i);  // wait for piece i's last copy; complete its deferred copy-out
};

// Copy between a device buffer and a caller host buffer: a direct async DMA when the host range
// is registered, else through `ring` (which must then be flushed before the host data is read).
hipError_t copy_h2d(uint8_t *d, const uint8_t *h, size_t n, bool pinned, BounceRing &ring, hipStream_t s);
hipError_t copy_d2h(uint8_t *h, const uint8_t *d, size_t n, bool pinned, BounceRing &ring, hipStream_t s);
// hipMemcpyAsync device -> page-locked host in pieces (host_mem.cpp: large single copies run at half rate)
hipError_t d2h_pieces(uint8_t *h, const uint8_t *d, size_t n, hipStream_t s);

}  // namespace decds

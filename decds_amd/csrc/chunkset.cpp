// chunkset.cpp — host-side mirror of decds-lib's chunkset API (chunkset.rs) over the gfx950 batch
// kernels. Same names, argument meaning and error behaviour as the reference, including
// ChunkSet::new's commitment (digests, Merkle root, proofs: computed on the device by the commit
// kernels) and RepairingChunkSet::add_chunk's proof check.
//
//   decds_chunkset_new                 ChunkSet::new                    chunkset.rs:37-69
//   decds_chunkset_get_chunk           ChunkSet::get_chunk              chunkset.rs:87-89
//   decds_repairing_chunkset_*         RepairingChunkSet                chunkset.rs:107-208
//
// The reference calls ChunkSet::new from rayon workers (blob.rs:256-264), so concurrent callers
// are the normal case: each call takes a lane from the context's pool — its own stream, device
// buffers and page-locked staging, all kept across calls — so callers neither allocate per call
// nor serialise on the null stream. Caller memory is copied through the lane's staging buffer
// (the library never page-locks it).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <new>
#include <vector>

#include "../../include/decds_rlnc.h"
#include "capi_internal.h"
#include "commit_kernels.h"
#include "rlnc_layout.h"

using namespace decds;

namespace decds {

// Device and pinned buffers of one in-flight chunkset-mirror call. Small-area offsets (device and
// host mirror alike):
constexpr size_t SM_CV = 0, SM_CAND = 256, SM_STATUS = 288, SM_VERD = 320, SM_PLAN = 384, SM_ROOT = 512,
                 SM_INFO = 768, SM_DIG = 1024, SM_PRF = 2048, SM_BYTES = 4096;
static_assert(SM_PRF + N * PROOF_SIZE * 32 <= SM_BYTES && SM_DIG + N * 32 <= SM_PRF, "lane small-area layout");

struct Lane {
    hipStream_t s = nullptr;
    uint8_t *d_cs = nullptr;     // CS: the chunkset (encode input / repaired output)
    uint8_t *d_coded = nullptr;  // N*F coded rows (encode output / repair input in rows 0..9)
    uint8_t *d_small = nullptr;  // SM_BYTES
    uint8_t *h_big = nullptr;    // N*F page-locked staging (>= CS, >= K*F)
    uint8_t *h_small = nullptr;  // SM_BYTES page-locked
    ~Lane() {
        if (s) hip_tolerate(hipStreamSynchronize(s), "hipStreamSynchronize");
        for (uint8_t *p : {d_cs, d_coded, d_small})
            if (p) hip_tolerate(hipFree(p), "hipFree");
        host_pinned_free(h_big, N * F);
        if (h_small) hip_tolerate(hipHostFree(h_small), "hipHostFree");
        if (s) hip_tolerate(hipStreamDestroy(s), "hipStreamDestroy");
    }
    hipError_t init() {
        hipError_t e;
        if ((e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) || (e = hipMalloc(reinterpret_cast<void **>(&d_cs), CS)) ||
            (e = hipMalloc(reinterpret_cast<void **>(&d_coded), N * F)) ||
            (e = hipMalloc(reinterpret_cast<void **>(&d_small), SM_BYTES)) ||
            (e = host_pinned_alloc(N * F, reinterpret_cast<void **>(&h_big))) ||
            (e = hipHostMalloc(reinterpret_cast<void **>(&h_small), SM_BYTES, DECDS_HOST_MALLOC_FLAGS)))
            return e;
        return hipSuccess;
    }
};
static_assert(N * F >= CS && N * F >= K * F, "lane staging holds every transfer");

namespace {

size_t max_lanes() {
    static const size_t m = [] {
        // 8 lanes: 16 concurrent lanes ran slower than 8 (19.0 against 25.0 GiB/s of ChunkSet::new at 16
        // callers, r05d) — further callers wait for a free lane instead
        const char *e = std::getenv("DECDS_MAX_LANES");
        const int v = e ? std::atoi(e) : 8;
        return (size_t)std::max(1, v);
    }();
    return m;
}

// a free lane of ctx (created on demand up to max_lanes, else wait for one); caller is bound
int lane_acquire(decds_ctx *ctx, Lane **out) {
    std::unique_lock<std::mutex> g(ctx->lane_mu);
    for (;;) {
        if (!ctx->lanes_free.empty()) {
            *out = ctx->lanes_free.back();
            ctx->lanes_free.pop_back();
            return DECDS_OK;
        }
        if (ctx->lanes_all.size() < max_lanes()) break;
        ctx->lane_cv.wait(g);
    }
    ctx->lanes_all.push_back(nullptr);  // reserve the slot while allocating outside the lock
    g.unlock();
    Lane *l = new Lane;
    hipError_t e = l->init();
    g.lock();
    auto it = std::find(ctx->lanes_all.begin(), ctx->lanes_all.end(), nullptr);
    if (e != hipSuccess) {
        ctx->lanes_all.erase(it);
        g.unlock();
        delete l;
        ctx->lane_cv.notify_one();
        return decds_hip_error(e, "lane setup (stream, device buffers, pinned staging)");
    }
    *it = l;
    *out = l;
    return DECDS_OK;
}

void lane_release(decds_ctx *ctx, Lane *l) {
    {
        std::lock_guard<std::mutex> g(ctx->lane_mu);
        ctx->lanes_free.push_back(l);
    }
    ctx->lane_cv.notify_one();
}

struct LaneGuard {
    decds_ctx *ctx;
    Lane *l = nullptr;
    ~LaneGuard() {
        if (l) lane_release(ctx, l);
    }
};

std::mutex g_rng_mu;
std::mt19937_64 &rng() {
    // the reference draws coding vectors from rand::rng() (chunkset.rs:42): OS-seeded, not
    // reproducible; the same holds here when the caller passes coeffs == NULL
    static std::mt19937_64 g{std::random_device{}()};
    return g;
}

}  // namespace

// ---- coalesced ChunkSet::new ---------------------------------------------------------------------
// The reference calls ChunkSet::new from rayon workers (blob.rs:256-264): one chunkset per call, many
// calls at once. Each call copies its chunkset into a page-locked block of its own and queues a
// request; whichever caller finds one of the context's two batch slots free takes every queued
// request (up to CO_MAX) and runs them as ONE batch on that slot's stream — H2D of every chunkset,
// one fused encode + chunk-hashing launch (rlnc_encode_hash_kernel, per-request chunkset ids) + fold
// + Merkle, D2H of each request's rows and proofs into its own page-locked block — then wakes the
// callers, who copy their rows out. Two slots: one batch's D2H overlaps the next batch's H2D.
// A lone caller runs a batch of one. Opt-in (DECDS_CHUNKSET_COALESCE=1, read per call): measured
// against per-call lanes capped at 8 it lost at every caller count (1 / 4 / 8 / 16 callers: 6.4 /
// 18.3 / 21.9 / 23.7 GiB/s against 10.5 / 23.1 / 25.0 / 25.0, r05d): the per-call H2D + kernels +
// D2H already keep the link busy from 4 callers on, and a batch adds its slowest member's latency.
constexpr size_t CO_MAX = 16;
constexpr size_t CO_P = DECDS_CODED_PITCH_ALIGNED;  // rows 16 bytes past a 128-byte boundary: the fused form

struct PinnedPool {  // page-locked blocks of one size, kept for reuse
    size_t bytes, keep;
    std::mutex mu;
    std::vector<uint8_t *> free;
    hipError_t get(uint8_t **out) {
        {
            std::lock_guard<std::mutex> g(mu);
            if (!free.empty()) {
                *out = free.back();
                free.pop_back();
                return hipSuccess;
            }
        }
        return host_pinned_alloc(bytes, reinterpret_cast<void **>(out));
    }
    void put(uint8_t *p) {
        if (!p) return;
        {
            std::lock_guard<std::mutex> g(mu);
            if (free.size() < keep) {
                free.push_back(p);
                return;
            }
        }
        host_pinned_free(p, bytes);
    }
    void clear() {
        std::lock_guard<std::mutex> g(mu);
        for (uint8_t *p : free) host_pinned_free(p, bytes);
        free.clear();
    }
};

struct EncReq {
    size_t id;
    uint8_t cv[N * K];
    uint8_t *in = nullptr;   // page-locked copy of the chunkset (CS)
    uint8_t *out = nullptr;  // page-locked: 16 x F rows, then root (32) and proofs (16 x 4 x 32)
    int status = DECDS_OK;
    std::string err;
    bool done = false;
};
constexpr size_t CO_OUT = N * F + 32 + N * PROOF_SIZE * 32;

struct CoSlot {
    hipStream_t s = nullptr;
    uint8_t *d_src = nullptr, *d_rows = nullptr, *d_packed = nullptr, *d_small = nullptr, *d_ws = nullptr,
            *h_small = nullptr;
    uint8_t *rows = nullptr;  // message-aligned: row 0 16 bytes past a 128-byte boundary
    bool busy = false;
    // d_small / h_small: cv (CO_MAX x 160) | ids (CO_MAX x 8) | digests | roots | proofs
    static constexpr size_t O_CV = 0, O_IDS = CO_MAX * N * K, O_DIG = O_IDS + CO_MAX * 8, O_ROOT = O_DIG + CO_MAX * N * 32,
                            O_PRF = O_ROOT + CO_MAX * 32, BYTES = O_PRF + CO_MAX * N * PROOF_SIZE * 32;
    hipError_t init() {
        hipError_t e;
        if ((e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) ||
            (e = hipMalloc(reinterpret_cast<void **>(&d_src), CO_MAX * CS)) ||
            (e = hipMalloc(reinterpret_cast<void **>(&d_rows), CO_MAX * N * CO_P + 256)) ||
            (e = hipMalloc(reinterpret_cast<void **>(&d_packed), CO_MAX * N * F)) ||
            (e = hipMalloc(reinterpret_cast<void **>(&d_small), BYTES)) ||
            (e = hipMalloc(reinterpret_cast<void **>(&d_ws), decds_encode_commit_workspace_bytes(CO_MAX))) ||
            (e = hipHostMalloc(reinterpret_cast<void **>(&h_small), BYTES, DECDS_HOST_MALLOC_FLAGS))) {
            release();  // all or nothing: a later call sees s == nullptr and sets the slot up again
            return e;
        }
        rows = d_rows + (16 - reinterpret_cast<uintptr_t>(d_rows)) % 128;
        return hipSuccess;
    }
    void release() {
        if (s) hip_tolerate(hipStreamSynchronize(s), "hipStreamSynchronize");
        for (uint8_t **p : {&d_src, &d_rows, &d_packed, &d_small, &d_ws}) {
            if (*p) hip_tolerate(hipFree(*p), "hipFree");
            *p = nullptr;
        }
        if (h_small) hip_tolerate(hipHostFree(h_small), "hipHostFree");
        if (s) hip_tolerate(hipStreamDestroy(s), "hipStreamDestroy");
        h_small = rows = nullptr;
        s = nullptr;
    }
    ~CoSlot() { release(); }
};

struct Coalescer {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<EncReq *> pending;
    CoSlot slot[2];
    PinnedPool in_pool{CS, 2 * CO_MAX}, out_pool{CO_OUT, 2 * CO_MAX};
    std::atomic<int> callers{0};
    ~Coalescer() {
        in_pool.clear();
        out_pool.clear();
    }
};

// off by default: per-call lanes capped at 8 measured faster at 1-16 callers
bool coalesce_enabled() {
    const char *e = std::getenv("DECDS_CHUNKSET_COALESCE");
    return e && std::atoi(e) != 0;
}

// one batch of m requests on slot sl (the caller holds sl.busy); returns the batch status
int co_run(decds_ctx *ctx, CoSlot &sl, EncReq *const *req, size_t m) {
    hipError_t e;
    if (!sl.s && (e = sl.init())) return decds_hip_error(e, "coalesced ChunkSet::new slot setup");
    for (size_t i = 0; i < m; i++) {
        std::memcpy(sl.h_small + CoSlot::O_CV + i * N * K, req[i]->cv, N * K);
        const uint64_t id = req[i]->id;
        std::memcpy(sl.h_small + CoSlot::O_IDS + i * 8, &id, 8);
        if ((e = hipMemcpyAsync(sl.d_src + i * CS, req[i]->in, CS, hipMemcpyHostToDevice, sl.s)))
            return decds_hip_error(e, "H2D (chunkset)");
    }
    if ((e = hipMemcpyAsync(sl.d_small, sl.h_small, CoSlot::O_DIG, hipMemcpyHostToDevice, sl.s)))
        return decds_hip_error(e, "H2D (coding vectors)");
    int s = encode_commit_ids(ctx, sl.d_src, m, sl.d_small + CoSlot::O_CV, sl.rows, CO_P, 0,
                              reinterpret_cast<const uint64_t *>(sl.d_small + CoSlot::O_IDS), sl.d_small + CoSlot::O_DIG,
                              sl.d_small + CoSlot::O_ROOT, sl.d_small + CoSlot::O_PRF, sl.d_ws, sl.s);
    if (s) return s;
    // rows repacked at pitch F on the device (a blit over HBM), so each request's 16 rows leave in one
    // contiguous DMA: a host-side 2D copy of odd-length rows was the slow path (r05c: 3.4 GiB/s)
    if ((e = hipMemcpy2DAsync(sl.d_packed, F, sl.rows, CO_P, F, m * N, hipMemcpyDeviceToDevice, sl.s)))
        return decds_hip_error(e, "D2D (row repack)");
    for (size_t i = 0; i < m; i++) {
        uint8_t *o = req[i]->out;
        if ((e = hipMemcpyAsync(o, sl.d_packed + i * N * F, N * F, hipMemcpyDeviceToHost, sl.s)) ||
            (e = hipMemcpyAsync(o + N * F, sl.d_small + CoSlot::O_ROOT + i * 32, 32, hipMemcpyDeviceToHost, sl.s)) ||
            (e = hipMemcpyAsync(o + N * F + 32, sl.d_small + CoSlot::O_PRF + i * N * PROOF_SIZE * 32, N * PROOF_SIZE * 32,
                                hipMemcpyDeviceToHost, sl.s)))
            return decds_hip_error(e, "D2H (coded rows)");
    }
    if ((e = hipStreamSynchronize(sl.s))) return decds_hip_error(e, "hipStreamSynchronize");
    return DECDS_OK;
}

// ChunkSet::new through the coalescer: data already checked (len == CS), cv drawn
int co_chunkset_new(decds_ctx *ctx, size_t chunkset_id, const uint8_t *data, const uint8_t *cv, decds_chunkset **out);

}  // namespace decds

void decds_lanes_destroy(decds_ctx *ctx) {
    {
        std::lock_guard<std::mutex> g(ctx->lane_mu);
        for (Lane *l : ctx->lanes_all) delete l;
        ctx->lanes_all.clear();
        ctx->lanes_free.clear();
    }
    delete ctx->coalescer;
    ctx->coalescer = nullptr;
}

struct decds_chunkset {
    size_t id;
    std::unique_ptr<uint8_t[]> coded;  // 16 x F, rlnc full coded pieces (not zero-filled first)
    uint8_t root[32];             // MerkleTree root of the 16 chunk digests (chunkset.rs:57)
    uint8_t proofs[N][PROOF_SIZE][32];
    std::vector<uint8_t> blob_proof;  // appended to every chunk's proof (chunkset.rs:98-102)
};

int decds::co_chunkset_new(decds_ctx *ctx, size_t chunkset_id, const uint8_t *data, const uint8_t *cv,
                           decds_chunkset **out) {
    Coalescer *co;
    {
        std::lock_guard<std::mutex> g(ctx->lane_mu);
        if (!ctx->coalescer) ctx->coalescer = new Coalescer;
        co = ctx->coalescer;
    }
    EncReq r;
    r.id = chunkset_id;
    std::memcpy(r.cv, cv, N * K);
    hipError_t e;
    if ((e = co->in_pool.get(&r.in)) || (e = co->out_pool.get(&r.out))) {
        co->in_pool.put(r.in);
        return decds_hip_error(e, "page-locked staging");
    }
    // the copy into page-locked memory runs on the caller's own thread when other callers are copying
    // too (they are the parallelism), else on the host pool
    if (co->callers.fetch_add(1) > 0)
        std::memcpy(r.in, data, CS);
    else
        par_memcpy(r.in, data, CS);
    co->callers.fetch_sub(1);
    {
        std::unique_lock<std::mutex> g(co->mu);
        co->pending.push_back(&r);
        while (!r.done) {
            int k = !co->slot[0].busy ? 0 : !co->slot[1].busy ? 1 : -1;
            if (k < 0 || co->pending.empty()) {
                co->cv.wait(g);
                continue;
            }
            CoSlot &sl = co->slot[k];
            sl.busy = true;
            EncReq *batch[CO_MAX];
            size_t m = 0;
            while (m < CO_MAX && !co->pending.empty()) {
                batch[m++] = co->pending.front();
                co->pending.pop_front();
            }
            g.unlock();
            int st = co_run(ctx, sl, batch, m);
            const std::string msg = st ? decds_last_error() : std::string();
            g.lock();
            for (size_t i = 0; i < m; i++) {
                batch[i]->status = st;
                batch[i]->err = msg;
                batch[i]->done = true;
            }
            sl.busy = false;
            co->cv.notify_all();
        }
    }
    co->in_pool.put(r.in);
    if (r.status != DECDS_OK) {
        co->out_pool.put(r.out);
        return decds_set_error(r.status, "%s", r.err.c_str());
    }
    auto *c = new decds_chunkset{chunkset_id, std::unique_ptr<uint8_t[]>(new uint8_t[N * F]), {}, {}, {}};
    std::memcpy(c->coded.get(), r.out, N * F);
    std::memcpy(c->root, r.out + N * F, 32);
    std::memcpy(c->proofs, r.out + N * F + 32, sizeof c->proofs);
    co->out_pool.put(r.out);
    *out = c;
    return DECDS_OK;
}

struct decds_repairing_chunkset {
    decds_ctx *ctx;
    size_t id;
    bool has_commitment;
    uint8_t commitment[32];
    uint8_t basis[K * K];
    uint8_t pivots[K];
    uint32_t rank;
    bool repaired;
    std::vector<uint8_t> rows;  // accepted full coded pieces, acceptance order
    // a repair whose out buffer was too small keeps its result here: the retry only copies it out
    std::vector<uint8_t> decoded;
    size_t decoded_len = 0;
};

extern "C" {

int decds_chunkset_new(decds_ctx *ctx, size_t chunkset_id, const uint8_t *data, size_t len,
                       const uint8_t *coeffs, decds_chunkset **out) {
    if (!out) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null out pointer");
    *out = nullptr;
    if (len != CS) return decds_set_error(DECDS_ERR_INVALID_CHUNKSET_SIZE, "invalid chunkset size: %zuB, expected: %lluB",
                                          len, (unsigned long long)CS);
    if (!data) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null data");
    int s = decds_ctx_bind(ctx);
    if (s) return s;
    if (coalesce_enabled()) {
        uint8_t cvb[N * K];
        if (coeffs) {
            std::memcpy(cvb, coeffs, N * K);
        } else {
            std::lock_guard<std::mutex> g(g_rng_mu);
            for (size_t i = 0; i < N * K; i++) cvb[i] = (uint8_t)rng()();
        }
        return co_chunkset_new(ctx, chunkset_id, data, cvb, out);
    }
    LaneGuard lg{ctx};
    if ((s = lane_acquire(ctx, &lg.l))) return s;
    Lane &L = *lg.l;
    uint8_t *cv = L.h_small + SM_CV;
    if (coeffs) {
        std::memcpy(cv, coeffs, N * K);
    } else {
        std::lock_guard<std::mutex> g(g_rng_mu);
        for (size_t i = 0; i < N * K; i++) cv[i] = (uint8_t)rng()();
    }
    par_memcpy(L.h_big, data, CS);
    hipError_t e;
    if ((e = hipMemcpyAsync(L.d_cs, L.h_big, CS, hipMemcpyHostToDevice, L.s)) ||
        (e = hipMemcpyAsync(L.d_small + SM_CV, cv, N * K, hipMemcpyHostToDevice, L.s)))
        return decds_hip_error(e, "H2D");
    if ((s = decds_encode_batch(ctx, L.d_cs, 1, L.d_small + SM_CV, L.d_coded, F, L.s))) return s;
    // chunkset.rs:54-63: chunk digests -> 16-leaf Merkle tree -> root + one proof per chunk
    if ((s = decds_commit_batch(ctx, L.d_coded, F, 1, chunkset_id, L.d_small + SM_DIG, L.d_small + SM_ROOT,
                                L.d_small + SM_PRF, L.s)))
        return s;
    if ((e = hipMemcpyAsync(L.h_big, L.d_coded, N * F, hipMemcpyDeviceToHost, L.s)) ||
        (e = hipMemcpyAsync(L.h_small + SM_ROOT, L.d_small + SM_ROOT, SM_BYTES - SM_ROOT, hipMemcpyDeviceToHost, L.s)) ||
        (e = hipStreamSynchronize(L.s)))
        return decds_hip_error(e, "D2H");
    auto *c = new decds_chunkset{chunkset_id, std::unique_ptr<uint8_t[]>(new uint8_t[N * F]), {}, {}, {}};
    par_memcpy(c->coded.get(), L.h_big, N * F);
    std::memcpy(c->root, L.h_small + SM_ROOT, 32);
    std::memcpy(c->proofs, L.h_small + SM_PRF, sizeof c->proofs);
    *out = c;
    return DECDS_OK;
}

int decds_chunkset_get_chunk(const decds_chunkset *cs, size_t chunk_id, uint8_t *out, size_t out_len,
                             size_t *global_chunk_id) {
    if (!cs) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null chunkset");
    if (chunk_id >= N) return decds_set_error(DECDS_ERR_INVALID_SHARE_ID, "invalid erasure coded share id: %zu (num_shares: %u)",
                                              chunk_id, N);
    if (out) {
        if (out_len < F) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "out buffer < %llu", (unsigned long long)F);
        std::memcpy(out, cs->coded.get() + chunk_id * F, F);
    }
    if (global_chunk_id) *global_chunk_id = cs->id * N + chunk_id;  // chunkset.rs:47
    return DECDS_OK;
}

int decds_chunkset_get_root_commitment(const decds_chunkset *cs, uint8_t out[32]) {
    if (!cs || !out) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null argument");
    std::memcpy(out, cs->root, 32);
    return DECDS_OK;
}

int decds_chunkset_get_chunk_proof(const decds_chunkset *cs, size_t chunk_id, uint8_t *out, size_t out_len,
                                   size_t *proof_len) {
    if (!cs) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null chunkset");
    if (chunk_id >= N) return decds_set_error(DECDS_ERR_INVALID_SHARE_ID, "invalid erasure coded share id: %zu (num_shares: %u)",
                                              chunk_id, N);
    const size_t hashes = PROOF_SIZE + cs->blob_proof.size() / 32;
    if (proof_len) *proof_len = hashes;
    if (out) {
        if (out_len < hashes * 32) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "out buffer < %zu", hashes * 32);
        std::memcpy(out, cs->proofs[chunk_id], PROOF_SIZE * 32);
        if (!cs->blob_proof.empty()) std::memcpy(out + PROOF_SIZE * 32, cs->blob_proof.data(), cs->blob_proof.size());
    }
    return DECDS_OK;
}

int decds_chunkset_append_blob_inclusion_proof(decds_chunkset *cs, const uint8_t *blob_proof, size_t len) {
    if (!cs || (len && !blob_proof)) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null argument");
    cs->blob_proof.insert(cs->blob_proof.end(), blob_proof, blob_proof + len * 32);  // empty: no-op (chunkset.rs:99)
    return DECDS_OK;
}

size_t decds_chunkset_id(const decds_chunkset *cs) { return cs ? cs->id : 0; }
void decds_chunkset_free(decds_chunkset *cs) { delete cs; }

int decds_repairing_chunkset_new(decds_ctx *ctx, size_t chunkset_id, const uint8_t *commitment,
                                 decds_repairing_chunkset **out) {
    if (!ctx || !out) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null argument");
    auto *r = new decds_repairing_chunkset;
    r->ctx = ctx;
    r->id = chunkset_id;
    r->has_commitment = commitment != nullptr;
    if (commitment) std::memcpy(r->commitment, commitment, 32);
    std::memset(r->basis, 0, sizeof r->basis);
    std::memset(r->pivots, 0, sizeof r->pivots);
    r->rank = 0;
    r->repaired = false;
    r->rows.reserve(K * F);
    *out = r;
    return DECDS_OK;
}

int decds_repairing_chunkset_add_chunk_unvalidated(decds_repairing_chunkset *r, size_t chunk_chunkset_id,
                                                   const uint8_t *data, size_t len) {
    if (!r) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null repairing chunkset");
    if (r->repaired) return decds_set_error(DECDS_ERR_CHUNKSET_ALREADY_REPAIRED, "chunkset %zu is already repaired", r->id);
    // chunkset.rs:174-176
    if (chunk_chunkset_id != r->id)
        return decds_set_error(DECDS_ERR_INVALID_CHUNK_METADATA, "invalid chunk for chunkset %zu", chunk_chunkset_id);
    // chunkset.rs:177-179
    if (r->rank == K) return decds_set_error(DECDS_ERR_CHUNKSET_READY_TO_REPAIR, "chunkset %zu is ready to repair", r->id);
    // chunkset.rs:181-183 -> rlnc Decoder::decode: wrong length or a piece that does not raise the
    // rank is an error mapped to ChunkDecodingFailed(chunkset_id, msg)
    if (!data || len != F)
        return decds_set_error(DECDS_ERR_CHUNK_DECODING_FAILED, "decoding chunk for chunkset %zu failed: invalid piece length %zu",
                               chunk_chunkset_id, len);
    if (!decds_rank_push(r->basis, r->pivots, &r->rank, data, r->ctx->poly))
        return decds_set_error(DECDS_ERR_CHUNK_DECODING_FAILED, "decoding chunk for chunkset %zu failed: received piece is not useful",
                               chunk_chunkset_id);
    r->rows.insert(r->rows.end(), data, data + F);
    return DECDS_OK;
}

int decds_repairing_chunkset_add_chunk(decds_repairing_chunkset *r, size_t chunk_chunkset_id, size_t chunk_id,
                                       const uint8_t *data, size_t len, const uint8_t *proof, size_t proof_len) {
    if (!r) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null repairing chunkset");
    if (!r->has_commitment) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "repairing chunkset has no commitment");
    // chunkset.rs:152 -> chunk.rs:103-110: leaf chunk_id % 16, first PROOF_SIZE hashes
    bool ok = proof && proof_len >= PROOF_SIZE && (data || len == 0);
    if (ok) {
        uint8_t leaf[32];
        decds_chunk_digest(chunk_chunkset_id, chunk_id, data, len, leaf);
        ok = decds_merkle_verify(chunk_id % N, leaf, proof, PROOF_SIZE, r->commitment) == 1;
    }
    if (!ok) return decds_set_error(DECDS_ERR_INVALID_PROOF_IN_CHUNK, "invalid proof in chunk of chunkset %zu", chunk_chunkset_id);
    return decds_repairing_chunkset_add_chunk_unvalidated(r, chunk_chunkset_id, data, len);
}

int decds_repairing_chunkset_is_ready_to_repair(const decds_repairing_chunkset *r) {
    return r && !r->repaired && r->rank == K;
}

int decds_repairing_chunkset_repair(decds_repairing_chunkset *r, uint8_t *out, size_t out_cap, size_t *out_len) {
    if (!r) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null repairing chunkset");
    if (r->repaired) return decds_set_error(DECDS_ERR_CHUNKSET_ALREADY_REPAIRED, "chunkset %zu is already repaired", r->id);
    // chunkset.rs:201,206
    if (r->rank != K) return decds_set_error(DECDS_ERR_CHUNKSET_NOT_YET_READY, "chunkset %zu is not ready to repair", r->id);
    if (!out) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null out buffer");
    // the decoder is consumed only by a repair that hands its bytes out (chunkset.rs:200)
    auto deliver = [&](const uint8_t *body, const uint8_t *tail, size_t len) -> int {
        if (out_len) *out_len = len;
        if (out_cap < len) {
            // kept (decoded bytes + tail, CS + 10 bytes held until the repair completes or the
            // object is freed): a retry with a larger buffer only copies. Without the memory for the
            // copy the caller still learns the length and the retry decodes again.
            if (r->decoded.empty()) {
                try {
                    r->decoded.resize(CS + K);
                } catch (const std::bad_alloc &) {
                    return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "out buffer %zu < decoded length %zu "
                                           "(no host memory to keep the decoded bytes: a retry decodes again)", out_cap, len);
                }
                par_memcpy(r->decoded.data(), body, CS);
                std::memcpy(r->decoded.data() + CS, tail, K);
                r->decoded_len = len;
            }
            return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "out buffer %zu < decoded length %zu", out_cap, len);
        }
        par_memcpy(out, body, std::min<size_t>(len, CS));
        if (len > CS) std::memcpy(out + CS, tail, len - CS);
        r->repaired = true;
        r->rows.clear();
        r->rows.shrink_to_fit();
        r->decoded.clear();
        r->decoded.shrink_to_fit();
        return DECDS_OK;
    };
    if (!r->decoded.empty()) return deliver(r->decoded.data(), r->decoded.data() + CS, r->decoded_len);
    decds_ctx *ctx = r->ctx;
    int s = decds_ctx_bind(ctx);
    if (s) return s;
    LaneGuard lg{ctx};
    if ((s = lane_acquire(ctx, &lg.l))) return s;
    Lane &L = *lg.l;
    // the accepted rows as coded rows 0..9 of one chunkset, arrival order = acceptance order
    uint8_t *cand = L.h_small + SM_CAND;
    for (uint32_t i = 0; i < N; i++) cand[i] = i < K ? (uint8_t)i : (uint8_t)DECDS_NO_CANDIDATE;
    par_memcpy(L.h_big, r->rows.data(), K * F);
    hipError_t e;
    if ((e = hipMemcpyAsync(L.d_coded, L.h_big, K * F, hipMemcpyHostToDevice, L.s)) ||
        (e = hipMemcpyAsync(L.d_small + SM_CAND, cand, N, hipMemcpyHostToDevice, L.s)))
        return decds_hip_error(e, "H2D");
    if ((s = decds_repair_batch(ctx, L.d_coded, F, 1, L.d_small + SM_CAND, L.d_small + SM_PLAN,
                                reinterpret_cast<int8_t *>(L.d_small + SM_VERD), L.d_cs,
                                reinterpret_cast<int32_t *>(L.d_small + SM_STATUS),
                                reinterpret_cast<decds_repair_info *>(L.d_small + SM_INFO), L.s)))
        return s;
    if ((e = hipMemcpyAsync(L.h_big, L.d_cs, CS, hipMemcpyDeviceToHost, L.s)) ||
        (e = hipMemcpyAsync(L.h_small + SM_STATUS, L.d_small + SM_STATUS, 4, hipMemcpyDeviceToHost, L.s)) ||
        (e = hipMemcpyAsync(L.h_small + SM_INFO, L.d_small + SM_INFO, sizeof(decds_repair_info), hipMemcpyDeviceToHost, L.s)) ||
        (e = hipStreamSynchronize(L.s)))
        return decds_hip_error(e, "D2H");
    int32_t st;
    std::memcpy(&st, L.h_small + SM_STATUS, 4);
    if (st != DECDS_OK)  // chunkset.rs:202-204: no boundary marker in the decoded data
        return decds_set_error(DECDS_ERR_CHUNKSET_REPAIRING_FAILED, "chunkset %zu repairing failed: RLNC Decoding error: %s",
                               r->id, st == DECDS_ERR_CHUNKSET_REPAIRING_FAILED ? "invalid decoded data format" : decds_status_string(st));
    decds_repair_info info;
    std::memcpy(&info, L.h_small + SM_INFO, sizeof info);
    // get_decoded_data's cut at the last marker (CS when intact)
    return deliver(L.h_big, info.tail, info.decoded_len);
}

void decds_repairing_chunkset_free(decds_repairing_chunkset *r) { delete r; }

}  // extern "C"

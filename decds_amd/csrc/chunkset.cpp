// chunkset.cpp — host-side mirror of decds-lib's chunkset API (chunkset.rs) and of the blob-level
// chunkset iteration (blob.rs) over the gfx950 batch kernels. Same names, argument meaning and
// error behaviour as the reference, including ChunkSet::new's commitment (digests, Merkle root,
// proofs: computed on the device by decds_commit_batch) and RepairingChunkSet::add_chunk's proof check.
//
//   decds_chunkset_new                 ChunkSet::new                    chunkset.rs:37-69
//   decds_chunkset_get_chunk           ChunkSet::get_chunk              chunkset.rs:87-89
//   decds_repairing_chunkset_*         RepairingChunkSet                chunkset.rs:107-208
//   decds_blob_encode_host             Blob::new chunkset loop          blob.rs:244-264
//   decds_blob_repair_host             RepairingBlob add/get_repaired   blob.rs:373-394, 451-473
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <random>
#include <vector>

#include "../../include/decds_rlnc.h"
#include "capi_internal.h"
#include "rlnc_layout.h"

using namespace decds;

namespace {

// RAII device buffer
struct DevBuf {
    uint8_t *p = nullptr;
    hipError_t alloc(size_t n) { return hipMalloc(reinterpret_cast<void **>(&p), n); }
    ~DevBuf() {
        if (p) (void)hipFree(p);
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

struct decds_chunkset {
    size_t id;
    std::vector<uint8_t> coded;   // 16 x F, rlnc full coded pieces
    uint8_t root[32];             // MerkleTree root of the 16 chunk digests (chunkset.rs:57)
    uint8_t proofs[N][PROOF_SIZE][32];
    std::vector<uint8_t> blob_proof;  // appended to every chunk's proof (chunkset.rs:98-102)
};

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
    uint8_t cv[N * K];
    if (coeffs) {
        std::memcpy(cv, coeffs, sizeof cv);
    } else {
        std::lock_guard<std::mutex> g(g_rng_mu);
        for (auto &b : cv) b = (uint8_t)rng()();
    }
    DevBuf dsrc, dcv, ddst, dcommit;
    constexpr size_t DIG = N * 32, ROOT = 32, PRF = N * PROOF_SIZE * 32;
    hipError_t e;
    if ((e = dsrc.alloc(CS)) || (e = dcv.alloc(sizeof cv)) || (e = ddst.alloc(N * F)) || (e = dcommit.alloc(DIG + ROOT + PRF)))
        return decds_hip_error(e, "hipMalloc");
    if ((e = hipMemcpy(dsrc.p, data, CS, hipMemcpyHostToDevice)) || (e = hipMemcpy(dcv.p, cv, sizeof cv, hipMemcpyHostToDevice)))
        return decds_hip_error(e, "hipMemcpy H2D");
    if ((s = decds_encode_batch(ctx, dsrc.p, 1, dcv.p, ddst.p, F, nullptr))) return s;
    // chunkset.rs:54-63: chunk digests -> 16-leaf Merkle tree -> root + one proof per chunk
    if ((s = decds_commit_batch(ctx, ddst.p, F, 1, chunkset_id, dcommit.p, dcommit.p + DIG, dcommit.p + DIG + ROOT, nullptr)))
        return s;
    auto *c = new decds_chunkset{chunkset_id, std::vector<uint8_t>(N * F), {}, {}, {}};
    if ((e = hipMemcpy(c->coded.data(), ddst.p, N * F, hipMemcpyDeviceToHost)) ||
        (e = hipMemcpy(c->root, dcommit.p + DIG, ROOT, hipMemcpyDeviceToHost)) ||
        (e = hipMemcpy(c->proofs, dcommit.p + DIG + ROOT, PRF, hipMemcpyDeviceToHost))) {
        delete c;
        return decds_hip_error(e, "hipMemcpy D2H");
    }
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
        std::memcpy(out, cs->coded.data() + chunk_id * F, F);
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

int decds_repairing_chunkset_repair(decds_repairing_chunkset *r, uint8_t *out, size_t out_len) {
    if (!r) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null repairing chunkset");
    if (r->repaired) return decds_set_error(DECDS_ERR_CHUNKSET_ALREADY_REPAIRED, "chunkset %zu is already repaired", r->id);
    // chunkset.rs:201,206
    if (r->rank != K) return decds_set_error(DECDS_ERR_CHUNKSET_NOT_YET_READY, "chunkset %zu is not ready to repair", r->id);
    if (!out || out_len < CS) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "out buffer < %llu", (unsigned long long)CS);
    int s = decds_ctx_bind(r->ctx);
    if (s) return s;
    DevBuf dcoded, dcand, dplan, dverd, dstat, ddst;
    hipError_t e;
    if ((e = dcoded.alloc(N * F)) || (e = dcand.alloc(N)) || (e = dplan.alloc(DECDS_REPAIR_PLAN_BYTES)) ||
        (e = dverd.alloc(N)) || (e = dstat.alloc(sizeof(int32_t))) || (e = ddst.alloc(CS)))
        return decds_hip_error(e, "hipMalloc");
    uint8_t cand[N];
    for (uint32_t i = 0; i < N; i++) cand[i] = i < K ? (uint8_t)i : (uint8_t)DECDS_NO_CANDIDATE;
    if ((e = hipMemcpy(dcoded.p, r->rows.data(), K * F, hipMemcpyHostToDevice)) ||
        (e = hipMemcpy(dcand.p, cand, N, hipMemcpyHostToDevice)))
        return decds_hip_error(e, "hipMemcpy H2D");
    if ((s = decds_repair_batch(r->ctx, dcoded.p, F, 1, dcand.p, dplan.p, reinterpret_cast<int8_t *>(dverd.p), ddst.p,
                                reinterpret_cast<int32_t *>(dstat.p), nullptr)))
        return s;
    int32_t st = 0;
    if ((e = hipMemcpy(&st, dstat.p, sizeof st, hipMemcpyDeviceToHost)) || (e = hipMemcpy(out, ddst.p, CS, hipMemcpyDeviceToHost)))
        return decds_hip_error(e, "hipMemcpy D2H");
    if (st != DECDS_OK)
        return decds_set_error(DECDS_ERR_CHUNKSET_REPAIRING_FAILED, "chunkset %zu repairing failed: RLNC Decoding error: %s",
                               r->id, st == DECDS_ERR_CHUNKSET_REPAIRING_FAILED ? "invalid decoded data format" : decds_status_string(st));
    r->repaired = true;  // repair(self) consumes the decoder (chunkset.rs:200)
    r->rows.clear();
    r->rows.shrink_to_fit();
    return DECDS_OK;
}

void decds_repairing_chunkset_free(decds_repairing_chunkset *r) { delete r; }

// ------------------------------------------------------------------ blob-level batching ------
// Two streams alternate over batches: while batch b runs its kernel, batch b+1's H2D and batch
// b-1's D2H proceed on the copy engines. Caller buffers are page-locked with hipHostRegister for
// the duration of the call so the copies DMA directly from/to them.
namespace {
// Page-locks a caller buffer for the duration of one call unless the caller already did
// (decds_host_register): then registration fails with "already registered" and is left alone.
struct HostReg {
    void *p = nullptr;
    bool ok = false;
    HostReg(const void *ptr, size_t n) : p(const_cast<void *>(ptr)) {
        ok = n && hipHostRegister(p, n, hipHostRegisterDefault) == hipSuccess;
        if (!ok) (void)hipGetLastError();
    }
    ~HostReg() {
        if (ok) (void)hipHostUnregister(p);
    }
};
}  // namespace

// Copy / compute pipeline of the host blob paths: one stream per engine (H2D, kernels, D2H) and
// SLOTS buffer sets, ordered by events, so the link carries H2D and D2H at the same time (PCIe is
// full duplex: 53 + 57 GB/s alone, 98 GB/s together, tools/pciebench.py). Round 1's two streams,
// each H2D -> kernel -> D2H in order, kept one direction busy at a time (60 GB/s in sum).
constexpr int SLOTS = 3;
inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
struct Pipe {
    hipStream_t h2d = nullptr, comp = nullptr, d2h = nullptr;
    hipEvent_t in_done[SLOTS] = {}, k_done[SLOTS] = {}, out_done[SLOTS] = {};
    hipError_t init() {
        hipError_t e;
        for (hipStream_t *st : {&h2d, &comp, &d2h})
            if ((e = hipStreamCreateWithFlags(st, hipStreamNonBlocking))) return e;
        for (int i = 0; i < SLOTS; i++)
            for (hipEvent_t *ev : {&in_done[i], &k_done[i], &out_done[i]}) {
                if ((e = hipEventCreateWithFlags(ev, hipEventDisableTiming))) return e;
                if ((e = hipEventRecord(*ev, comp))) return e;  // every slot starts free
            }
        return hipSuccess;
    }
    hipError_t drain() {
        hipError_t e = hipSuccess, f;
        for (hipStream_t st : {h2d, comp, d2h})
            if (st && (f = hipStreamSynchronize(st)) && !e) e = f;
        return e;
    }
    ~Pipe() {
        (void)drain();
        for (int i = 0; i < SLOTS; i++)
            for (hipEvent_t ev : {in_done[i], k_done[i], out_done[i]})
                if (ev) (void)hipEventDestroy(ev);
        for (hipStream_t st : {h2d, comp, d2h})
            if (st) (void)hipStreamDestroy(st);
    }
};

int decds_blob_encode_host(decds_ctx *ctx, const uint8_t *blob, size_t blob_len, const uint8_t *coeffs_host,
                           uint8_t *coded_host, size_t batch) {
    if (blob_len == 0) return decds_set_error(DECDS_ERR_EMPTY_DATA_FOR_BLOB, "empty data for blob");  // blob.rs:245-247
    if (!blob || !coeffs_host || !coded_host) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null buffer");
    int s = decds_ctx_bind(ctx);
    if (s) return s;
    const size_t n = (blob_len + CS - 1) / CS;  // blob.rs:252
    if (batch == 0) batch = 16;  // 8-32 measured best
    batch = std::min(batch, n);
    HostReg rin(blob, blob_len), rout(coded_host, n * N * F), rcv(coeffs_host, n * N * K);
    std::lock_guard<std::mutex> lock(ctx->host_mu);
    uint8_t *din[SLOTS], *dout[SLOTS], *dcv[SLOTS];
    const size_t sz_in = align256(batch * CS), sz_out = align256(batch * N * F), sz_cv = align256(batch * N * K);
    uint8_t *base;
    hipError_t e;
    if ((e = decds_ctx_scratch(ctx, SLOTS * (sz_in + sz_out + sz_cv), &base))) return decds_hip_error(e, "hipMalloc");
    for (int i = 0; i < SLOTS; i++, base += sz_in + sz_out + sz_cv) din[i] = base, dout[i] = base + sz_in, dcv[i] = base + sz_in + sz_out;
    Pipe pp;
    if ((e = pp.init())) return decds_hip_error(e, "stream/event setup");
    int rc = DECDS_OK;
    for (size_t b0 = 0, it = 0; b0 < n && rc == DECDS_OK; b0 += batch, it++) {
        const int k = (int)(it % SLOTS);
        const size_t nb = std::min(batch, n - b0);
        const size_t off = b0 * CS, have = std::min(blob_len - off, nb * CS);
        // inputs of slot k: free once the slot's previous kernel has read them
        if ((e = hipStreamWaitEvent(pp.h2d, pp.k_done[k], 0)) ||
            (e = hipMemcpyAsync(din[k], blob + off, have, hipMemcpyHostToDevice, pp.h2d)) ||
            (have < nb * CS && (e = hipMemsetAsync(din[k] + have, 0, nb * CS - have, pp.h2d))) ||  // blob.rs:254 zero pad
            (e = hipMemcpyAsync(dcv[k], coeffs_host + b0 * N * K, nb * N * K, hipMemcpyHostToDevice, pp.h2d)) ||
            (e = hipEventRecord(pp.in_done[k], pp.h2d))) {
            rc = decds_hip_error(e, "H2D");
            break;
        }
        // coded rows of slot k: free once the slot's previous D2H has read them
        if ((e = hipStreamWaitEvent(pp.comp, pp.in_done[k], 0)) || (e = hipStreamWaitEvent(pp.comp, pp.out_done[k], 0))) {
            rc = decds_hip_error(e, "hipStreamWaitEvent");
            break;
        }
        if ((rc = decds_encode_batch(ctx, din[k], nb, dcv[k], dout[k], F, pp.comp))) break;
        if ((e = hipEventRecord(pp.k_done[k], pp.comp)) || (e = hipStreamWaitEvent(pp.d2h, pp.k_done[k], 0)) ||
            (e = hipMemcpyAsync(coded_host + b0 * N * F, dout[k], nb * N * F, hipMemcpyDeviceToHost, pp.d2h)) ||
            (e = hipEventRecord(pp.out_done[k], pp.d2h))) {
            rc = decds_hip_error(e, "D2H");
            break;
        }
    }
    if ((e = pp.drain()) && rc == DECDS_OK) rc = decds_hip_error(e, "hipStreamSynchronize");
    return rc;
}

int decds_blob_repair_host(decds_ctx *ctx, const uint8_t *coded_host, size_t n, const uint8_t *cand_host,
                           size_t blob_len, uint8_t *out, int32_t *status_host, size_t batch) {
    if (!coded_host || !cand_host || !out || !status_host || n == 0)
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null buffer or no chunksets");
    if (blob_len > n * CS || blob_len <= (n - 1) * CS)
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "blob length %zu inconsistent with %zu chunksets", blob_len, n);
    int s = decds_ctx_bind(ctx);
    if (s) return s;
    if (batch == 0) batch = 16;  // 8-32 measured best
    batch = std::min(batch, n);
    // RepairingBlob::add_chunk over the arrival order (blob.rs:373-394): the rank test runs on the
    // 10-byte coding vectors on the host, so only the 10 accepted rows of each chunkset cross PCIe
    std::vector<uint8_t> sel(n * K, 0);
    for (size_t c = 0; c < n; c++) {
        uint8_t basis[K * K], piv[K];
        uint32_t rank = 0;
        for (uint32_t a = 0; a < N && rank < K; a++) {
            const uint8_t row = cand_host[c * N + a];
            if (row >= N) break;
            if (decds_rank_push(basis, piv, &rank, coded_host + (c * N + row) * F, ctx->poly)) sel[c * K + rank - 1] = row;
        }
        status_host[c] = rank == K ? DECDS_OK : DECDS_ERR_CHUNKSET_NOT_YET_READY;
    }
    // per-slot candidate lists and device statuses in page-locked memory: a pageable source or
    // target would make hipMemcpyAsync a staged copy that blocks this thread until its stream
    // reaches it, stalling the issue of the next slot
    struct Pinned {
        void *p = nullptr;
        ~Pinned() {
            if (p) (void)hipHostFree(p);
        }
    } pin;
    {
        hipError_t pe = hipHostMalloc(&pin.p, SLOTS * batch * (N + sizeof(int32_t)), hipHostMallocDefault);
        if (pe) return decds_hip_error(pe, "hipHostMalloc");
    }
    uint8_t *cand_h[SLOTS];
    int32_t *stat_h[SLOTS];
    for (int i = 0; i < SLOTS; i++) {
        stat_h[i] = reinterpret_cast<int32_t *>(pin.p) + i * batch;
        cand_h[i] = reinterpret_cast<uint8_t *>(pin.p) + SLOTS * batch * sizeof(int32_t) + i * batch * N;
    }
    HostReg rout(out, blob_len), rin(coded_host, n * N * F);
    std::lock_guard<std::mutex> lock(ctx->host_mu);
    uint8_t *dcoded[SLOTS], *dcand[SLOTS], *dplan[SLOTS], *dverd[SLOTS], *dstat[SLOTS], *ddst[SLOTS];
    const size_t sz[6] = {align256(batch * N * F), align256(batch * N), align256(batch * DECDS_REPAIR_PLAN_BYTES),
                          align256(batch * N), align256(batch * sizeof(int32_t)), align256(batch * CS)};
    const size_t per = sz[0] + sz[1] + sz[2] + sz[3] + sz[4] + sz[5];
    uint8_t *base;
    hipError_t e;
    if ((e = decds_ctx_scratch(ctx, SLOTS * per, &base))) return decds_hip_error(e, "hipMalloc");
    for (int i = 0; i < SLOTS; i++) {
        uint8_t **dst[6] = {&dcoded[i], &dcand[i], &dplan[i], &dverd[i], &dstat[i], &ddst[i]};
        for (int j = 0; j < 6; j++) *dst[j] = base, base += sz[j];
    }
    Pipe pp;
    if ((e = pp.init())) return decds_hip_error(e, "stream/event setup");
    int rc = DECDS_OK;
    size_t pending_b0[SLOTS], pending_nb[SLOTS] = {};
    for (int i = 0; i < SLOTS; i++) pending_b0[i] = (size_t)-1;
    // host side of slot k once its D2H is done: device statuses, zeroed output of unrepaired chunksets
    auto finish = [&](int k) -> int {
        if (pending_b0[k] == (size_t)-1) return DECDS_OK;
        hipError_t ee = hipEventSynchronize(pp.out_done[k]);
        if (ee) return decds_hip_error(ee, "hipEventSynchronize");
        for (size_t c = 0; c < pending_nb[k]; c++) {
            const size_t cs = pending_b0[k] + c;
            int32_t &hs = status_host[cs];
            if (hs == DECDS_OK && stat_h[k][c] != DECDS_OK) hs = DECDS_ERR_CHUNKSET_REPAIRING_FAILED;
            if (hs != DECDS_OK) {  // no data for a chunkset that could not be repaired
                const size_t off = cs * CS;
                std::memset(out + off, 0, std::min(blob_len - off, (size_t)CS));
            }
        }
        pending_b0[k] = (size_t)-1;
        return DECDS_OK;
    };
    for (size_t b0 = 0, it = 0; b0 < n && rc == DECDS_OK; b0 += batch, it++) {
        const int k = (int)(it % SLOTS);
        if ((rc = finish(k))) break;  // slot k's previous batch fully done: all its buffers are free
        const size_t nb = std::min(batch, n - b0);
        // the accepted rows keep their own row slots on the device (slot layout = host layout less
        // b0 chunksets), so runs of consecutive accepted rows — across chunkset boundaries too —
        // cross the link as one copy each instead of one copy per row
        std::vector<uint8_t> take(nb * N, 0);
        for (size_t c = 0; c < nb; c++) {
            const bool ready = status_host[b0 + c] == DECDS_OK;
            for (uint32_t a = 0; a < N; a++)
                cand_h[k][c * N + a] = ready && a < K ? sel[(b0 + c) * K + a] : (uint8_t)DECDS_NO_CANDIDATE;
            if (ready)
                for (uint32_t a = 0; a < K; a++) take[c * N + sel[(b0 + c) * K + a]] = 1;
        }
        for (size_t r0 = 0; r0 < nb * N && rc == DECDS_OK;) {
            if (!take[r0]) {
                r0++;
                continue;
            }
            size_t r1 = r0 + 1;
            while (r1 < nb * N && take[r1]) r1++;
            if ((e = hipMemcpyAsync(dcoded[k] + r0 * F, coded_host + (b0 * N + r0) * F, (r1 - r0) * F,
                                    hipMemcpyHostToDevice, pp.h2d)))
                rc = decds_hip_error(e, "H2D");
            r0 = r1;
        }
        if (rc) break;
        if ((e = hipMemcpyAsync(dcand[k], cand_h[k], nb * N, hipMemcpyHostToDevice, pp.h2d)) ||
            (e = hipEventRecord(pp.in_done[k], pp.h2d)) || (e = hipStreamWaitEvent(pp.comp, pp.in_done[k], 0))) {
            rc = decds_hip_error(e, "H2D");
            break;
        }
        if ((rc = decds_repair_batch(ctx, dcoded[k], F, nb, dcand[k], dplan[k], reinterpret_cast<int8_t *>(dverd[k]),
                                     ddst[k], reinterpret_cast<int32_t *>(dstat[k]), pp.comp)))
            break;
        // blob.rs:464: truncate the last chunkset to its real size
        const size_t off = b0 * CS, keep = std::min(blob_len - off, nb * CS);
        if ((e = hipEventRecord(pp.k_done[k], pp.comp)) || (e = hipStreamWaitEvent(pp.d2h, pp.k_done[k], 0)) ||
            (e = hipMemcpyAsync(stat_h[k], dstat[k], nb * sizeof(int32_t), hipMemcpyDeviceToHost, pp.d2h)) ||
            (e = hipMemcpyAsync(out + off, ddst[k], keep, hipMemcpyDeviceToHost, pp.d2h)) ||
            (e = hipEventRecord(pp.out_done[k], pp.d2h))) {
            rc = decds_hip_error(e, "D2H");
            break;
        }
        pending_b0[k] = b0;
        pending_nb[k] = nb;
    }
    for (size_t j = 0; j < SLOTS; j++) {  // oldest pending slot first
        int r2 = finish((int)(j % SLOTS));
        if (r2 && rc == DECDS_OK) rc = r2;
    }
    if ((e = pp.drain()) && rc == DECDS_OK) rc = decds_hip_error(e, "hipStreamSynchronize");
    return rc;
}

int decds_host_register(const void *ptr, size_t len) {
    if (!ptr || !len) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null or empty buffer");
    hipError_t e = hipHostRegister(const_cast<void *>(ptr), len, hipHostRegisterDefault);
    return e == hipSuccess ? DECDS_OK : decds_hip_error(e, "hipHostRegister");
}

int decds_host_unregister(const void *ptr) {
    hipError_t e = hipHostUnregister(const_cast<void *>(ptr));
    return e == hipSuccess ? DECDS_OK : decds_hip_error(e, "hipHostUnregister");
}

}  // extern "C"

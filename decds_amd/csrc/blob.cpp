// blob.cpp — decds-lib's blob level (decds-lib/src/blob.rs) over the batch kernels:
//
//   decds_blob_encode_host[_multi]     Blob::new chunkset loop          blob.rs:244-264
//   decds_blob_repair_host[_multi]     RepairingBlob over all chunks    blob.rs:373-394, 451-473
//   decds_blob_*                       Blob (new, header, get_share)    blob.rs:227-318
//   decds_repairing_blob_*             RepairingBlob                    blob.rs:321-473
//
// Host paths stream batches of chunksets through one HIP stream per engine (H2D, kernels, D2H)
// over three event-ordered buffer slots, so PCIe carries both directions at once. Caller buffers
// registered with the library (decds_host_register / decds_host_alloc) are DMA'd directly; any
// other host memory goes through the context's pinned bounce rings (host_mem.h). The _multi forms
// shard chunksets by contiguous index range over several contexts (devices), one host thread each,
// with no collective: chunksets are independent (blob.rs:256-264).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/decds_rlnc.h"
#include "blake3_host.h"
#include "capi_internal.h"
#include "commit_kernels.h"
#include "rlnc_kernels.h"
#include "rlnc_layout.h"

using namespace decds;

namespace {
constexpr int SLOTS = 3;      // buffer slots of the encode pipeline and of the repair run form
constexpr int MAX_SLOTS = 6;  // events a Pipe holds (the gather form's slot count is tunable)
inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
}  // namespace

namespace decds {
// The host paths' three streams and per-slot events, one set per context (ctx->pipe): created by the
// context's first host-path call and kept (creating three streams and 18 events per call cost every
// call their set-up, and an event of a ring piece could outlive the stream it was recorded on).
// Calls on one context are serialised by ctx->host_mu; each ends with every stream drained, so the
// next call finds every slot event complete (every slot free).
struct Pipe {
    hipStream_t h2d = nullptr, comp = nullptr, d2h = nullptr;
    hipEvent_t in_done[MAX_SLOTS] = {}, k_done[MAX_SLOTS] = {}, out_done[MAX_SLOTS] = {};
    hipError_t init() {
        hipError_t e;
        // Stream priorities keep the two copy directions on different hardware queues. HIP backs the
        // streams of each priority level with a pool of at most GPU_MAX_HW_QUEUES (4) queues and, once
        // a pool is full, puts a new stream on the pool's least-used queue: with three equal-priority
        // streams created per call, whether H2D and D2H landed on one queue (copies then run one after
        // the other: blob encode 49-50 ms instead of 38 at 1 GiB, r07r) depended on how many streams the
        // process already held. The H2D stream goes on the high-priority pool (empty in most processes,
        // so it gets a queue of its own), the kernel and D2H streams on the normal one: the two copy
        // directions can never share a queue (encode/repair held 38 / 30 ms with 0-4 caller streams
        // alive, r07u). The range is [0, -1] here: two levels. Round 5 raised the kernel stream as well
        // ("h2d+comp"); that measured the same (encode 36.4-36.8 ms, repair 28.5-29.7 either way, r09e)
        // and gave the library's kernels precedence over the caller's own work on the device, so round 6
        // raises the H2D stream only. DECDS_PIPE_STREAMS=plain (all normal) | h2d+comp are
        // study switches.
        static const int mode = [] {
            const char *v = std::getenv("DECDS_PIPE_STREAMS");
            return !v ? 1 : !std::strcmp(v, "plain") ? 0 : !std::strcmp(v, "h2d+comp") ? 2 : 1;
        }();
        int least = 0, greatest = 0;
        if (mode == 0) {
            for (hipStream_t *st : {&h2d, &comp, &d2h})
                if ((e = hipStreamCreateWithFlags(st, hipStreamNonBlocking))) return e;
        } else if ((e = hipDeviceGetStreamPriorityRange(&least, &greatest)) ||
                   (e = hipStreamCreateWithPriority(&h2d, hipStreamNonBlocking, mode ? greatest : least)) ||
                   (e = hipStreamCreateWithPriority(&comp, hipStreamNonBlocking, mode == 2 ? greatest : least)) ||
                   (e = hipStreamCreateWithPriority(&d2h, hipStreamNonBlocking, least)))
            return e;
        for (int i = 0; i < MAX_SLOTS; i++)
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
        hip_tolerate(drain(), "hipStreamSynchronize (pipe teardown)");
        for (int i = 0; i < MAX_SLOTS; i++)
            for (hipEvent_t ev : {in_done[i], k_done[i], out_done[i]})
                if (ev) hip_tolerate(hipEventDestroy(ev), "hipEventDestroy");
        for (hipStream_t st : {h2d, comp, d2h})
            if (st) hip_tolerate(hipStreamDestroy(st), "hipStreamDestroy");
    }
};

void pipe_destroy(Pipe *p) { delete p; }
}  // namespace decds

namespace {
// the context's pipe, created on first use (caller holds ctx->host_mu)
hipError_t ctx_pipe(decds_ctx *ctx, Pipe **out) {
    if (!ctx->pipe) {
        auto *p = new Pipe;
        if (hipError_t e = p->init()) {
            delete p;
            return e;
        }
        ctx->pipe = p;
    }
    *out = ctx->pipe;
    return hipSuccess;
}

// commitment outputs of the encode pipeline (Blob::new: chunkset.rs:54-63 per chunkset)
struct CommitOut {
    uint8_t *roots;      // n x 32
    uint8_t *proofs;     // n x 16 x PROOF_SIZE x 32
    uint64_t first_id;
    uint8_t *group_cvs;  // whole-blob digest: the range's full 1 MiB groups' subtree values (32 B each), or null
};
constexpr size_t BLOB_GROUP = (size_t)1 << 20;  // blob_group_kernel's unit: 1024 BLAKE3 chunks

// Batch sizes of a host-path call over n chunksets. A pipeline over the three engines only overlaps
// once its first batch is in and until its last one is out: the first H2D and the last D2H run with
// the link's other direction idle (a 16-chunkset batch: 168 MB of inputs, ~3 ms). Ramped, the call
// starts and ends with small batches (batch/8, /4, /2 ... /2, /4, /8, /8) so those unoverlapped ends
// are short, and runs full batches in between: blob encode of 1 GiB −5 % at batch 16, −10 % at 32,
// repair ±1 % (r08c). DECDS_HOST_RAMP=0: fixed batches, =enc: ramped encode
// only (study switches).
std::vector<size_t> batch_sizes(size_t n, size_t batch, bool repair) {
    static const int mode = [] {  // 0 off, 1 encode only, 2 both
        const char *v = std::getenv("DECDS_HOST_RAMP");
        return !v ? 2 : !std::strcmp(v, "0") ? 0 : !std::strcmp(v, "enc") ? 1 : 2;
    }();
    const bool ramp = repair ? mode == 2 : mode >= 1;
    std::vector<size_t> head, tail, out;
    if (ramp && batch >= 16) {  // at 8, batches of 1 cost more than the short ends save (r08c)
        head = {batch / 8, batch / 4, batch / 2};
        tail = {batch / 2, batch / 4, batch / 8, batch / 8};
    }
    size_t ends = 0;
    for (size_t x : head) ends += x;
    for (size_t x : tail) ends += x;
    if (ends == 0 || n < ends + batch) {  // too short to ramp
        for (size_t b0 = 0; b0 < n; b0 += batch) out.push_back(std::min(batch, n - b0));
        return out;
    }
    out = head;
    size_t mid = n - ends;
    if (mid % batch) out.push_back(mid % batch);  // the odd batch first: it overlaps like the rest
    for (size_t i = 0; i < mid / batch; i++) out.push_back(batch);
    out.insert(out.end(), tail.begin(), tail.end());
    return out;
}

// End of a host-path call: complete the deferred copy-outs, drain every stream; after a failure
// the rings drop whatever they still hold for this call.
int finish_call(decds_ctx *ctx, Pipe &pp, int rc) {
    hipError_t e;
    if (rc == DECDS_OK && (e = ctx->out_ring.flush())) rc = decds_hip_error(e, "D2H (staged)");
    if ((e = pp.drain()) && rc == DECDS_OK) rc = decds_hip_error(e, "hipStreamSynchronize");
    if (rc != DECDS_OK) {
        ctx->out_ring.abandon();
        ctx->in_ring.abandon();
    }
    // the pipe's streams are drained: no ring piece keeps an event of this call for the next call (on
    // this context or, through the library's shared rings, another) to wait on
    ctx->in_ring.retire();
    ctx->out_ring.retire();
    return rc;
}

// Blob::new's chunkset loop over chunksets [0, ceil(blob_len / CS)) of `blob` (a shard's slice)
int encode_range(decds_ctx *ctx, const uint8_t *blob, size_t blob_len, const uint8_t *coeffs, uint8_t *coded,
                 size_t batch, const CommitOut *cm) {
    int s = decds_ctx_bind(ctx);
    if (s) return s;
    const size_t n = (blob_len + CS - 1) / CS;  // blob.rs:252
    if (batch == 0) batch = 16;                 // 8-32 measured best
    batch = std::min(batch, n);
    const size_t PRF = N * PROOF_SIZE * 32;
    HostUse uin(blob, blob_len), ucv(coeffs, n * N * K), uout(coded, n * N * F);
    std::lock_guard<std::mutex> lock(ctx->host_mu);
    // the commitment outputs (roots, proofs: 2,080 bytes per chunkset) land in the context's small
    // page-locked area and are copied to the caller's memory at the end: staged through the out ring,
    // two small copies per batch held ring pieces, and the host thread waited on them while the direct
    // input copies of a page-locked blob could have run ahead (Blob::new of a page-locked 1 GiB blob
    // 69 ms against 41 from pageable memory, r09c)
    // with group_cvs, the whole-blob digest's full 1 MiB groups are hashed on the device from each
    // batch's uploaded inputs (blob_group_kernel) and come back with the commitment outputs
    const size_t n_groups = cm && cm->group_cvs ? blob_len / BLOB_GROUP : 0;
    uint8_t *h_roots = nullptr, *h_prf = nullptr, *h_gcv = nullptr;
    if (cm) {
        hipError_t pe = decds_ctx_host_small(ctx, n * (32 + PRF) + n_groups * 32, &h_roots);
        if (pe) return decds_hip_error(pe, "hipHostMalloc (commitment outputs)");
        h_prf = h_roots + n * 32;
        h_gcv = h_prf + n * PRF;
    }
    // the coding vectors of the whole range go over in one copy ahead of the first batch (160 bytes
    // per chunkset): staged per batch from pageable memory, each small copy held a ring piece and
    // stalled the host's run-ahead (blob encode 15-17 GiB/s against 29 with them registered, r02zd)
    const size_t cv_all = align256(n * N * K), gcv_all = align256(n_groups * 32);
    const size_t sz[5] = {align256(batch * CS), align256(batch * N * F), cm ? align256(batch * N * 32) : 0,
                          cm ? align256(batch * 32) : 0, cm ? align256(batch * PRF) : 0};
    const size_t per = sz[0] + sz[1] + sz[2] + sz[3] + sz[4];
    uint8_t *base, *dcv, *dgcv, *din[SLOTS], *dout[SLOTS], *ddig[SLOTS], *drt[SLOTS], *dprf[SLOTS];
    hipError_t e;
    if ((e = decds_ctx_scratch(ctx, cv_all + gcv_all + SLOTS * per, &base))) return decds_hip_error(e, "hipMalloc");
    dcv = base, base += cv_all;
    dgcv = base, base += gcv_all;
    for (int i = 0; i < SLOTS; i++) {
        uint8_t **dst[5] = {&din[i], &dout[i], &ddig[i], &drt[i], &dprf[i]};
        for (int j = 0; j < 5; j++) *dst[j] = base, base += sz[j];
    }
    Pipe *ppp;
    if ((e = ctx_pipe(ctx, &ppp))) return decds_hip_error(e, "stream/event setup");
    Pipe &pp = *ppp;
    if ((e = copy_h2d(dcv, coeffs, n * N * K, ucv.pinned(), ctx->in_ring, pp.h2d)))
        return finish_call(ctx, pp, decds_hip_error(e, "H2D"));
    auto issue_d2h = [&](int k, size_t b0, size_t nb) -> int {
        if ((e = hipStreamWaitEvent(pp.d2h, pp.k_done[k], 0)) ||
            (e = copy_d2h(coded + b0 * N * F, dout[k], nb * N * F, uout.pinned(), ctx->out_ring, pp.d2h)) ||
            (cm && (e = hipMemcpyAsync(h_roots + b0 * 32, drt[k], nb * 32, hipMemcpyDeviceToHost, pp.d2h))) ||
            (cm && (e = hipMemcpyAsync(h_prf + b0 * PRF, dprf[k], nb * PRF, hipMemcpyDeviceToHost, pp.d2h))) ||
            (e = hipEventRecord(pp.out_done[k], pp.d2h)))
            return decds_hip_error(e, "D2H");
        return DECDS_OK;
    };
    int rc = DECDS_OK, pend = -1;
    size_t pend_b0 = 0, pend_nb = 0;
    const std::vector<size_t> sizes = batch_sizes(n, batch, false);
    for (size_t b0 = 0, it = 0; it < sizes.size() && rc == DECDS_OK; b0 += sizes[it], it++) {
        const int k = (int)(it % SLOTS);
        const size_t nb = sizes[it];
        const size_t off = b0 * CS, have = std::min(blob_len - off, nb * CS);
        // inputs of slot k: free once the slot's previous kernel has read them
        if ((e = hipStreamWaitEvent(pp.h2d, pp.k_done[k], 0)) ||
            (e = copy_h2d(din[k], blob + off, have, uin.pinned(), ctx->in_ring, pp.h2d)) ||
            (have < nb * CS && (e = hipMemsetAsync(din[k] + have, 0, nb * CS - have, pp.h2d))) ||  // blob.rs:254 zero pad
            (e = hipEventRecord(pp.in_done[k], pp.h2d))) {
            rc = decds_hip_error(e, "H2D");
            break;
        }
        // outputs of slot k: free once the slot's previous D2H has read them
        if ((e = hipStreamWaitEvent(pp.comp, pp.in_done[k], 0)) || (e = hipStreamWaitEvent(pp.comp, pp.out_done[k], 0))) {
            rc = decds_hip_error(e, "hipStreamWaitEvent");
            break;
        }
        if ((rc = decds_encode_batch(ctx, din[k], nb, dcv + b0 * N * K, dout[k], F, pp.comp))) break;
        if (cm && (rc = decds_commit_batch(ctx, dout[k], F, nb, cm->first_id + b0, ddig[k], drt[k], dprf[k], pp.comp)))
            break;
        if (n_groups && (e = launch_blob_groups(din[k], have / BLOB_GROUP, (cm->first_id * CS + off) / 1024,
                                                dgcv + off / BLOB_GROUP * 32, pp.comp))) {
            rc = decds_hip_error(e, "blob_group_kernel launch");
            break;
        }
        if ((e = hipEventRecord(pp.k_done[k], pp.comp))) {
            rc = decds_hip_error(e, "hipEventRecord");
            break;
        }
        // the previous batch's D2H goes out after this batch's inputs: on the staged path the host
        // then fills batch b+1's inputs while batch b-1's outputs drain
        if (pend >= 0 && (rc = issue_d2h(pend, pend_b0, pend_nb))) break;
        pend = k, pend_b0 = b0, pend_nb = nb;
    }
    if (rc == DECDS_OK && pend >= 0) rc = issue_d2h(pend, pend_b0, pend_nb);
    // the group values after the last batch's kernels (one stream: every earlier batch's too)
    if (rc == DECDS_OK && n_groups &&
        ((e = hipStreamWaitEvent(pp.d2h, pp.k_done[pend], 0)) ||
         (e = hipMemcpyAsync(h_gcv, dgcv, n_groups * 32, hipMemcpyDeviceToHost, pp.d2h))))
        rc = decds_hip_error(e, "D2H (blob digest groups)");
    rc = finish_call(ctx, pp, rc);
    if (rc == DECDS_OK && cm) {
        std::memcpy(cm->roots, h_roots, n * 32);
        std::memcpy(cm->proofs, h_prf, n * PRF);
        if (n_groups) std::memcpy(cm->group_cvs, h_gcv, n_groups * 32);
    }
    return rc;
}

// RepairingBlob::add_chunk's rank step over the arrival order of every chunkset (blob.rs:373-394,
// chunkset.rs:173-184) on the 10-byte coding vectors: sel[c*K + a] = the a-th accepted row of
// chunkset c, status NOT_YET_READY where the rank stays below 10
void accept_rows(decds_ctx *ctx, const uint8_t *coded_host, size_t n, const uint8_t *cand_host, uint8_t *sel,
                 int32_t *status_host) {
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
}

// The repair host path (RepairingBlob over every arrival + get_repaired_chunkset for chunksets [0, n)
// of a shard; coded / cand / out / status point at the shard's first chunkset, blob_len is its
// length), host-gather form: per batch, the host pool copies each ready chunkset's 10 accepted rows
// into the slot's page-locked staging buffer, densely (chunkset i of the batch's ready ones at
// i * 10 * F, rows in acceptance order), and the whole batch crosses the link as ONE copy; the plans
// (rows 0..9 in order + the inverse of the accepted coding vectors, host_gf_invert — RepairingBlob's
// decode_ready) go over beside them and the decode runs in its gather form. The gather of batch b+1
// overlaps batch b's copy. The run form below (repair_range_runs) sent each run of consecutive
// accepted rows as its own hipMemcpyAsync — about 500 per GiB, 29.6-31 ms at 1 GiB against 27.1-27.5
// gathered (r09b / r09e), a duplex link bound of about 22 ms. DECDS_REPAIR_GATHER=0 selects the run form
// (A/B switch).
int repair_range_gather(decds_ctx *ctx, const uint8_t *coded_host, size_t n, const uint8_t *cand_host, size_t blob_len,
                        uint8_t *out, int32_t *status_host, size_t batch) {
    int s = decds_ctx_bind(ctx);
    if (s) return s;
    if (batch == 0) batch = 16;
    batch = std::min(batch, n);
    // three slots (DECDS_REPAIR_SLOTS: 2-6): four or five, which let the gather of batch b start a batch
    // earlier, measured slower at 1 GiB (29.5-30.7 ms at batch 16, 36-41 at batch 8, against 27.1-27.5
    // with three, r09e)
    static const int S = [] {
        const char *v = std::getenv("DECDS_REPAIR_SLOTS");
        return v ? std::max(2, std::min(MAX_SLOTS, std::atoi(v))) : 3;
    }();
    std::vector<uint8_t> sel(n * K, 0);
    accept_rows(ctx, coded_host, n, cand_host, sel.data(), status_host);
    // per slot, page-locked: the staged rows (batch x 10 x F), and a small area of plans + decode
    // bases (H2D) and statuses + repair infos (D2H)
    const size_t stage = align256(batch * K * F);
    const size_t sm_plan = 0, sm_inb = align256(batch * sizeof(RepairPlan)), sm_outb = sm_inb + align256(batch * 8),
                 sm_h2d = sm_outb + align256(batch * 8), sm_stat = sm_h2d, sm_info = sm_stat + align256(batch * 4),
                 sm_bytes = sm_info + align256(batch * sizeof(decds_repair_info));
    struct Pinned {
        void *p = nullptr;
        size_t n = 0;
        ~Pinned() {
            if (p) host_pinned_free(p, n);
        }
    } hst;
    hipError_t e;
    if ((e = host_pinned_alloc(S * stage, &hst.p))) return decds_hip_error(e, "page-locked staging for accepted rows");
    hst.n = S * stage;
    HostUse uout(out, blob_len);
    std::lock_guard<std::mutex> lock(ctx->host_mu);
    uint8_t *hsm;
    if ((e = decds_ctx_host_small(ctx, S * sm_bytes, &hsm))) return decds_hip_error(e, "hipHostMalloc");
    uint8_t *hstage[MAX_SLOTS], *hsmall[MAX_SLOTS];
    for (int i = 0; i < S; i++) {
        hstage[i] = static_cast<uint8_t *>(hst.p) + i * stage;
        hsmall[i] = hsm + i * sm_bytes;
    }
    const size_t dsz = stage + sm_bytes + align256(batch * CS);
    uint8_t *base, *dstage[MAX_SLOTS], *dsmall[MAX_SLOTS], *ddst[MAX_SLOTS];
    if ((e = decds_ctx_scratch(ctx, S * dsz, &base))) return decds_hip_error(e, "hipMalloc");
    for (int i = 0; i < S; i++, base += dsz) {
        dstage[i] = base;
        dsmall[i] = base + stage;
        ddst[i] = base + stage + sm_bytes;
    }
    Pipe *ppp;
    if ((e = ctx_pipe(ctx, &ppp))) return decds_hip_error(e, "stream/event setup");
    Pipe &pp = *ppp;
    int rc = DECDS_OK;
    size_t pending_b0[MAX_SLOTS];
    std::vector<size_t> ready[MAX_SLOTS];  // batch positions of the slot's decoded chunksets
    for (int i = 0; i < S; i++) pending_b0[i] = (size_t)-1;
    // host side of slot k once its D2H is done (as repair_range_runs' finish): a chunkset whose decoded
    // data holds no boundary marker is ChunksetRepairingFailed and gets no data; one whose cut falls
    // inside the chunkset is zero past the cut (blob.rs:464 truncates only)
    auto finish = [&](int k) -> int {
        if (pending_b0[k] == (size_t)-1) return DECDS_OK;
        hipError_t ee = hipEventSynchronize(pp.out_done[k]);
        if (ee) return decds_hip_error(ee, "hipEventSynchronize");
        const int32_t *stat = reinterpret_cast<const int32_t *>(hsmall[k] + sm_stat);
        const decds_repair_info *info = reinterpret_cast<const decds_repair_info *>(hsmall[k] + sm_info);
        for (size_t i = 0; i < ready[k].size(); i++) {
            const size_t cs = pending_b0[k] + ready[k][i];
            const size_t off = cs * CS, size = std::min(blob_len - off, (size_t)CS);
            const size_t keep = stat[i] != DECDS_OK ? 0 : std::min<size_t>(info[i].decoded_len, size);
            if (stat[i] != DECDS_OK) status_host[cs] = DECDS_ERR_CHUNKSET_REPAIRING_FAILED;
            if (keep < size) {
                if (!uout.pinned() && (ee = ctx->out_ring.flush())) return decds_hip_error(ee, "D2H (staged)");
                std::memset(out + off + keep, 0, size - keep);
            }
        }
        pending_b0[k] = (size_t)-1;
        return DECDS_OK;
    };
    // Per batch b in slot k = b mod S, the host waits for as little as it can, as late as it can:
    // before gathering into the staging buffer only for batch b-S's H2D (long done), and only after
    // batch b's H2D and decode are queued for batch b-S's D2H (to post-process its statuses) — so the
    // link's H2D side always has the next batch queued. Device buffers are ordered on the device:
    // batch b's H2D after batch b-S's decode (k_done), its decode after batch b-S's D2H (out_done).
    const std::vector<size_t> sizes = batch_sizes(n, batch, true);
    std::vector<size_t> rl;
    for (size_t b0 = 0, it = 0; it < sizes.size() && rc == DECDS_OK; b0 += sizes[it], it++) {
        const int k = (int)(it % S);
        const size_t nb = sizes[it];
        if ((e = hipEventSynchronize(pp.in_done[k]))) {  // the staging buffer and plans of batch b-S sent
            rc = decds_hip_error(e, "hipEventSynchronize");
            break;
        }
        rl.clear();
        for (size_t c = 0; c < nb; c++)
            if (status_host[b0 + c] == DECDS_OK) rl.push_back(c);
        const size_t m = rl.size();
        RepairPlan *plans = reinterpret_cast<RepairPlan *>(hsmall[k] + sm_plan);
        uint64_t *inb = reinterpret_cast<uint64_t *>(hsmall[k] + sm_inb), *outb = reinterpret_cast<uint64_t *>(hsmall[k] + sm_outb);
        for (size_t i = 0; i < m && rc == DECDS_OK; i++) {
            const size_t c = b0 + rl[i];
            uint8_t cv[K * K], inv[K * K];
            for (uint32_t a = 0; a < K; a++) std::memcpy(cv + a * K, coded_host + (c * N + sel[c * K + a]) * F, K);
            std::memset(&plans[i], 0, sizeof(RepairPlan));
            for (uint32_t a = 0; a < K; a++) plans[i].sel[a] = (uint8_t)a;
            plans[i].rank = K;
            if (!host_gf_invert(cv, inv, ctx->poly)) {  // rank 10 was just established: cannot happen
                rc = decds_set_error(DECDS_ERR_CHUNKSET_REPAIRING_FAILED, "accepted coding vectors of chunkset %zu are singular", c);
                break;
            }
            for (uint32_t r = 0; r < K; r++)  // RepairPlan::inv is input-major
                for (uint32_t q = 0; q < K; q++) plans[i].inv[q * K + r] = inv[r * K + q];
            inb[i] = reinterpret_cast<uint64_t>(dstage[k] + i * K * F);
            outb[i] = reinterpret_cast<uint64_t>(ddst[k] + rl[i] * CS);
        }
        if (rc) break;
        // the gather: one 1 MiB row per job on the host pool, overlapping the previous batches' copies
        host_parallel(m * K, [&](size_t j) {
            const size_t i = j / K, a = j % K, c = b0 + rl[i];
            std::memcpy(hstage[k] + (i * K + a) * F, coded_host + (c * N + sel[c * K + a]) * F, F);
        });
        if ((e = hipStreamWaitEvent(pp.h2d, pp.k_done[k], 0)) ||  // batch b-S's decode has read dstage[k]
            (m && (e = hipMemcpyAsync(dstage[k], hstage[k], m * K * F, hipMemcpyHostToDevice, pp.h2d))) ||
            (e = hipMemcpyAsync(dsmall[k], hsmall[k], sm_h2d, hipMemcpyHostToDevice, pp.h2d)) ||
            (e = hipEventRecord(pp.in_done[k], pp.h2d)) || (e = hipStreamWaitEvent(pp.comp, pp.in_done[k], 0)) ||
            (e = hipStreamWaitEvent(pp.comp, pp.out_done[k], 0)) ||  // batch b-S's D2H has read ddst[k], its statuses
            (e = hipMemsetAsync(dsmall[k] + sm_stat, 0, align256(batch * 4), pp.comp))) {
            rc = decds_hip_error(e, "H2D");
            break;
        }
        if (m && (e = launch_decode(ctx->geom, nullptr, F, m, dsmall[k] + sm_plan, nullptr,
                                    reinterpret_cast<int32_t *>(dsmall[k] + sm_stat),
                                    reinterpret_cast<const uint64_t *>(dsmall[k] + sm_inb),
                                    reinterpret_cast<const uint64_t *>(dsmall[k] + sm_outb), ctx->poly, ctx->marker,
                                    dsmall[k] + sm_info, pp.comp))) {
            rc = decds_hip_error(e, "rlnc decode launch");
            break;
        }
        if ((e = hipEventRecord(pp.k_done[k], pp.comp))) {
            rc = decds_hip_error(e, "hipEventRecord");
            break;
        }
        // batch b-S's statuses are read before batch b's D2H overwrites them
        if ((rc = finish(k))) break;
        ready[k] = rl;
        if ((e = hipStreamWaitEvent(pp.d2h, pp.k_done[k], 0)) ||
            (m && (e = hipMemcpyAsync(hsmall[k] + sm_stat, dsmall[k] + sm_stat, sm_bytes - sm_stat, hipMemcpyDeviceToHost,
                                      pp.d2h)))) {
            rc = decds_hip_error(e, "D2H");
            break;
        }
        // repaired data of the ready chunksets, runs of consecutive ones as one copy each; the last
        // chunkset of the blob truncated to its real size (blob.rs:464). Unready chunksets get no data.
        for (size_t c0 = 0; c0 < nb && rc == DECDS_OK;) {
            const size_t off0 = (b0 + c0) * CS;
            if (status_host[b0 + c0] != DECDS_OK) {
                std::memset(out + off0, 0, std::min(blob_len - off0, (size_t)CS));
                c0++;
                continue;
            }
            size_t c1 = c0 + 1;
            while (c1 < nb && status_host[b0 + c1] == DECDS_OK) c1++;
            const size_t len = std::min(blob_len - off0, (c1 - c0) * CS);
            if ((e = copy_d2h(out + off0, ddst[k] + c0 * CS, len, uout.pinned(), ctx->out_ring, pp.d2h)))
                rc = decds_hip_error(e, "D2H");
            c0 = c1;
        }
        if (rc) break;
        if ((e = hipEventRecord(pp.out_done[k], pp.d2h))) {
            rc = decds_hip_error(e, "hipEventRecord");
            break;
        }
        pending_b0[k] = b0;
    }
    for (int j = 0; j < S && rc == DECDS_OK; j++) rc = finish(j);  // each finish() waits on its own event
    return finish_call(ctx, pp, rc);
}

// The run form of the repair host path (DECDS_REPAIR_GATHER=0): accepted rows keep their row slots on
// the device, each run of consecutive accepted rows one hipMemcpyAsync, the device plan kernel
int repair_range_runs(decds_ctx *ctx, const uint8_t *coded_host, size_t n, const uint8_t *cand_host, size_t blob_len,
                      uint8_t *out, int32_t *status_host, size_t batch) {
    int s = decds_ctx_bind(ctx);
    if (s) return s;
    if (batch == 0) batch = 16;  // 8-32 measured best
    batch = std::min(batch, n);
    // the rank test runs on the 10-byte coding vectors on the host, so only the 10 accepted rows of
    // each chunkset cross PCIe
    std::vector<uint8_t> sel(n * K, 0);
    accept_rows(ctx, coded_host, n, cand_host, sel.data(), status_host);
    // per-slot candidate lists and device statuses in page-locked memory (tiny, per call)
    struct Pinned {
        void *p = nullptr;
        ~Pinned() {
            if (p) hip_tolerate(hipHostFree(p), "hipHostFree");
        }
    } pin;
    {
        hipError_t pe = hipHostMalloc(&pin.p, SLOTS * batch * (sizeof(decds_repair_info) + sizeof(int32_t) + N),
                                      DECDS_HOST_MALLOC_FLAGS);
        if (pe) return decds_hip_error(pe, "hipHostMalloc");
    }
    uint8_t *cand_h[SLOTS];
    int32_t *stat_h[SLOTS];
    decds_repair_info *info_h[SLOTS];
    for (int i = 0; i < SLOTS; i++) {
        info_h[i] = reinterpret_cast<decds_repair_info *>(pin.p) + i * batch;
        stat_h[i] = reinterpret_cast<int32_t *>(reinterpret_cast<uint8_t *>(pin.p) + SLOTS * batch * sizeof(decds_repair_info)) +
                    i * batch;
        cand_h[i] = reinterpret_cast<uint8_t *>(pin.p) + SLOTS * batch * (sizeof(decds_repair_info) + sizeof(int32_t)) +
                    i * batch * N;
    }
    HostUse uout(out, blob_len), uin(coded_host, n * N * F);
    std::lock_guard<std::mutex> lock(ctx->host_mu);
    uint8_t *dcoded[SLOTS], *dcand[SLOTS], *dplan[SLOTS], *dverd[SLOTS], *dstat[SLOTS], *ddst[SLOTS], *dinfo[SLOTS];
    const size_t sz[7] = {align256(batch * N * F), align256(batch * N), align256(batch * DECDS_REPAIR_PLAN_BYTES),
                          align256(batch * N), align256(batch * sizeof(int32_t)), align256(batch * CS),
                          align256(batch * sizeof(decds_repair_info))};
    const size_t per = sz[0] + sz[1] + sz[2] + sz[3] + sz[4] + sz[5] + sz[6];
    uint8_t *base;
    hipError_t e;
    if ((e = decds_ctx_scratch(ctx, SLOTS * per, &base))) return decds_hip_error(e, "hipMalloc");
    for (int i = 0; i < SLOTS; i++) {
        uint8_t **dst[7] = {&dcoded[i], &dcand[i], &dplan[i], &dverd[i], &dstat[i], &ddst[i], &dinfo[i]};
        for (int j = 0; j < 7; j++) *dst[j] = base, base += sz[j];
    }
    Pipe *ppp;
    if ((e = ctx_pipe(ctx, &ppp))) return decds_hip_error(e, "stream/event setup");
    Pipe &pp = *ppp;
    int rc = DECDS_OK;
    size_t pending_b0[SLOTS], pending_nb[SLOTS] = {};
    for (int i = 0; i < SLOTS; i++) pending_b0[i] = (size_t)-1;
    // host side of slot k once its D2H is done: a ready chunkset whose decoded data holds no boundary
    // marker is ChunksetRepairingFailed and gets no data (its region was written: clear it); one whose
    // cut (get_decoded_data, rows accepted unvalidated) falls inside the chunkset is zero past the cut
    // (blob.rs:464 truncates only: a cut past the chunkset changes nothing)
    auto finish = [&](int k) -> int {
        if (pending_b0[k] == (size_t)-1) return DECDS_OK;
        hipError_t ee = hipEventSynchronize(pp.out_done[k]);
        if (ee) return decds_hip_error(ee, "hipEventSynchronize");
        for (size_t c = 0; c < pending_nb[k]; c++) {
            const size_t cs = pending_b0[k] + c;
            if (status_host[cs] != DECDS_OK) continue;
            const size_t off = cs * CS, size = std::min(blob_len - off, (size_t)CS);
            const size_t keep = stat_h[k][c] != DECDS_OK ? 0 : std::min<size_t>(info_h[k][c].decoded_len, size);
            if (stat_h[k][c] != DECDS_OK) status_host[cs] = DECDS_ERR_CHUNKSET_REPAIRING_FAILED;
            if (keep < size) {
                if (!uout.pinned() && (ee = ctx->out_ring.flush())) return decds_hip_error(ee, "D2H (staged)");
                std::memset(out + off + keep, 0, size - keep);
            }
        }
        pending_b0[k] = (size_t)-1;
        return DECDS_OK;
    };
    const std::vector<size_t> sizes = batch_sizes(n, batch, true);
    for (size_t b0 = 0, it = 0; it < sizes.size() && rc == DECDS_OK; b0 += sizes[it], it++) {
        const int k = (int)(it % SLOTS);
        if ((rc = finish(k))) break;  // slot k's previous batch fully done: all its buffers are free
        const size_t nb = sizes[it];
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
            if ((e = copy_h2d(dcoded[k] + r0 * F, coded_host + (b0 * N + r0) * F, (r1 - r0) * F, uin.pinned(),
                              ctx->in_ring, pp.h2d)))
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
                                     ddst[k], reinterpret_cast<int32_t *>(dstat[k]),
                                     reinterpret_cast<decds_repair_info *>(dinfo[k]), pp.comp)))
            break;
        if ((e = hipEventRecord(pp.k_done[k], pp.comp)) || (e = hipStreamWaitEvent(pp.d2h, pp.k_done[k], 0)) ||
            (e = hipMemcpyAsync(stat_h[k], dstat[k], nb * sizeof(int32_t), hipMemcpyDeviceToHost, pp.d2h)) ||
            (e = hipMemcpyAsync(info_h[k], dinfo[k], nb * sizeof(decds_repair_info), hipMemcpyDeviceToHost, pp.d2h))) {
            rc = decds_hip_error(e, "D2H");
            break;
        }
        // repaired data of the ready chunksets, runs of consecutive ones as one copy each; the last
        // chunkset of the blob truncated to its real size (blob.rs:464). Unready chunksets get no data.
        for (size_t c0 = 0; c0 < nb && rc == DECDS_OK;) {
            const size_t off0 = (b0 + c0) * CS;
            if (status_host[b0 + c0] != DECDS_OK) {
                std::memset(out + off0, 0, std::min(blob_len - off0, (size_t)CS));
                c0++;
                continue;
            }
            size_t c1 = c0 + 1;
            while (c1 < nb && status_host[b0 + c1] == DECDS_OK) c1++;
            const size_t len = std::min(blob_len - off0, (c1 - c0) * CS);
            if ((e = copy_d2h(out + off0, ddst[k] + c0 * CS, len, uout.pinned(), ctx->out_ring, pp.d2h)))
                rc = decds_hip_error(e, "D2H");
            c0 = c1;
        }
        if (rc) break;
        if ((e = hipEventRecord(pp.out_done[k], pp.d2h))) {
            rc = decds_hip_error(e, "hipEventRecord");
            break;
        }
        pending_b0[k] = b0;
        pending_nb[k] = nb;
    }
    for (int j = 0; j < SLOTS && rc == DECDS_OK; j++) rc = finish(j);  // each finish() waits on its own event
    return finish_call(ctx, pp, rc);
}

int repair_range(decds_ctx *ctx, const uint8_t *coded_host, size_t n, const uint8_t *cand_host, size_t blob_len,
                 uint8_t *out, int32_t *status_host, size_t batch) {
    static const bool gather = [] {
        const char *v = std::getenv("DECDS_REPAIR_GATHER");
        return !v || std::strcmp(v, "0") != 0;
    }();
    return gather ? repair_range_gather(ctx, coded_host, n, cand_host, blob_len, out, status_host, batch)
                  : repair_range_runs(ctx, coded_host, n, cand_host, blob_len, out, status_host, batch);
}

// Runs fn(ctx_g, lo, hi) for contiguous chunkset shards [lo, hi) of [0, n), one host thread per
// context; the first failing shard's status and message are the call's.
template <class Fn>
int run_shards(decds_ctx *const *ctxs, size_t n_ctx, size_t n, Fn fn) {
    if (!ctxs || n_ctx == 0) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "no contexts");
    for (size_t g = 0; g < n_ctx; g++)
        if (!ctxs[g]) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null context %zu", g);
    const size_t per = (n + n_ctx - 1) / n_ctx;
    if (n_ctx == 1) return fn(ctxs[0], (size_t)0, n);
    std::vector<int> st(n_ctx, DECDS_OK);
    std::vector<std::string> msg(n_ctx);
    std::vector<std::thread> th;
    for (size_t g = 0; g < n_ctx; g++) {
        const size_t lo = std::min(g * per, n), hi = std::min(lo + per, n);
        if (lo == hi) continue;
        th.emplace_back([&, g, lo, hi] {
            st[g] = fn(ctxs[g], lo, hi);
            if (st[g] != DECDS_OK) msg[g] = decds_last_error();
        });
    }
    for (auto &t : th) t.join();
    for (size_t g = 0; g < n_ctx; g++)
        if (st[g] != DECDS_OK) return decds_set_error(st[g], "shard %zu: %s", g, msg[g].c_str());
    return DECDS_OK;
}

std::mutex g_rng_mu;
void random_coeffs(uint8_t *out, size_t len) {
    // the reference draws coding vectors from rand::rng() (chunkset.rs:42): OS-seeded, not reproducible
    static std::mt19937_64 g{std::random_device{}()};
    std::lock_guard<std::mutex> lk(g_rng_mu);
    for (size_t i = 0; i < len; i++) out[i] = (uint8_t)g();
}

}  // namespace

// ------------------------------------------------------------------------------------ Blob ----
struct decds_blob {
    uint64_t byte_length = 0, n = 0;
    uint8_t digest[32], root[32];
    std::vector<uint8_t> roots;      // n x 32 chunkset root commitments
    std::vector<uint8_t> cs_proofs;  // n x 16 x PROOF_SIZE x 32 chunkset-level proofs
    std::vector<uint8_t> blob_proofs;  // n x depth x 32 blob-level proofs (blob.rs:266-273)
    size_t depth = 0;
    uint8_t *coded = nullptr;        // n x 16 x F coded rows (page-locked via decds_host_alloc)
    std::vector<uint8_t> coded_vec;  // fallback storage when a page-locked allocation is refused
    ~decds_blob() {
        if (coded && coded_vec.empty()) (void)decds_host_free(coded);
    }
};

// ---------------------------------------------------------------------------- RepairingBlob ----
// Sharded over n contexts by contiguous chunkset index (shard_range, as decds_blob_new); each shard
// owns its stream, bounce rings and memory. Accepted rows (10 x F per chunkset) go to a device row
// slot while the shard is under its device budget, else to a page-locked host spill slot (the
// reference keeps them in host RAM, chunkset.rs:129-135). Decoding uses a small pool of device
// decode areas (a spilled chunkset's rows are staged there, and every decoded chunkset's 10 MiB
// output waits there until get_repaired_chunkset copies it out); an area holding a decoded but not
// yet fetched chunkset is reclaimed when needed (that chunkset is decoded again later).
namespace {
struct RbChunkset {
    uint8_t basis[K * K], piv[K];
    uint8_t cv[K][K];  // coding vectors of the accepted rows, acceptance order
    uint32_t rank = 0;
    bool repaired = false;  // get_repaired_chunkset took it (blob.rs:458-462: even if repair fails)
    bool decoded = false;   // decoded on the device into decode area `area`
    int32_t dec_status = DECDS_OK;
    uint32_t dec_len = 0;  // get_decoded_data's cut (decds_repair_info::decoded_len)
    int32_t slot = -1;   // device row slot
    int32_t hslot = -1;  // page-locked host spill slot
    int32_t area = -1;   // decode area holding its decoded bytes
};
constexpr size_t RB_SLAB_SLOTS = 8;
constexpr size_t RB_MAX_DECODE = 64;   // chunksets decoded per device batch (and decode areas per shard)
constexpr size_t RB_MAX_ROWS = 256;    // rows validated per device batch (decds_repairing_blob_add_chunks)
constexpr size_t RB_ROWS_BYTES = (K * F + 255) & ~(size_t)255;
constexpr size_t RB_OUT_BYTES = (CS + 255) & ~(size_t)255;
constexpr size_t RB_AREA_BYTES = RB_ROWS_BYTES + RB_OUT_BYTES;
constexpr size_t RB_SLAB_BYTES = RB_SLAB_SLOTS * RB_ROWS_BYTES;
// small device / pinned areas: plans, bases, statuses, valid flags
constexpr size_t RB_SM_PLAN = 0, RB_SM_INB = RB_SM_PLAN + RB_MAX_DECODE * 128, RB_SM_OUTB = RB_SM_INB + RB_MAX_DECODE * 8,
                 RB_SM_STAT = RB_SM_OUTB + RB_MAX_DECODE * 8, RB_SM_INFO = RB_SM_STAT + RB_MAX_DECODE * 4,
                 RB_SM_VALID = RB_SM_INFO + RB_MAX_DECODE * sizeof(decds_repair_info), RB_SM_BYTES = RB_SM_VALID + RB_MAX_ROWS;

struct RbShard {
    decds_ctx *ctx = nullptr;
    size_t lo = 0, hi = 0;  // chunksets [lo, hi)
    hipStream_t s = nullptr;
    BounceRing in_ring, out_ring;
    std::vector<uint8_t *> slabs, hslabs, areas;
    std::vector<int32_t> free_slots, free_hslots, free_areas;
    std::vector<int64_t> area_owner;  // chunkset whose decoded bytes area a holds, -1 = free
    size_t max_slabs = 0, max_areas = 1;  // from the device budget
    uint64_t budget = 0;
    uint8_t *d_small = nullptr, *h_small = nullptr;
    uint8_t *d_hdr = nullptr;    // chunkset roots (n x 32) + blob root (32), for decds_validate_batch
    uint8_t *d_batch = nullptr;  // RB_MAX_ROWS rows + ids + proofs + digests of one validation batch
    size_t batch_plen = 0;
    uint64_t batch_bytes = 0;

    ~RbShard() {
        if (ctx) hip_tolerate(hipSetDevice(ctx->device), "hipSetDevice");
        if (s) hip_tolerate(hipStreamSynchronize(s), "hipStreamSynchronize");
        in_ring.abandon();
        out_ring.abandon();
        for (uint8_t *p : slabs) hip_tolerate(hipFree(p), "hipFree");
        for (uint8_t *p : areas) hip_tolerate(hipFree(p), "hipFree");
        for (uint8_t *p : hslabs) host_pinned_free(p, RB_SLAB_BYTES);
        for (uint8_t *p : {d_small, d_hdr, d_batch})
            if (p) hip_tolerate(hipFree(p), "hipFree");
        if (h_small) hip_tolerate(hipHostFree(h_small), "hipHostFree");
        if (s) hip_tolerate(hipStreamDestroy(s), "hipStreamDestroy");
    }
    // device budget per context: a quarter for decode areas (at least one), the rest for row slots
    void set_budget(uint64_t bytes) {
        budget = bytes;
        max_areas = std::max<size_t>(1, std::min<size_t>(RB_MAX_DECODE, (size_t)(bytes / 4 / RB_AREA_BYTES)));
        const uint64_t rest = bytes > max_areas * RB_AREA_BYTES ? bytes - max_areas * RB_AREA_BYTES : 0;
        max_slabs = (size_t)(rest / RB_SLAB_BYTES);
    }
    uint64_t device_bytes() const {
        return slabs.size() * RB_SLAB_BYTES + areas.size() * RB_AREA_BYTES + batch_bytes + RB_SM_BYTES;
    }
    uint8_t *slot_rows(int32_t slot) const { return slabs[slot / RB_SLAB_SLOTS] + (slot % RB_SLAB_SLOTS) * RB_ROWS_BYTES; }
    uint8_t *hslot_rows(int32_t h) const { return hslabs[h / RB_SLAB_SLOTS] + (h % RB_SLAB_SLOTS) * RB_ROWS_BYTES; }
    uint8_t *area_rows(int32_t a) const { return areas[a]; }
    uint8_t *area_out(int32_t a) const { return areas[a] + RB_ROWS_BYTES; }

    // a device row slot while under budget, else a host spill slot
    int take_slot(RbChunkset &c) {
        if (c.slot >= 0 || c.hslot >= 0) return DECDS_OK;
        if (free_slots.empty() && slabs.size() < max_slabs) {
            uint8_t *p = nullptr;
            const hipError_t me = hipMalloc(reinterpret_cast<void **>(&p), RB_SLAB_BYTES);
            if (me == hipSuccess) {
                slabs.push_back(p);
                for (size_t i = RB_SLAB_SLOTS; i-- > 0;) free_slots.push_back((int32_t)((slabs.size() - 1) * RB_SLAB_SLOTS + i));
            } else {  // device memory ran out below the budget: spill from here on
                hip_tolerate(me, "hipMalloc (RepairingBlob row slab; spilling to host memory)");
                max_slabs = slabs.size();
            }
        }
        if (!free_slots.empty()) {
            c.slot = free_slots.back();
            free_slots.pop_back();
            return DECDS_OK;
        }
        if (free_hslots.empty()) {
            void *p = nullptr;
            hipError_t e = host_pinned_alloc(RB_SLAB_BYTES, &p);
            if (e) return decds_hip_error(e, "page-locked host memory for spilled rows");
            hslabs.push_back(static_cast<uint8_t *>(p));
            for (size_t i = RB_SLAB_SLOTS; i-- > 0;) free_hslots.push_back((int32_t)((hslabs.size() - 1) * RB_SLAB_SLOTS + i));
        }
        c.hslot = free_hslots.back();
        free_hslots.pop_back();
        return DECDS_OK;
    }
    void drop_slot(RbChunkset &c) {
        if (c.slot >= 0) free_slots.push_back(c.slot);
        if (c.hslot >= 0) free_hslots.push_back(c.hslot);
        c.slot = c.hslot = -1;
    }
    void drop_area(RbChunkset &c) {
        if (c.area >= 0) {
            area_owner[c.area] = -1;
            free_areas.push_back(c.area);
        }
        c.area = -1;
        c.decoded = false;
    }
    // a decode area: a free one, a new one within the budget, or (evict) one whose decoded chunkset
    // has not been fetched yet; -1 when none (*err set only when not even one area can be allocated).
    // Every get_repaired_chunkset frees the area of the chunkset it returns, so a later call always
    // finds a free one: the eviction is a guard, not a path the API's call orders reach.
    int32_t take_area(std::vector<RbChunkset> &cs, bool evict, int *err) {
        if (!free_areas.empty()) {
            const int32_t a = free_areas.back();
            free_areas.pop_back();
            return a;
        }
        if (areas.size() < max_areas) {
            uint8_t *p = nullptr;
            const hipError_t me = hipMalloc(reinterpret_cast<void **>(&p), RB_AREA_BYTES);
            if (me == hipSuccess) {
                areas.push_back(p);
                area_owner.push_back(-1);
                return (int32_t)(areas.size() - 1);
            }
            hip_tolerate(me, "hipMalloc (RepairingBlob decode area; reusing the areas held)");
            max_areas = std::max<size_t>(1, areas.size());
            if (areas.empty()) {
                *err = decds_set_error(DECDS_ERR_OUT_OF_DEVICE_MEMORY,
                                       "device %d has no memory left for a %zu-byte decode area", ctx->device, RB_AREA_BYTES);
                return -1;
            }
        }
        if (!evict) return -1;
        for (size_t a = 0; a < areas.size(); a++) {
            const int64_t o = area_owner[a];
            if (o >= 0) {
                cs[o].area = -1;
                cs[o].decoded = false;  // decoded again when asked for
                area_owner[a] = -1;
                return (int32_t)a;
            }
        }
        return -1;
    }
    // decode `first` and further ready, undecoded chunksets of this shard for which a decode area is
    // free, in one launch (the decode kernel's gather form)
    int decode_ready(std::vector<RbChunkset> &cs, size_t first) {
        int err = DECDS_OK;
        std::vector<size_t> todo;
        std::vector<int32_t> area;
        const int32_t a0 = take_area(cs, true, &err);
        if (a0 < 0) return err ? err : decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "no decode area");
        todo.push_back(first);
        area.push_back(a0);
        for (size_t c = lo; c < hi && todo.size() < RB_MAX_DECODE; c++) {
            if (c == first || cs[c].rank != K || cs[c].decoded || cs[c].repaired) continue;
            int e2 = DECDS_OK;
            const int32_t a = take_area(cs, false, &e2);
            if (a < 0) break;
            todo.push_back(c);
            area.push_back(a);
        }
        const size_t m = todo.size();
        RepairPlan *plans = reinterpret_cast<RepairPlan *>(h_small + RB_SM_PLAN);
        uint64_t *inb = reinterpret_cast<uint64_t *>(h_small + RB_SM_INB), *outb = reinterpret_cast<uint64_t *>(h_small + RB_SM_OUTB);
        hipError_t e;
        int st = DECDS_OK;
        for (size_t i = 0; i < m; i++) {  // every area taken is owned before anything can fail
            cs[todo[i]].area = area[i];
            area_owner[area[i]] = (int64_t)todo[i];
        }
        for (size_t i = 0; i < m && st == DECDS_OK; i++) {
            RbChunkset &c = cs[todo[i]];
            std::memset(&plans[i], 0, sizeof(RepairPlan));
            for (uint32_t k = 0; k < K; k++) plans[i].sel[k] = (uint8_t)k;
            plans[i].rank = K;
            uint8_t inv[K * K];
            if (!host_gf_invert(&c.cv[0][0], inv, ctx->poly)) {
                st = decds_set_error(DECDS_ERR_CHUNKSET_REPAIRING_FAILED, "accepted coding vectors are singular");
                break;
            }
            for (uint32_t r = 0; r < K; r++)  // RepairPlan::inv is input-major
                for (uint32_t k = 0; k < K; k++) plans[i].inv[k * K + r] = inv[r * K + k];
            if (c.slot >= 0) {
                inb[i] = reinterpret_cast<uint64_t>(slot_rows(c.slot));
            } else {  // spilled: stage its rows into the area (page-locked host memory: direct DMA)
                if ((e = hipMemcpyAsync(area_rows(area[i]), hslot_rows(c.hslot), K * F, hipMemcpyHostToDevice, s)))
                    st = decds_hip_error(e, "H2D (spilled rows)");
                inb[i] = reinterpret_cast<uint64_t>(area_rows(area[i]));
            }
            outb[i] = reinterpret_cast<uint64_t>(area_out(area[i]));
        }
        if (st == DECDS_OK) {
            if ((e = hipMemcpyAsync(d_small, h_small, RB_SM_STAT, hipMemcpyHostToDevice, s)) ||
                (e = hipMemsetAsync(d_small + RB_SM_STAT, 0, m * 4, s)))
                st = decds_hip_error(e, "H2D (plans)");
        }
        if (st == DECDS_OK &&
            (e = launch_decode(ctx->geom, nullptr, F, m, d_small + RB_SM_PLAN, nullptr,
                               reinterpret_cast<int32_t *>(d_small + RB_SM_STAT), reinterpret_cast<const uint64_t *>(d_small + RB_SM_INB),
                               reinterpret_cast<const uint64_t *>(d_small + RB_SM_OUTB), ctx->poly, ctx->marker,
                               d_small + RB_SM_INFO, s)))
            st = decds_hip_error(e, "rlnc_decode_kernel launch");
        if (st == DECDS_OK &&
            ((e = hipMemcpyAsync(h_small + RB_SM_STAT, d_small + RB_SM_STAT, RB_SM_VALID - RB_SM_STAT, hipMemcpyDeviceToHost, s)) ||
             (e = hipStreamSynchronize(s))))
            st = decds_hip_error(e, "D2H (statuses)");
        if (st != DECDS_OK) {
            for (size_t i = 0; i < m; i++) drop_area(cs[todo[i]]);
            return st;
        }
        const int32_t *stat = reinterpret_cast<const int32_t *>(h_small + RB_SM_STAT);
        const decds_repair_info *info = reinterpret_cast<const decds_repair_info *>(h_small + RB_SM_INFO);
        for (size_t i = 0; i < m; i++) {
            cs[todo[i]].decoded = true;
            cs[todo[i]].dec_status = stat[i];
            cs[todo[i]].dec_len = info[i].decoded_len;
        }
        return DECDS_OK;
    }
};
}  // namespace

struct decds_repairing_blob {
    uint64_t byte_length = 0, n = 0, per = 1;
    uint8_t root[32];
    std::vector<uint8_t> cs_roots;
    std::vector<RbChunkset> cs;
    std::vector<RbShard *> shards;
    ~decds_repairing_blob() {
        for (RbShard *sh : shards) delete sh;
    }
    RbShard &shard_of(uint64_t c) { return *shards[c / per]; }
    size_t chunkset_size(size_t c) const {  // BlobHeader::get_chunkset_size (blob.rs:84-94)
        const uint64_t from = c * CS;
        return (size_t)(std::min<uint64_t>(from + CS, byte_length) - from);
    }
    // the routing checks of RepairingBlob::add_chunk that precede validation (blob.rs:374-381)
    int route_check(uint64_t cs_id) {
        if (cs_id >= n)
            return decds_set_error(DECDS_ERR_INVALID_CHUNKSET_ID, "invalid chunkset id: %llu (num_chunksets: %llu)",
                                   (unsigned long long)cs_id, (unsigned long long)n);
        if (cs[cs_id].repaired)
            return decds_set_error(DECDS_ERR_CHUNKSET_ALREADY_REPAIRED, "chunkset %llu is already repaired",
                                   (unsigned long long)cs_id);
        return DECDS_OK;
    }
    // after validation (blob.rs:383-388): ready check, then add_chunk_unvalidated's rank step
    // (chunkset.rs:177-183). On success the row's coding vector is recorded and its slot row index
    // (rank - 1) returned through *row; the caller then stores the row (store_row).
    int accept(uint64_t cs_id, const uint8_t *cv, size_t len, uint32_t *row) {
        RbChunkset &c = cs[cs_id];
        if (c.rank == K)
            return decds_set_error(DECDS_ERR_CHUNKSET_READY_TO_REPAIR, "chunkset %llu is ready to repair",
                                   (unsigned long long)cs_id);
        if (len != F)
            return decds_set_error(DECDS_ERR_CHUNK_DECODING_FAILED,
                                   "decoding chunk for chunkset %llu failed: invalid piece length %zu",
                                   (unsigned long long)cs_id, len);
        RbShard &sh = shard_of(cs_id);
        // the rank step on a copy: a slot is taken only for a useful piece, and a failed slot
        // allocation leaves the chunkset as it was
        uint8_t basis[K * K], piv[K];
        uint32_t rank = c.rank;
        std::memcpy(basis, c.basis, sizeof(basis));
        std::memcpy(piv, c.piv, sizeof(piv));
        if (!decds_rank_push(basis, piv, &rank, cv, sh.ctx->poly))
            return decds_set_error(DECDS_ERR_CHUNK_DECODING_FAILED,
                                   "decoding chunk for chunkset %llu failed: received piece is not useful",
                                   (unsigned long long)cs_id);
        int s = sh.take_slot(c);
        if (s) return s;
        std::memcpy(c.basis, basis, sizeof(basis));
        std::memcpy(c.piv, piv, sizeof(piv));
        c.rank = rank;
        std::memcpy(c.cv[c.rank - 1], cv, K);
        *row = c.rank - 1;
        return DECDS_OK;
    }
};

extern "C" {

int decds_blob_encode_host(decds_ctx *ctx, const uint8_t *blob, size_t blob_len, const uint8_t *coeffs_host,
                           uint8_t *coded_host, size_t batch) {
    if (blob_len == 0) return decds_set_error(DECDS_ERR_EMPTY_DATA_FOR_BLOB, "empty data for blob");  // blob.rs:245-247
    if (!blob || !coeffs_host || !coded_host) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null buffer");
    return encode_range(ctx, blob, blob_len, coeffs_host, coded_host, batch, nullptr);
}

int decds_blob_encode_host_multi(decds_ctx *const *ctxs, size_t n_ctx, const uint8_t *blob, size_t blob_len,
                                 const uint8_t *coeffs_host, uint8_t *coded_host, size_t batch) {
    if (blob_len == 0) return decds_set_error(DECDS_ERR_EMPTY_DATA_FOR_BLOB, "empty data for blob");
    if (!blob || !coeffs_host || !coded_host) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null buffer");
    const size_t n = (blob_len + CS - 1) / CS;
    return run_shards(ctxs, n_ctx, n, [&](decds_ctx *ctx, size_t lo, size_t hi) {
        const size_t len = std::min<uint64_t>(blob_len, hi * CS) - lo * CS;
        return encode_range(ctx, blob + lo * CS, len, coeffs_host + lo * N * K, coded_host + lo * N * F, batch, nullptr);
    });
}

static int check_repair_args(const uint8_t *coded_host, size_t n, const uint8_t *cand_host, size_t blob_len,
                             const uint8_t *out, const int32_t *status_host) {
    if (!coded_host || !cand_host || !out || !status_host || n == 0)
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null buffer or no chunksets");
    if (blob_len > n * CS || blob_len <= (n - 1) * CS)
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "blob length %zu inconsistent with %zu chunksets", blob_len, n);
    return DECDS_OK;
}

int decds_blob_repair_host(decds_ctx *ctx, const uint8_t *coded_host, size_t n, const uint8_t *cand_host,
                           size_t blob_len, uint8_t *out, int32_t *status_host, size_t batch) {
    int s = check_repair_args(coded_host, n, cand_host, blob_len, out, status_host);
    if (s) return s;
    return repair_range(ctx, coded_host, n, cand_host, blob_len, out, status_host, batch);
}

int decds_blob_repair_host_multi(decds_ctx *const *ctxs, size_t n_ctx, const uint8_t *coded_host, size_t n,
                                 const uint8_t *cand_host, size_t blob_len, uint8_t *out, int32_t *status_host,
                                 size_t batch) {
    int s = check_repair_args(coded_host, n, cand_host, blob_len, out, status_host);
    if (s) return s;
    return run_shards(ctxs, n_ctx, n, [&](decds_ctx *ctx, size_t lo, size_t hi) {
        const size_t len = std::min<uint64_t>(blob_len, hi * CS) - lo * CS;
        return repair_range(ctx, coded_host + lo * N * F, hi - lo, cand_host + lo * N, len, out + lo * CS,
                            status_host + lo, batch);
    });
}

// ---- Blob -------------------------------------------------------------------------------------
int decds_blob_new(decds_ctx *const *ctxs, size_t n_ctx, const uint8_t *data, size_t len, const uint8_t *coeffs,
                   decds_blob **out) {
    if (!out) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null out pointer");
    *out = nullptr;
    if (len == 0) return decds_set_error(DECDS_ERR_EMPTY_DATA_FOR_BLOB, "empty data for blob");  // blob.rs:245-247
    if (!data) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null data");
    if (!ctxs || n_ctx == 0) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "no contexts");
    auto *b = new decds_blob;
    b->byte_length = len;
    b->n = (len + CS - 1) / CS;  // blob.rs:252
    const size_t n = b->n;
    std::vector<uint8_t> cv;
    if (!coeffs) {
        cv.resize(n * N * K);
        random_coeffs(cv.data(), cv.size());
        coeffs = cv.data();
    }
    void *p = nullptr;
    if (decds_host_alloc(n * N * F, &p) == DECDS_OK) {
        b->coded = static_cast<uint8_t *>(p);
    } else {  // page-locked memory refused: plain memory, staged copies
        b->coded_vec.resize(n * N * F);
        b->coded = b->coded_vec.data();
    }
    b->roots.resize(n * 32);
    b->cs_proofs.resize(n * N * PROOF_SIZE * 32);
    // blob.rs:249 whole-blob BLAKE3. Above 1 MiB: the full 1 MiB groups' subtree values on the device,
    // from the inputs each batch uploads anyway (blob_group_kernel, 1024 chunks per workgroup), the last
    // partial group's on the host, and the host folds them (round 6; until then 16 host threads hashed
    // the whole blob beside the device pipeline, competing with its staging copies for the CPUs). Up to
    // 1 MiB: on the host.
    static const bool host_digest = [] {  // DECDS_BLOB_DIGEST=host: the whole digest on host threads (A/B)
        const char *v = std::getenv("DECDS_BLOB_DIGEST");
        return v && !std::strcmp(v, "host");
    }();
    const size_t full_groups = len > BLOB_GROUP && !host_digest ? len / BLOB_GROUP : 0;
    const bool part = full_groups && len % BLOB_GROUP;
    std::vector<uint32_t> gcv((full_groups + part) * 8);
    std::thread dig([&] {
        const unsigned hw = std::thread::hardware_concurrency();
        const int th = (int)std::min(16u, hw ? hw : 4u);
        if (!full_groups)
            decds_blake3_parallel(data, len, b->digest, th);
        else if (part)
            blake3_subtree_cv(data + full_groups * BLOB_GROUP, len - full_groups * BLOB_GROUP, full_groups * (BLOB_GROUP / 1024),
                              &gcv[full_groups * 8], th);
    });
    int s = run_shards(ctxs, n_ctx, n, [&](decds_ctx *ctx, size_t lo, size_t hi) {
        const size_t l = std::min<uint64_t>(len, hi * CS) - lo * CS;
        const CommitOut cm{b->roots.data() + lo * 32, b->cs_proofs.data() + lo * N * PROOF_SIZE * 32, lo,
                           full_groups ? reinterpret_cast<uint8_t *>(&gcv[lo * (CS / BLOB_GROUP) * 8]) : nullptr};
        return encode_range(ctx, data + lo * CS, l, coeffs + lo * N * K, b->coded + lo * N * F, 0, &cm);
    });
    dig.join();
    if (s) {
        delete b;
        return s;
    }
    if (full_groups)
        blake3_fold_root(reinterpret_cast<const uint32_t(*)[8]>(gcv.data()), full_groups + part, b->digest);
    // blob.rs:266-273: Merkle tree over the chunkset roots; every chunk carries its chunkset's path
    int depth = 0;
    while (((size_t)1 << depth) < n) depth++;
    b->depth = (size_t)depth;
    b->blob_proofs.resize(std::max<size_t>(1, n * b->depth * 32));
    if ((s = decds_merkle_tree(b->roots.data(), n, b->root, b->blob_proofs.data())) < 0) {
        delete b;
        return s;
    }
    *out = b;
    return DECDS_OK;
}

int decds_blob_get_header(const decds_blob *b, uint64_t *byte_length, uint64_t *num_chunksets, uint8_t *digest,
                          uint8_t *root, const uint8_t **chunkset_roots) {
    if (!b) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null blob");
    if (byte_length) *byte_length = b->byte_length;
    if (num_chunksets) *num_chunksets = b->n;
    if (digest) std::memcpy(digest, b->digest, 32);
    if (root) std::memcpy(root, b->root, 32);
    if (chunkset_roots) *chunkset_roots = b->roots.data();
    return DECDS_OK;
}

size_t decds_blob_proof_len(const decds_blob *b) { return b ? PROOF_SIZE + b->depth : 0; }

int decds_blob_get_chunk(const decds_blob *b, size_t chunkset_id, size_t share_id, const uint8_t **data,
                         uint8_t *proof, size_t proof_cap) {
    if (!b) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null blob");
    if (share_id >= N)
        return decds_set_error(DECDS_ERR_INVALID_SHARE_ID, "invalid erasure coded share id: %zu (num_shares: %u)", share_id, N);
    if (chunkset_id >= b->n)
        return decds_set_error(DECDS_ERR_INVALID_CHUNKSET_ID, "invalid chunkset id: %zu (num_chunksets: %llu)", chunkset_id,
                               (unsigned long long)b->n);
    if (data) *data = b->coded + (chunkset_id * N + share_id) * F;
    if (proof) {
        const size_t plen = PROOF_SIZE + b->depth;
        if (proof_cap < plen * 32) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "proof buffer < %zu", plen * 32);
        std::memcpy(proof, &b->cs_proofs[(chunkset_id * N + share_id) * PROOF_SIZE * 32], PROOF_SIZE * 32);
        if (b->depth) std::memcpy(proof + PROOF_SIZE * 32, &b->blob_proofs[chunkset_id * b->depth * 32], b->depth * 32);
    }
    return DECDS_OK;
}

int decds_blob_get_share(const decds_blob *b, size_t share_id, uint8_t *data, size_t data_cap, uint8_t *proofs,
                         size_t proofs_cap) {
    if (!b) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null blob");
    if (share_id >= N)  // blob.rs:307-309
        return decds_set_error(DECDS_ERR_INVALID_SHARE_ID, "invalid erasure coded share id: %zu (num_shares: %u)", share_id, N);
    const size_t plen = PROOF_SIZE + b->depth;
    if ((data && data_cap < b->n * F) || (proofs && proofs_cap < b->n * plen * 32))
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "output buffers too small");
    for (size_t c = 0; c < b->n; c++) {
        const uint8_t *d;
        int s = decds_blob_get_chunk(b, c, share_id, &d, proofs ? proofs + c * plen * 32 : nullptr, plen * 32);
        if (s) return s;
        if (data) std::memcpy(data + c * F, d, F);
    }
    return DECDS_OK;
}

void decds_blob_free(decds_blob *b) { delete b; }

// ---- RepairingBlob ----------------------------------------------------------------------------
static uint64_t rb_default_budget(decds_ctx *const *ctxs, size_t n_ctx, size_t g) {
    // DECDS_RB_DEVICE_MB, else half the device's free memory shared by the shards on that device
    if (const char *env = getenv("DECDS_RB_DEVICE_MB")) return (uint64_t)strtoull(env, nullptr, 10) << 20;
    size_t fr = 0, total = 0;
    if (const hipError_t me = hipMemGetInfo(&fr, &total)) {
        hip_tolerate(me, "hipMemGetInfo (RepairingBlob default budget: 4 GiB)");
        return (uint64_t)4 << 30;
    }
    size_t same = 0;
    for (size_t k = 0; k < n_ctx; k++) same += ctxs[k]->device == ctxs[g]->device;
    return (uint64_t)fr / 2 / std::max<size_t>(1, same);
}

int decds_repairing_blob_new_multi(decds_ctx *const *ctxs, size_t n_ctx, uint64_t byte_length, uint64_t num_chunksets,
                                   const uint8_t *root, const uint8_t *chunkset_roots, decds_repairing_blob **out) {
    if (!out) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null out pointer");
    *out = nullptr;
    if (!ctxs || n_ctx == 0) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "no contexts");
    for (size_t g = 0; g < n_ctx; g++)
        if (!ctxs[g]) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null context %zu", g);
    if (!root || (num_chunksets && !chunkset_roots) || num_chunksets == 0)
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null header field or no chunksets");
    if (byte_length > num_chunksets * CS || byte_length <= (num_chunksets - 1) * CS)
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "blob length %llu inconsistent with %llu chunksets",
                               (unsigned long long)byte_length, (unsigned long long)num_chunksets);
    auto *rb = new decds_repairing_blob;
    rb->byte_length = byte_length;
    rb->n = num_chunksets;
    // the contiguous chunkset-index plan of decds_blob_new / run_shards
    rb->per = (num_chunksets + n_ctx - 1) / n_ctx;
    std::memcpy(rb->root, root, 32);
    rb->cs_roots.assign(chunkset_roots, chunkset_roots + num_chunksets * 32);
    rb->cs.resize(num_chunksets);
    for (size_t g = 0; g * rb->per < num_chunksets; g++) {
        auto *sh = new RbShard;
        rb->shards.push_back(sh);
        sh->ctx = ctxs[g];
        sh->lo = g * rb->per;
        sh->hi = std::min<uint64_t>(sh->lo + rb->per, num_chunksets);
        int st = decds_ctx_bind(sh->ctx);
        if (st) {
            delete rb;
            return st;
        }
        sh->set_budget(rb_default_budget(ctxs, n_ctx, g));
        hipError_t e;
        if ((e = hipStreamCreateWithFlags(&sh->s, hipStreamNonBlocking)) ||
            (e = hipMalloc(reinterpret_cast<void **>(&sh->d_small), RB_SM_BYTES)) ||
            (e = hipHostMalloc(reinterpret_cast<void **>(&sh->h_small), RB_SM_BYTES, DECDS_HOST_MALLOC_FLAGS)) ||
            (e = hipMalloc(reinterpret_cast<void **>(&sh->d_hdr), (num_chunksets + 1) * 32)) ||
            (e = hipMemcpyAsync(sh->d_hdr, chunkset_roots, num_chunksets * 32, hipMemcpyHostToDevice, sh->s)) ||
            (e = hipMemcpyAsync(sh->d_hdr + num_chunksets * 32, root, 32, hipMemcpyHostToDevice, sh->s)) ||
            (e = hipStreamSynchronize(sh->s))) {
            delete rb;
            return decds_hip_error(e, "RepairingBlob setup");
        }
    }
    *out = rb;
    return DECDS_OK;
}

int decds_repairing_blob_new(decds_ctx *ctx, uint64_t byte_length, uint64_t num_chunksets, const uint8_t *root,
                             const uint8_t *chunkset_roots, decds_repairing_blob **out) {
    decds_ctx *const ctxs[1] = {ctx};
    return decds_repairing_blob_new_multi(ctxs, 1, byte_length, num_chunksets, root, chunkset_roots, out);
}

int decds_repairing_blob_set_device_budget(decds_repairing_blob *rb, uint64_t bytes_per_context) {
    if (!rb) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null repairing blob");
    for (RbShard *sh : rb->shards) sh->set_budget(bytes_per_context);
    return DECDS_OK;
}

int decds_repairing_blob_memory(const decds_repairing_blob *rb, uint64_t *stats, size_t n_stats) {
    if (!rb || !stats) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null argument");
    uint64_t v[6] = {0, 0, 0, 0, 0, (uint64_t)rb->shards.size()};
    for (const RbShard *sh : rb->shards) {
        v[0] += sh->device_bytes();
        v[3] += sh->hslabs.size() * RB_SLAB_BYTES;
        v[4] += sh->areas.size();
    }
    for (const RbChunkset &c : rb->cs) {
        v[1] += c.slot >= 0;
        v[2] += c.hslot >= 0;
    }
    for (size_t i = 0; i < n_stats && i < 6; i++) stats[i] = v[i];
    return DECDS_OK;
}

int decds_repairing_blob_add_chunk(decds_repairing_blob *rb, uint64_t chunkset_id, uint64_t chunk_id,
                                   const uint8_t *data, size_t len, const uint8_t *proof, size_t proof_len) {
    if (!rb) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null repairing blob");
    int s = rb->route_check(chunkset_id);
    if (s) return s;
    RbShard &sh = rb->shard_of(chunkset_id);
    // BlobHeader::validate_chunk (blob.rs:211-215): blob-level proof at the global chunk id, the
    // chunkset id in range, then the first 4 hashes against the chunkset root (chunk.rs:88-110)
    bool ok = proof && proof_len >= PROOF_SIZE && (data || len == 0);
    if ((s = decds_ctx_bind(sh.ctx))) return s;
    // a full-length row is copied while it is hashed: into a staging piece (sent to the device only if
    // the chunk is accepted into a device slot), or, for a chunkset whose rows are spilled, straight
    // into the host slot row it would take (rank unchanged on rejection: the row is simply reused);
    // the caller's buffer is free on return
    int piece = -1;
    uint8_t *staged = nullptr, *direct = nullptr;
    {
        const RbChunkset &cc = rb->cs[chunkset_id];
        if (cc.hslot >= 0 && cc.rank < K) direct = sh.hslot_rows(cc.hslot) + cc.rank * F;
    }
    if (ok) {
        uint8_t leaf[32];
        if (len == F && b3h::simd_available()) {
            hipError_t e = direct ? hipSuccess : sh.in_ring.stage(&piece, &staged);
            if (e) return decds_hip_error(e, "staging piece");
            uint8_t *const to = direct ? direct : staged;
            constexpr size_t HALF = (F + 1) / 2;
            const std::function<void(size_t)> copy = [&](size_t h) {
                std::memcpy(to + h * HALF, data + h * HALF, h ? F - HALF : HALF);
            };
            full_piece_digest(chunkset_id, chunk_id, data, leaf, &copy, 2);
        } else {
            decds_chunk_digest(chunkset_id, chunk_id, data, len, leaf);
        }
        ok = decds_merkle_verify(chunk_id, leaf, proof, proof_len, rb->root) == 1 &&
             decds_merkle_verify(chunk_id % N, leaf, proof, PROOF_SIZE, &rb->cs_roots[chunkset_id * 32]) == 1;
    }
    if (!ok)
        return decds_set_error(DECDS_ERR_INVALID_PROOF_IN_CHUNK, "invalid proof in chunk of chunkset %llu",
                               (unsigned long long)chunkset_id);
    uint32_t row;
    if ((s = rb->accept(chunkset_id, data, len, &row))) return s;
    const RbChunkset &c = rb->cs[chunkset_id];
    if (c.hslot >= 0) {  // spilled: the row stays in page-locked host memory until its decode
        uint8_t *dst = sh.hslot_rows(c.hslot) + row * F;
        const bool copied = dst == direct && len == F && b3h::simd_available();  // during the hashing
        if (!copied) par_memcpy(dst, staged ? staged : data, F);
        return DECDS_OK;
    }
    uint8_t *dst = sh.slot_rows(c.slot) + row * F;
    hipError_t e = staged ? sh.in_ring.commit(piece, dst, F, sh.s) : sh.in_ring.h2d(dst, data, F, sh.s);
    return e ? decds_hip_error(e, "H2D (accepted row)") : DECDS_OK;
}

// decds_repairing_blob_add_chunks for the rows `idx` (arrival order) of one shard
static int rb_add_rows_shard(decds_repairing_blob *rb, RbShard &sh, const std::vector<size_t> &idx, const uint64_t *ids,
                             const uint8_t *rows, const uint8_t *proofs, size_t proof_len, int32_t *status) {
    int s = decds_ctx_bind(sh.ctx);
    if (s) return s;
    const size_t P = proof_len * 32;
    // device batch area: RB_MAX_ROWS rows | ids | proofs (sized for the longest proof seen) | digests
    hipError_t e;
    if (!sh.d_batch || sh.batch_plen < proof_len) {
        if (sh.d_batch) {
            hip_tolerate(hipStreamSynchronize(sh.s), "hipStreamSynchronize");
            hip_tolerate(hipFree(sh.d_batch), "hipFree");
            sh.d_batch = nullptr;
            sh.batch_bytes = 0;
        }
        const size_t total = RB_MAX_ROWS * (F + 16 + P + 32);
        if ((e = hipMalloc(reinterpret_cast<void **>(&sh.d_batch), total))) {
            (void)hipGetLastError();
            return decds_set_error(DECDS_ERR_OUT_OF_DEVICE_MEMORY, "device %d has no memory left for a %zu-byte "
                                   "validation batch", sh.ctx->device, total);
        }
        sh.batch_plen = proof_len;
        sh.batch_bytes = total;
    }
    const size_t a_ids = RB_MAX_ROWS * F, a_prf = a_ids + RB_MAX_ROWS * 16, a_dig = a_prf + RB_MAX_ROWS * sh.batch_plen * 32;
    const size_t n_rows = idx.empty() ? 0 : idx.back() + 1;
    HostUse urows(rows, n_rows * F), uids(ids, n_rows * 16), uprf(proofs, n_rows * P);
    for (size_t r0 = 0; r0 < idx.size(); r0 += RB_MAX_ROWS) {
        const size_t m = std::min(RB_MAX_ROWS, idx.size() - r0);
        // the batch's rows, ids and proofs, copied in runs of consecutive arrival indices
        for (size_t i = 0; i < m;) {
            size_t j = i + 1;
            while (j < m && idx[r0 + j] == idx[r0 + j - 1] + 1) j++;
            const size_t a = idx[r0 + i], len = j - i;
            if ((e = copy_h2d(sh.d_batch + i * F, rows + a * F, len * F, urows.pinned(), sh.in_ring, sh.s)) ||
                (e = copy_h2d(sh.d_batch + a_ids + i * 16, reinterpret_cast<const uint8_t *>(ids + 2 * a), len * 16,
                              uids.pinned(), sh.in_ring, sh.s)) ||
                (P && (e = copy_h2d(sh.d_batch + a_prf + i * P, proofs + a * P, len * P, uprf.pinned(), sh.in_ring, sh.s))))
                return decds_hip_error(e, "H2D (rows)");
            i = j;
        }
        // BlobHeader::validate_chunk for the whole batch on the device (one digest per row, both proofs)
        if ((s = decds_validate_batch(sh.ctx, sh.d_batch, F, m, reinterpret_cast<const uint64_t *>(sh.d_batch + a_ids),
                                      sh.d_batch + a_prf, proof_len, sh.d_hdr, rb->n, sh.d_hdr + rb->n * 32,
                                      sh.d_batch + a_dig, sh.d_small + RB_SM_VALID, sh.s)))
            return s;
        if ((e = hipMemcpyAsync(sh.h_small + RB_SM_VALID, sh.d_small + RB_SM_VALID, m, hipMemcpyDeviceToHost, sh.s)) ||
            (e = hipStreamSynchronize(sh.s)))
            return decds_hip_error(e, "D2H (verdicts)");
        // RepairingBlob::add_chunk's checks in arrival order (blob.rs:373-394)
        for (size_t i = 0; i < m; i++) {
            const size_t a = idx[r0 + i];
            const uint64_t cid = ids[2 * a];
            int st = rb->route_check(cid);
            if (st == DECDS_OK && !sh.h_small[RB_SM_VALID + i])
                st = decds_set_error(DECDS_ERR_INVALID_PROOF_IN_CHUNK, "invalid proof in chunk of chunkset %llu",
                                     (unsigned long long)cid);
            uint32_t row = 0;
            if (st == DECDS_OK) st = rb->accept(cid, rows + a * F, F, &row);
            if (st == DECDS_OK) {
                const RbChunkset &c = rb->cs[cid];
                if (c.hslot >= 0)
                    par_memcpy(sh.hslot_rows(c.hslot) + row * F, rows + a * F, F);
                else if ((e = hipMemcpyAsync(sh.slot_rows(c.slot) + row * F, sh.d_batch + i * F, F, hipMemcpyDeviceToDevice,
                                             sh.s)))
                    return decds_hip_error(e, "D2D (accepted row)");
            }
            status[a] = st;
        }
    }
    if ((e = hipStreamSynchronize(sh.s))) return decds_hip_error(e, "hipStreamSynchronize");
    return DECDS_OK;
}

int decds_repairing_blob_add_chunks(decds_repairing_blob *rb, size_t n_rows, const uint64_t *ids, const uint8_t *rows,
                                    const uint8_t *proofs, size_t proof_len, int32_t *status) {
    if (!rb || (n_rows && (!ids || !rows || !status))) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null argument");
    if (n_rows && proof_len && !proofs) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null proofs");
    // rows go to the shard of their claimed chunkset (the reference routes by the chunk's own id,
    // blob.rs:376); an id out of range is refused here, before validation, as blob.rs:374-377
    std::vector<std::vector<size_t>> part(rb->shards.size());
    for (size_t a = 0; a < n_rows; a++) {
        const uint64_t cid = ids[2 * a];
        if (cid >= rb->n)
            status[a] = rb->route_check(cid);
        else
            part[cid / rb->per].push_back(a);
    }
    std::vector<int> st(rb->shards.size(), DECDS_OK);
    std::vector<std::string> msg(rb->shards.size());
    std::vector<std::thread> th;
    size_t busy = 0;
    for (size_t g = 0; g < part.size(); g++) busy += !part[g].empty();
    for (size_t g = 0; g < part.size(); g++) {
        if (part[g].empty()) continue;
        auto run = [&, g] {
            st[g] = rb_add_rows_shard(rb, *rb->shards[g], part[g], ids, rows, proofs, proof_len, status);
            if (st[g] != DECDS_OK) msg[g] = decds_last_error();
        };
        if (busy == 1)
            run();
        else
            th.emplace_back(run);
    }
    for (auto &t : th) t.join();
    for (size_t g = 0; g < part.size(); g++)
        if (st[g] != DECDS_OK) return busy == 1 ? st[g] : decds_set_error(st[g], "shard %zu: %s", g, msg[g].c_str());
    return DECDS_OK;
}

int decds_repairing_blob_is_chunkset_ready_to_repair(const decds_repairing_blob *rb, size_t chunkset_id, int *out) {
    if (!rb || !out) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null argument");
    if (chunkset_id >= rb->n)  // blob.rs:407-414
        return decds_set_error(DECDS_ERR_INVALID_CHUNKSET_ID, "invalid chunkset id: %zu (num_chunksets: %llu)", chunkset_id,
                               (unsigned long long)rb->n);
    *out = !rb->cs[chunkset_id].repaired && rb->cs[chunkset_id].rank == K;
    return DECDS_OK;
}

int decds_repairing_blob_is_chunkset_already_repaired(const decds_repairing_blob *rb, size_t chunkset_id, int *out) {
    if (!rb || !out) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null argument");
    if (chunkset_id >= rb->n)  // blob.rs:424-430
        return decds_set_error(DECDS_ERR_INVALID_CHUNKSET_ID, "invalid chunkset id: %zu (num_chunksets: %llu)", chunkset_id,
                               (unsigned long long)rb->n);
    *out = rb->cs[chunkset_id].repaired;
    return DECDS_OK;
}

int decds_repairing_blob_get_repaired_chunkset(decds_repairing_blob *rb, size_t chunkset_id, uint8_t *out,
                                               size_t out_cap, size_t *out_len) {
    if (!rb) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null repairing blob");
    // blob.rs:451-473: id check, already repaired, not yet ready, then the chunkset is consumed
    if (chunkset_id >= rb->n)
        return decds_set_error(DECDS_ERR_INVALID_CHUNKSET_ID, "invalid chunkset id: %zu (num_chunksets: %llu)", chunkset_id,
                               (unsigned long long)rb->n);
    RbChunkset &c = rb->cs[chunkset_id];
    if (c.repaired) return decds_set_error(DECDS_ERR_CHUNKSET_ALREADY_REPAIRED, "chunkset %zu is already repaired", chunkset_id);
    if (c.rank != K) return decds_set_error(DECDS_ERR_CHUNKSET_NOT_YET_READY, "chunkset %zu is not ready to repair", chunkset_id);
    const size_t size = rb->chunkset_size(chunkset_id);
    if (!out || out_cap < size) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "out buffer < %zu", size);
    RbShard &sh = rb->shard_of(chunkset_id);
    int s = decds_ctx_bind(sh.ctx);
    if (s) return s;
    if (!c.decoded && (s = sh.decode_ready(rb->cs, chunkset_id))) return s;
    c.repaired = true;  // blob.rs:458-462 takes the decoder out before repairing
    if (c.dec_status != DECDS_OK) {
        sh.drop_area(c);
        sh.drop_slot(c);
        return decds_set_error(DECDS_ERR_CHUNKSET_REPAIRING_FAILED, "chunkset %zu repairing failed: RLNC Decoding error: %s",
                               chunkset_id, "invalid decoded data format");
    }
    // get_decoded_data's vector (cut at the last boundary marker: CS for any validated chunk set,
    // the decode kernels' tail_scan_decoded) truncated to the chunkset's real size (blob.rs:464 truncates only)
    const size_t len = std::min<size_t>(size, c.dec_len);
    HostUse uo(out, len);
    hipError_t e;
    if ((e = copy_d2h(out, sh.area_out(c.area), len, uo.pinned(), sh.out_ring, sh.s)) || (e = sh.out_ring.flush()) ||
        (e = hipStreamSynchronize(sh.s))) {
        sh.out_ring.abandon();
        sh.drop_area(c);  // consumed either way (blob.rs:458-462): its area and slot go back to the pools
        sh.drop_slot(c);
        return decds_hip_error(e, "D2H (repaired chunkset)");
    }
    sh.drop_area(c);
    sh.drop_slot(c);
    if (out_len) *out_len = len;
    return DECDS_OK;
}

void decds_repairing_blob_free(decds_repairing_blob *rb) { delete rb; }

}  // extern "C"

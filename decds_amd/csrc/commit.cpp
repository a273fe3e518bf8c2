// commit.cpp — C-ABI of the commitment layer: the batched device path (ChunkSet::new's digests,
// chunkset Merkle roots and proofs) and host helpers for the blob-level tree (blob.rs:266-273),
// which covers only the 32-byte chunkset roots.
#include <algorithm>
#include <array>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

#include "../../include/decds_rlnc.h"
#include "blake3_host.h"
#include "blake3_impl.h"
#include "capi_internal.h"
#include "commit_kernels.h"
#include "host_mem.h"
#include "rlnc_kernels.h"
#include "rlnc_layout.h"

using namespace decds;

namespace {

void to_words(const uint8_t *b, size_t len, uint32_t w[16]) {
    uint8_t blk[64] = {0};
    std::memcpy(blk, b, len);
    for (int i = 0; i < 16; i++)
        w[i] = blk[4 * i] | (uint32_t)blk[4 * i + 1] << 8 | (uint32_t)blk[4 * i + 2] << 16 | (uint32_t)blk[4 * i + 3] << 24;
}

void to_bytes(const uint32_t w[8], uint8_t out[32]) {
    for (int i = 0; i < 8; i++)
        for (int b = 0; b < 4; b++) out[4 * i + b] = (uint8_t)(w[i] >> (8 * b));
}

// chaining value of chunk `index` (len <= 1024 bytes); `root` finalises a single-chunk message
void chunk_cv(const uint8_t *p, size_t len, uint64_t index, bool root, uint32_t cv[8]) {
    for (int i = 0; i < 8; i++) cv[i] = b3::K3.iv[i];
    const size_t blocks = len == 0 ? 1 : (len + 63) / 64;
    for (size_t b = 0; b < blocks; b++) {
        const size_t bl = b + 1 < blocks ? 64 : len - 64 * b;
        uint32_t m[16];
        to_words(p + 64 * b, bl, m);
        uint32_t flags = (b == 0 ? b3::CHUNK_START : 0u) | (b + 1 == blocks ? b3::CHUNK_END : 0u);
        if (root && b + 1 == blocks) flags |= b3::ROOT;
        b3::compress(cv, m, index, (uint32_t)bl, flags, cv);
    }
}

// BLAKE3 tree hash of [p, p+len) starting at chunk `first`: left subtree = largest power-of-two
// number of chunks that leaves at least one byte to the right (the BLAKE3 tree rule)
void subtree_cv(const uint8_t *p, size_t len, uint64_t first, bool root, uint32_t cv[8]) {
    if (len <= b3::CHUNK) {
        chunk_cv(p, len, first, root, cv);
        return;
    }
    // complete power-of-two subtrees of 8 .. 1024 chunks: 8 chunks / parents per AVX2 compression
    const size_t nch = len / b3::CHUNK;
    if (!root && len % b3::CHUNK == 0 && (nch & (nch - 1)) == 0 && nch >= 8 && nch <= b3h::MAX_SIMD_SUBTREE &&
        b3h::simd_available()) {
        b3h::simd_subtree(p, nch, first, cv);
        return;
    }
    size_t left_chunks = 1;
    while ((left_chunks * 2) * b3::CHUNK < len) left_chunks *= 2;
    const size_t left_len = left_chunks * b3::CHUNK;
    uint32_t l[8], r[8];
    subtree_cv(p, left_len, first, false, l);
    subtree_cv(p + left_len, len - left_len, first + left_chunks, false, r);
    b3::parent(l, r, root ? b3::ROOT : 0u, cv);
}

// the same tree with the two halves of each split on separate threads while the thread budget lasts
void subtree_cv_par(const uint8_t *p, size_t len, uint64_t first, bool root, uint32_t cv[8], int threads) {
    if (threads <= 1 || len <= ((size_t)1 << 20)) {
        subtree_cv(p, len, first, root, cv);
        return;
    }
    size_t left_chunks = 1;
    while ((left_chunks * 2) * b3::CHUNK < len) left_chunks *= 2;
    const size_t left_len = left_chunks * b3::CHUNK;
    uint32_t l[8], r[8];
    const int lt = threads / 2;
    std::thread t([&] { subtree_cv_par(p, left_len, first, false, l, lt); });
    subtree_cv_par(p + left_len, len - left_len, first + left_chunks, false, r, threads - lt);
    t.join();
    b3::parent(l, r, root ? b3::ROOT : 0u, cv);
}

void hash_pair(const uint8_t *l, const uint8_t *r, uint8_t out[32]) {
    uint8_t buf[64];
    std::memcpy(buf, l, 32);
    std::memcpy(buf + 32, r, 32);
    uint32_t m[16], w[8];
    to_words(buf, 64, m);
    b3::compress(b3::K3.iv, m, 0, 64, b3::CHUNK_START | b3::CHUNK_END | b3::ROOT, w);
    to_bytes(w, out);
}

}  // namespace

namespace decds {
// Chunk::digest of a full coded piece (chunk.rs:40-46) without copying it: message chunk c >= 8 is
// data[1024c - 16, 1024c + 1008), so chunks 8..1023 are hashed in place as complete subtrees; chunks
// 0..7 (the ids' chunk) from an 8 KiB copy; the 27-byte 1025th chunk joins the 1024-chunk left tree
// under ROOT. PIECE_PARTS aligned parts of 1024 / PIECE_PARTS chunks run on the host pool (per
// RepairingBlob::add_chunk, r04p: 4 parts 75-76 us, 8 parts 72-75, 16 parts 89-119); side(0 ..
// side_tasks - 1), if any, run beside them (RepairingBlob::add_chunk stages the piece for its H2D copy).
#ifndef DECDS_PIECE_PARTS
#define DECDS_PIECE_PARTS 4
#endif
constexpr size_t PIECE_PARTS = DECDS_PIECE_PARTS, PART_CHUNKS = 1024 / PIECE_PARTS;
static_assert(PART_CHUNKS >= 16 && (PART_CHUNKS & (PART_CHUNKS - 1)) == 0, "parts are power-of-two subtrees");
void full_piece_digest(uint64_t chunkset_id, uint64_t chunk_id, const uint8_t *data, uint8_t out[32],
                       const std::function<void(size_t)> *side, size_t side_tasks) {
    auto at = [&](size_t c) { return data + c * b3::CHUNK - 16; };
    uint32_t q[PIECE_PARTS][8];
    host_parallel(PIECE_PARTS + (side ? side_tasks : 0), [&](size_t task) {
        if (task >= PIECE_PARTS) {
            (*side)(task - PIECE_PARTS);
        } else if (task == 0) {
            alignas(64) uint8_t head[8 * b3::CHUNK];
            for (int b = 0; b < 8; b++) {
                head[b] = (uint8_t)(chunkset_id >> (8 * b));
                head[8 + b] = (uint8_t)(chunk_id >> (8 * b));
            }
            std::memcpy(head + 16, data, sizeof(head) - 16);
            uint32_t sub[8];
            b3h::simd_subtree(head, 8, 0, q[0]);
            for (size_t k = 8; k < PART_CHUNKS; k *= 2) {
                b3h::simd_subtree(at(k), k, k, sub);
                b3::parent(q[0], sub, 0, q[0]);
            }
        } else {
            b3h::simd_subtree(at(PART_CHUNKS * task), PART_CHUNKS, PART_CHUNKS * task, q[task]);
        }
    });
    for (size_t w = PIECE_PARTS; w > 1; w /= 2)  // fold the parts pairwise up to the 1024-chunk left tree
        for (size_t i = 0; i < w / 2; i++) b3::parent(q[2 * i], q[2 * i + 1], 0, q[i]);
    uint32_t last[8], root[8];
    chunk_cv(at(1024), F + 16 - 1024 * b3::CHUNK, 1024, false, last);
    b3::parent(q[0], last, b3::ROOT, root);
    to_bytes(root, out);
}

// the chaining value of the BLAKE3 subtree of [p, p + len) from chunk `first` (not finalised), on up to
// `threads` host threads
void blake3_subtree_cv(const uint8_t *p, size_t len, uint64_t first, uint32_t cv[8], int threads) {
    subtree_cv_par(p, len, first, false, cv, threads);
}

// blake3::hash of a message given as the chaining values of its consecutive aligned subtrees of 2^k
// chunks each (the last one possibly smaller): pairwise PARENT levels, an odd last node carried up
// unchanged — BLAKE3's left-balanced tree — and ROOT on the final parent; n >= 2
void blake3_fold_root(const uint32_t (*cvs)[8], size_t n, uint8_t out[32]) {
    std::vector<std::array<uint32_t, 8>> lvl(n);
    for (size_t i = 0; i < n; i++)
        for (int w = 0; w < 8; w++) lvl[i][w] = cvs[i][w];
    while (lvl.size() > 2) {
        std::vector<std::array<uint32_t, 8>> up((lvl.size() + 1) / 2);
        for (size_t i = 0; i < up.size(); i++) {
            if (2 * i + 1 < lvl.size())
                b3::parent(lvl[2 * i].data(), lvl[2 * i + 1].data(), 0, up[i].data());
            else
                up[i] = lvl[2 * i];
        }
        lvl.swap(up);
    }
    uint32_t root[8];
    b3::parent(lvl[0].data(), lvl[1].data(), b3::ROOT, root);
    to_bytes(root, out);
}
}  // namespace decds

extern "C" {

void decds_blake3(const uint8_t *data, size_t len, uint8_t out[32]) {
    uint32_t cv[8];
    subtree_cv(data, len, 0, true, cv);
    to_bytes(cv, out);
}

void decds_blake3_parallel(const uint8_t *data, size_t len, uint8_t out[32], int nthreads) {
    uint32_t cv[8];
    subtree_cv_par(data, len, 0, true, cv, nthreads < 1 ? 1 : nthreads);
    to_bytes(cv, out);
}

}  // extern "C"

// Incremental BLAKE3 over consecutive pieces of one message (the repaired blob's digest from the
// file flow's output slots, handle_repair.rs:129-151): the hasher of the blake3 crate — a stack of
// chaining values merged lazily, complete power-of-two subtrees aligned to the chunks hashed so far
// taken from each piece (split over host threads), at most one chunk held back for finalize.
struct decds_blake3_stream {
    std::vector<std::array<uint32_t, 8>> stack;
    uint64_t chunks = 0;  // chunks pushed (the counter of the held-back chunk)
    uint8_t part[b3::CHUNK];
    size_t part_len = 0;
    void merge(uint64_t total) {  // post-merge stack depth = popcount(total)
        while (stack.size() > (size_t)__builtin_popcountll(total)) {
            std::array<uint32_t, 8> r = stack.back(), l;
            stack.pop_back();
            l = stack.back();
            stack.pop_back();
            b3::parent(l.data(), r.data(), 0, l.data());
            stack.push_back(l);
        }
    }
    void push(const uint32_t cv[8], uint64_t counter) {
        merge(counter);
        std::array<uint32_t, 8> a;
        std::memcpy(a.data(), cv, 32);
        stack.push_back(a);
    }
};

extern "C" {

decds_blake3_stream *decds_blake3_stream_new(void) { return new decds_blake3_stream; }

void decds_blake3_stream_update(decds_blake3_stream *s, const uint8_t *p, size_t len, int nthreads) {
    if (!s || (!p && len)) return;
    constexpr size_t C = b3::CHUNK;
    uint32_t cv[8];
    if (s->part_len > 0) {  // fill the held-back chunk; finalise it only when more input follows
        const size_t take = std::min(C - s->part_len, len);
        std::memcpy(s->part + s->part_len, p, take);
        s->part_len += take, p += take, len -= take;
        if (len == 0) return;
        chunk_cv(s->part, C, s->chunks, false, cv);
        s->push(cv, s->chunks);
        s->chunks++;
        s->part_len = 0;
    }
    while (len > C) {  // the largest power-of-two subtree that fits and divides the chunks so far
        size_t sub = (size_t)1 << (63 - __builtin_clzll((unsigned long long)len));
        while (((sub - 1) & (s->chunks * C)) != 0) sub /= 2;
        if (sub <= C) {
            chunk_cv(p, C, s->chunks, false, cv);
            s->push(cv, s->chunks);
            s->chunks++;
        } else {  // its two halves pushed separately: the lazy merge never merges a would-be root
            const size_t half = sub / 2;
            uint32_t l[8], r[8];
            subtree_cv_par(p, half, s->chunks, false, l, nthreads < 1 ? 1 : nthreads);
            subtree_cv_par(p + half, half, s->chunks + half / C, false, r, nthreads < 1 ? 1 : nthreads);
            s->push(l, s->chunks);
            s->push(r, s->chunks + half / C);
            s->chunks += sub / C;
        }
        p += sub, len -= sub;
    }
    if (len > 0) {
        std::memcpy(s->part, p, len);
        s->part_len = len;
        s->merge(s->chunks);
    }
}

void decds_blake3_stream_finalize(const decds_blake3_stream *s, uint8_t out[32]) {
    uint32_t cur[8];
    size_t n = s->stack.size();
    if (n == 0) {  // one chunk or less: the chunk is the root
        chunk_cv(s->part, s->part_len, s->chunks, true, cur);
        to_bytes(cur, out);
        return;
    }
    if (s->part_len > 0) {
        chunk_cv(s->part, s->part_len, s->chunks, false, cur);
    } else {  // no held-back chunk: the top two entries are the last subtree's halves (n >= 2)
        b3::parent(s->stack[n - 2].data(), s->stack[n - 1].data(), n == 2 ? b3::ROOT : 0u, cur);
        n -= 2;
    }
    for (; n > 0; n--) b3::parent(s->stack[n - 1].data(), cur, n == 1 ? b3::ROOT : 0u, cur);
    to_bytes(cur, out);
}

void decds_blake3_stream_free(decds_blake3_stream *s) { delete s; }

void decds_chunk_digest(uint64_t chunkset_id, uint64_t chunk_id, const uint8_t *data, size_t len, uint8_t out[32]) {
    if (len == F && b3h::simd_available()) {
        full_piece_digest(chunkset_id, chunk_id, data, out, nullptr, 0);
        return;
    }
    std::vector<uint8_t> msg(16 + len);
    for (int b = 0; b < 8; b++) {
        msg[b] = (uint8_t)(chunkset_id >> (8 * b));
        msg[8 + b] = (uint8_t)(chunk_id >> (8 * b));
    }
    if (len) std::memcpy(msg.data() + 16, data, len);
    decds_blake3(msg.data(), msg.size(), out);
}

int decds_merkle_tree(const uint8_t *leaves, size_t n, uint8_t root[32], uint8_t *proofs) {
    if (!leaves || !root || n == 0)
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "no leaf nodes to build merkle tree on");
    int depth = 0;
    while (((size_t)1 << depth) < n) depth++;
    std::vector<uint8_t> cur(leaves, leaves + n * 32), nxt;
    std::vector<size_t> idx(n);
    for (size_t i = 0; i < n; i++) idx[i] = i;
    uint8_t zero[32] = {0};
    for (int lvl = 0; cur.size() > 32; lvl++) {
        const size_t len = cur.size() / 32, plen = (len + 1) / 2;
        nxt.assign(plen * 32, 0);
        for (size_t p = 0; p < plen; p++)
            hash_pair(&cur[2 * p * 32], 2 * p + 1 < len ? &cur[(2 * p + 1) * 32] : zero, &nxt[p * 32]);
        if (proofs)
            for (size_t i = 0; i < n; i++) {
                const size_t s = idx[i] ^ 1;
                std::memcpy(proofs + (i * depth + lvl) * 32, s < len ? &cur[s * 32] : zero, 32);
                idx[i] >>= 1;
            }
        uint8_t z2[32];
        hash_pair(zero, zero, z2);  // merkle_tree.rs:41 — the padding hash climbs with the level
        std::memcpy(zero, z2, 32);
        cur.swap(nxt);
    }
    std::memcpy(root, cur.data(), 32);
    return depth;
}

int decds_merkle_verify(size_t leaf_index, const uint8_t leaf[32], const uint8_t *proof, size_t proof_len,
                        const uint8_t root[32]) {
    uint8_t h[32], t[32];
    std::memcpy(h, leaf, 32);
    for (size_t k = 0; k < proof_len; k++) {
        if ((leaf_index & 1) == 0)
            hash_pair(h, proof + 32 * k, t);
        else
            hash_pair(proof + 32 * k, h, t);
        std::memcpy(h, t, 32);
        leaf_index >>= 1;
    }
    return std::memcmp(h, root, 32) == 0;
}

int decds_commit_batch(decds_ctx *ctx, const uint8_t *coded, size_t pitch, size_t n, uint64_t first_chunkset_id,
                       uint8_t *digests, uint8_t *roots, uint8_t *proofs, void *stream) {
    int s = decds_ctx_bind(ctx);
    if (s) return s;
    if (!coded || !digests || !roots || !proofs || n == 0)
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null buffer or no chunksets");
    if (pitch < F) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "coded pitch %zu < %llu", pitch, (unsigned long long)F);
    hipError_t e = launch_commit(coded, pitch, n, first_chunkset_id, digests, roots, proofs, (hipStream_t)stream);
    return e == hipSuccess ? DECDS_OK : decds_hip_error(e, "commit kernels launch");
}

size_t decds_encode_commit_workspace_bytes(size_t n) { return n * N * encode_commit_subtrees() * 32; }

int decds_encode_commit_batch(decds_ctx *ctx, const uint8_t *src, size_t n, const uint8_t *coeffs, uint8_t *dst,
                              size_t pitch, uint64_t first_chunkset_id, uint8_t *digests, uint8_t *roots,
                              uint8_t *proofs, void *workspace, void *stream) {
    return encode_commit_ids(ctx, src, n, coeffs, dst, pitch, first_chunkset_id, nullptr, digests, roots, proofs,
                             workspace, stream);
}

}  // extern "C"

// decds_encode_commit_batch with per-chunkset ids (device, n x u64; NULL: first_chunkset_id + c) on
// message-aligned rows: the coalesced ChunkSet::new batches of callers' unrelated chunkset ids
int encode_commit_ids(decds_ctx *ctx, const uint8_t *src, size_t n, const uint8_t *coeffs, uint8_t *dst, size_t pitch,
                      uint64_t first_chunkset_id, const uint64_t *ids, uint8_t *digests, uint8_t *roots, uint8_t *proofs,
                      void *workspace, void *stream) {
    if (!encode_commit_fusable(dst, pitch) || !n) {  // unaligned rows: encode, then the commitment kernels
        if (ids) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "per-chunkset ids need message-aligned rows");
        int s = decds_encode_batch(ctx, src, n, coeffs, dst, pitch, stream);
        return s ? s : decds_commit_batch(ctx, dst, pitch, n, first_chunkset_id, digests, roots, proofs, stream);
    }
    int s = decds_ctx_bind(ctx);
    if (s) return s;
    if (!src || !coeffs || !dst || !digests || !roots || !proofs || !workspace)
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null buffer");
    if (n > (1u << 24)) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "chunkset count %zu too large", n);
    if (pitch < F || (N - 1) * (uint64_t)pitch + F >= (1ull << 31))
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "coded pitch %zu outside [%llu, 2 GiB / 16)", pitch,
                               (unsigned long long)F);
    auto *sub = static_cast<uint32_t *>(workspace);
    hipError_t e = launch_encode_commit(src, n, coeffs, dst, pitch, ctx->poly, ctx->marker, first_chunkset_id, ids, sub,
                                        (hipStream_t)stream);
    if (e) return decds_hip_error(e, "fused encode + chunk hashing launch");
    e = launch_commit_fold(dst, pitch, n, sub, encode_commit_subtrees(), digests, roots, proofs, (hipStream_t)stream);
    return e == hipSuccess ? DECDS_OK : decds_hip_error(e, "commit_fold_kernel launch");
}

extern "C" {

int decds_validate_batch(decds_ctx *ctx, const uint8_t *coded, size_t pitch, size_t n_rows, const uint64_t *ids,
                         const uint8_t *proofs, size_t proof_len, const uint8_t *chunkset_roots,
                         size_t num_chunksets, const uint8_t *blob_root, uint8_t *digests, uint8_t *valid,
                         void *stream) {
    int s = decds_ctx_bind(ctx);
    if (s) return s;
    if (!coded || !ids || !digests || !valid || (proof_len && !proofs) || (num_chunksets && !chunkset_roots))
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null buffer");
    if (pitch < F) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "coded pitch %zu < %llu", pitch, (unsigned long long)F);
    if (n_rows > (1u << 30)) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "row count %zu too large", n_rows);
    hipError_t e = launch_validate(coded, pitch, n_rows, ids, proofs, proof_len, chunkset_roots, num_chunksets, blob_root,
                                   digests, valid, (hipStream_t)stream);
    return e == hipSuccess ? DECDS_OK : decds_hip_error(e, "validate kernels launch");
}

}  // extern "C"

// commit_kernels.hip — gfx950 kernels for the commitment layer that ChunkSet::new builds right
// after encoding (chunkset.rs:54-63): the BLAKE3 digest of every coded chunk (chunk.rs:40-46,
// message = chunkset_id as u64 LE || chunk_id as u64 LE || the 1,048,587-byte coded piece) and the
// 16-leaf Merkle tree of each chunkset with every leaf's inclusion proof (merkle_tree.rs:23-116).
//
// Digest: one workgroup per coded row. The 1,048,603-byte message is 1024 full BLAKE3 chunks + one
// 27-byte chunk; the root is PARENT|ROOT(subtree of the 1024 chunks, last chunk) — BLAKE3's tree
// for 1025 chunks. ~17.4 K compressions per row (16,384 chunk blocks + 1,023 parents + 2):
// VALU-bound at 12 VALU per G x 8 G x 7 rounds = 672 per 64-byte block.
#include <hip/hip_runtime.h>

#include "blake3_impl.h"
#include "commit_kernels.h"
#include "rlnc_layout.h"

namespace decds {

constexpr uint32_t MSG_BYTES = 16 + (uint32_t)F;                   // ids || coded piece
constexpr uint32_t FULL_CHUNKS = MSG_BYTES / b3::CHUNK;            // 1024
constexpr uint32_t LAST_BYTES = MSG_BYTES - FULL_CHUNKS * b3::CHUNK;  // 27
static_assert(FULL_CHUNKS == 1024 && LAST_BYTES == 27, "BLAKE3 tree shape of a coded chunk message");

#ifndef DECDS_DG_PREFETCH
#define DECDS_DG_PREFETCH 1  // 1: block b+1's loads issued before block b's compression
#endif
constexpr uint32_t CPT = 4;                       // consecutive BLAKE3 chunks per thread
constexpr uint32_t DG_WG = FULL_CHUNKS / CPT;     // 256 threads per row

struct Block {
    uint32_t w[16];
};

// One 64-byte message block (block b of full chunk c of a row). Message bytes 0..15 are the two
// little-endian u64 ids, so piece offset = message offset - 16 (≡ 0 mod 16): every block starts at
// the row's own misalignment s = piece mod 16. Byte-misaligned dwordx4 loads in this lane-per-chunk
// order run at a third of the aligned rate (tools/hashmem.hip: 2.3 vs 5.5 TB/s), so each block is
// read as 16-byte-ALIGNED words — four, plus a fifth when s != 0 — and funnel-shifted into place:
// dword shift Q = s / 4 is a template parameter (the row picks the instantiation once, a
// wave-uniform branch), byte shift r = s % 4 one v_alignbyte per message word. Q = -1: s == 0.
// The fifth word of the last block of a row with s in 1..4 reaches up to 4 bytes past the row —
// inside the same 16-byte granule as the row's last byte, so never a separate page.
template <int Q>
__device__ __forceinline__ Block load_block(const uint8_t *piece, const uint8_t *abase, uint32_t r, uint32_t c,
                                            uint32_t b, uint64_t cs_id, uint64_t chunk_id) {
    Block m;
    const int64_t off = (int64_t)c * b3::CHUNK + b * b3::BLOCK - 16;
    if (off >= 0) {
        const uint4 *pa = reinterpret_cast<const uint4 *>(abase + off);
        uint32_t w[20];
#pragma unroll
        for (int k = 0; k < (Q < 0 ? 4 : 5); k++) {
            const uint4 v = pa[k];
            w[4 * k] = v.x, w[4 * k + 1] = v.y, w[4 * k + 2] = v.z, w[4 * k + 3] = v.w;
        }
#pragma unroll
        for (int i = 0; i < 16; i++) {
            if constexpr (Q < 0)
                m.w[i] = w[i];
            else
                m.w[i] = __builtin_amdgcn_alignbyte(w[i + Q + 1], w[i + Q], r);
        }
    } else {
        // block 0 of chunk 0: ids, then piece bytes 0..47. The address is wave-uniform here: spelled
        // byte-wise so it cannot become a scalar (s_load) access, which drops misalignment
        m.w[0] = (uint32_t)cs_id, m.w[1] = (uint32_t)(cs_id >> 32);
        m.w[2] = (uint32_t)chunk_id, m.w[3] = (uint32_t)(chunk_id >> 32);
#pragma unroll
        for (int i = 4; i < 16; i++) {
            const uint8_t *p = piece + 4 * (i - 4);
            m.w[i] = p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
        }
    }
    return m;
}

// chaining value of full chunk c of a row (16 blocks)
template <int Q>
__device__ __forceinline__ void chunk_cv(const uint8_t *piece, const uint8_t *abase, uint32_t r, uint32_t c,
                                         uint64_t cs_id, uint64_t chunk_id, uint32_t cv[8]) {
#pragma unroll
    for (int i = 0; i < 8; i++) cv[i] = b3::K3.iv[i];
#if DECDS_DG_PREFETCH
    Block m = load_block<Q>(piece, abase, r, c, 0, cs_id, chunk_id);
#pragma unroll 1
    for (uint32_t b = 0; b < 16; b++) {
        const Block nxt = load_block<Q>(piece, abase, r, c, b < 15 ? b + 1 : b, cs_id, chunk_id);
        const uint32_t flags = (b == 0 ? b3::CHUNK_START : 0u) | (b == 15 ? b3::CHUNK_END : 0u);
        b3::compress(cv, m.w, c, b3::BLOCK, flags, cv);
        m = nxt;
    }
#else
#pragma unroll 1
    for (uint32_t b = 0; b < 16; b++) {
        const Block m = load_block<Q>(piece, abase, r, c, b, cs_id, chunk_id);
        const uint32_t flags = (b == 0 ? b3::CHUNK_START : 0u) | (b == 15 ? b3::CHUNK_END : 0u);
        b3::compress(cv, m.w, c, b3::BLOCK, flags, cv);
    }
#endif
}

// thread t: chunks 4t..4t+3 folded into the chaining value of their 4-chunk subtree (all lanes busy)
template <int Q>
__device__ __forceinline__ void subtree4_cv(const uint8_t *piece, uint32_t t, uint64_t cs_id, uint64_t chunk_id,
                                            uint32_t acc[8]) {
    const uint32_t s = (uint32_t)(reinterpret_cast<uintptr_t>(piece) & 15);
    const uint8_t *abase = piece - s;
    const uint32_t r = s & 3;
    uint32_t a[8], b[8], lo[8], hi[8];
    chunk_cv<Q>(piece, abase, r, 4 * t, cs_id, chunk_id, a);
    chunk_cv<Q>(piece, abase, r, 4 * t + 1, cs_id, chunk_id, b);
    b3::parent(a, b, 0, lo);
    chunk_cv<Q>(piece, abase, r, 4 * t + 2, cs_id, chunk_id, a);
    chunk_cv<Q>(piece, abase, r, 4 * t + 3, cs_id, chunk_id, b);
    b3::parent(a, b, 0, hi);
    b3::parent(lo, hi, 0, acc);
}

// Digest of one coded row per 256-thread workgroup: 4-chunk subtrees in registers, the 256
// subtree values folded in LDS (8 PARENT levels), then thread 0 adds the 27-byte 1025th chunk under
// the ROOT parent.
// ids == NULL: row = c*16 + j of a freshly encoded batch, chunkset_id = first + c and chunk_id =
// chunkset_id*16 + j (chunkset.rs:47); else the row's claimed (chunkset_id, chunk_id) = ids[2row..].
__global__ __launch_bounds__(DG_WG) void chunk_digest_kernel(const uint8_t *__restrict__ coded, size_t pitch,
                                                             uint64_t first_chunkset_id,
                                                             const uint64_t *__restrict__ ids,
                                                             uint8_t *__restrict__ digests) {
    __shared__ uint32_t cvs[DG_WG][8];
    const uint32_t row = blockIdx.x;
    const uint64_t cs_id = ids ? ids[2 * (size_t)row] : first_chunkset_id + row / N;
    const uint64_t chunk_id = ids ? ids[2 * (size_t)row + 1] : cs_id * N + row % N;
    const uint8_t *piece = coded + (size_t)row * pitch;
    const uint32_t t = threadIdx.x;
    uint32_t acc[8];
    switch ((uint32_t)(reinterpret_cast<uintptr_t>(piece) & 15) >> 2 |
            ((reinterpret_cast<uintptr_t>(piece) & 15) == 0 ? 4u : 0u)) {
        case 0: subtree4_cv<0>(piece, t, cs_id, chunk_id, acc); break;
        case 1: subtree4_cv<1>(piece, t, cs_id, chunk_id, acc); break;
        case 2: subtree4_cv<2>(piece, t, cs_id, chunk_id, acc); break;
        case 3: subtree4_cv<3>(piece, t, cs_id, chunk_id, acc); break;
        default: subtree4_cv<-1>(piece, t, cs_id, chunk_id, acc); break;
    }
#pragma unroll
    for (int i = 0; i < 8; i++) cvs[t][i] = acc[i];
    __syncthreads();
    // PARENT levels over the 256 subtree values (complete binary tree, in place)
#pragma unroll 1
    for (uint32_t width = DG_WG / 2; width >= 1; width /= 2) {
        uint32_t out[8];
        if (t < width) b3::parent(cvs[2 * t], cvs[2 * t + 1], 0, out);
        __syncthreads();
        if (t < width)
#pragma unroll
            for (int i = 0; i < 8; i++) cvs[t][i] = out[i];
        __syncthreads();
    }
    if (t == 0) {
        // last chunk: LAST_BYTES message bytes = the piece's final 27 bytes, one partial block
        uint32_t m[16], last[8], root[8], left[8];
#pragma unroll
        for (int i = 0; i < 16; i++) {
            uint32_t w = 0;
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (4 * i + k < (int)LAST_BYTES) w |= (uint32_t)piece[FULL_CHUNKS * b3::CHUNK - 16 + 4 * i + k] << (8 * k);
            m[i] = w;
        }
        b3::compress(b3::K3.iv, m, FULL_CHUNKS, LAST_BYTES, b3::CHUNK_START | b3::CHUNK_END, last);
#pragma unroll
        for (int i = 0; i < 8; i++) left[i] = cvs[0][i];
        b3::parent(left, last, b3::ROOT, root);
        uint32_t *d = reinterpret_cast<uint32_t *>(digests + (size_t)row * 32);
#pragma unroll
        for (int i = 0; i < 8; i++) d[i] = root[i];
    }
}

// Digest of each coded row from the fused encode's 256 aligned 4-chunk subtree values
// (rlnc_encode_hash_kernel). One wave per row: lane i folds subtrees 4i .. 4i+3 into the 16-chunk
// subtree i, six PARENT levels fold those into the 1024-chunk left tree, then the 27-byte 1025th
// chunk joins under ROOT, as chunk_digest_kernel.
constexpr uint32_t FOLD_LANES = 64, SUB_PER_ROW = FULL_CHUNKS / 4;  // 256
__global__ __launch_bounds__(FOLD_LANES) void commit_fold_kernel(const uint8_t *__restrict__ coded, size_t pitch,
                                                                 const uint32_t *__restrict__ sub,
                                                                 uint8_t *__restrict__ digests) {
    const size_t row = blockIdx.x;
    const uint32_t i = threadIdx.x;
    const uint32_t *p = sub + (row * SUB_PER_ROW + 4 * i) * 8;
    uint32_t a[8], b[8], lo[8], hi[8], cv[8];
#pragma unroll
    for (int w = 0; w < 8; w++) a[w] = p[w], b[w] = p[8 + w];
    b3::parent(a, b, 0, lo);
#pragma unroll
    for (int w = 0; w < 8; w++) a[w] = p[16 + w], b[w] = p[24 + w];
    b3::parent(a, b, 0, hi);
    b3::parent(lo, hi, 0, cv);
#pragma unroll
    for (uint32_t k = 0; k < 6; k++) {
        uint32_t sib[8];
        const bool right = (i >> k) & 1u;
#pragma unroll
        for (int w = 0; w < 8; w++) {
            sib[w] = __shfl_xor(cv[w], 1 << k, FOLD_LANES);
            lo[w] = right ? sib[w] : cv[w];
            hi[w] = right ? cv[w] : sib[w];
        }
        b3::parent(lo, hi, 0, cv);
    }
    if (i == 0) {
        const uint8_t *piece = coded + row * pitch;
        uint32_t m[16], last[8], root[8];
#pragma unroll
        for (int w = 0; w < 16; w++) {
            uint32_t x = 0;
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (4 * w + k < (int)LAST_BYTES) x |= (uint32_t)piece[FULL_CHUNKS * b3::CHUNK - 16 + 4 * w + k] << (8 * k);
            m[w] = x;
        }
        b3::compress(b3::K3.iv, m, FULL_CHUNKS, LAST_BYTES, b3::CHUNK_START | b3::CHUNK_END, last);
        b3::parent(cv, last, b3::ROOT, root);
        uint32_t *d = reinterpret_cast<uint32_t *>(digests + row * 32);
#pragma unroll
        for (int w = 0; w < 8; w++) d[w] = root[w];
    }
}

// Merkle tree of one chunkset's 16 digests (merkle_tree.rs:23-50) and the 4-hash inclusion proof of
// every leaf (merkle_tree.rs:75-116); 16 leaves make a complete tree, no zero-hash padding. Lane
// j of a 16-lane group holds the node above leaf j; at level l its sibling node sits in lane
// j ^ 2^l, which is also leaf j's proof element for that level. Every lane hashes its own parent
// (redundantly within a pair), so the 4 levels cost 4 compressions with all lanes active.
constexpr uint32_t MK_WG = 64;
__global__ __launch_bounds__(MK_WG) void chunkset_merkle_kernel(const uint8_t *__restrict__ digests, size_t n,
                                                                uint8_t *__restrict__ roots,
                                                                uint8_t *__restrict__ proofs) {
    const size_t g = (size_t)blockIdx.x * MK_WG + threadIdx.x;  // = cs * 16 + leaf
    const uint32_t j = threadIdx.x & (N - 1);
    const bool live = g < n * N;
    uint32_t node[8];
    const uint32_t *d = reinterpret_cast<const uint32_t *>(digests + (live ? g : 0) * 32);
#pragma unroll
    for (int w = 0; w < 8; w++) node[w] = d[w];
    uint32_t *pr = reinterpret_cast<uint32_t *>(proofs + g * 4 * 32);
#pragma unroll
    for (uint32_t level = 0; level < 4; level++) {
        uint32_t sib[8], l[8], r[8];
        const bool right = (j >> level) & 1u;
#pragma unroll
        for (int w = 0; w < 8; w++) {
            sib[w] = __shfl_xor(node[w], 1 << level, N);
            l[w] = right ? sib[w] : node[w];
            r[w] = right ? node[w] : sib[w];
            if (live) pr[level * 8 + w] = sib[w];
        }
        b3::hash64(l, r, node);
    }
    if (live && j == 0) {
        uint32_t *rt = reinterpret_cast<uint32_t *>(roots + (g / N) * 32);
#pragma unroll
        for (int w = 0; w < 8; w++) rt[w] = node[w];
    }
}

// BlobHeader::validate_chunk (blob.rs:211-215) per received row, one lane per row:
// MerkleTree::verify_proof (merkle_tree.rs:131-146) = fold the proof from the leaf upwards,
// sibling on the right when the index bit is 0, compare with the root.
__device__ __forceinline__ bool verify_path(uint64_t index, const uint32_t leaf[8], const uint8_t *proof, size_t len,
                                            const uint8_t *root) {
    uint32_t h[8];
#pragma unroll
    for (int w = 0; w < 8; w++) h[w] = leaf[w];
    for (size_t k = 0; k < len; k++) {
        uint32_t sib[8], t[8];
        const uint32_t *ps = reinterpret_cast<const uint32_t *>(proof + 32 * k);
#pragma unroll
        for (int w = 0; w < 8; w++) sib[w] = ps[w];
        if ((index & 1) == 0)
            b3::hash64(h, sib, t);
        else
            b3::hash64(sib, h, t);
#pragma unroll
        for (int w = 0; w < 8; w++) h[w] = t[w];
        index >>= 1;
    }
    const uint32_t *r = reinterpret_cast<const uint32_t *>(root);
    bool eq = true;
#pragma unroll
    for (int w = 0; w < 8; w++) eq &= h[w] == r[w];
    return eq;
}

__global__ __launch_bounds__(64) void validate_kernel(const uint8_t *__restrict__ digests, size_t n_rows,
                                                      const uint64_t *__restrict__ ids,
                                                      const uint8_t *__restrict__ proofs, size_t proof_len,
                                                      const uint8_t *__restrict__ chunkset_roots,
                                                      size_t num_chunksets, const uint8_t *__restrict__ blob_root,
                                                      uint8_t *__restrict__ valid) {
    const size_t r = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (r >= n_rows) return;
    const uint64_t cs_id = ids[2 * r], chunk_id = ids[2 * r + 1];
    uint32_t leaf[8];
    const uint32_t *d = reinterpret_cast<const uint32_t *>(digests + r * 32);
#pragma unroll
    for (int w = 0; w < 8; w++) leaf[w] = d[w];
    const uint8_t *proof = proofs + r * proof_len * 32;
    bool ok = proof_len >= PROOF_SIZE;
    if (ok && blob_root) ok = verify_path(chunk_id, leaf, proof, proof_len, blob_root);       // chunk.rs:88-90
    if (ok) ok = cs_id < num_chunksets;                                                        // blob.rs:213
    if (ok) ok = verify_path(chunk_id % N, leaf, proof, PROOF_SIZE, chunkset_roots + cs_id * 32);  // chunk.rs:103-110
    valid[r] = ok ? 1 : 0;
}

hipError_t launch_commit(const uint8_t *coded, size_t pitch, size_t n, uint64_t first_chunkset_id, uint8_t *digests,
                         uint8_t *roots, uint8_t *proofs, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(chunk_digest_kernel, dim3((uint32_t)(n * N)), dim3(DG_WG), 0, stream, coded, pitch,
                       first_chunkset_id, (const uint64_t *)nullptr, digests);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(chunkset_merkle_kernel, dim3((uint32_t)((n * N + MK_WG - 1) / MK_WG)), dim3(MK_WG), 0, stream,
                       digests, n, roots, proofs);
    return hipGetLastError();
}

hipError_t launch_commit_fold(const uint8_t *coded, size_t pitch, size_t n, const uint32_t *sub, uint32_t per_row,
                              uint8_t *digests, uint8_t *roots, uint8_t *proofs, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (per_row != SUB_PER_ROW) return hipErrorInvalidValue;
    hipLaunchKernelGGL(commit_fold_kernel, dim3((uint32_t)(n * N)), dim3(FOLD_LANES), 0, stream, coded, pitch, sub, digests);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(chunkset_merkle_kernel, dim3((uint32_t)((n * N + MK_WG - 1) / MK_WG)), dim3(MK_WG), 0, stream,
                       digests, n, roots, proofs);
    return hipGetLastError();
}

hipError_t launch_validate(const uint8_t *coded, size_t pitch, size_t n_rows, const uint64_t *ids,
                           const uint8_t *proofs, size_t proof_len, const uint8_t *chunkset_roots,
                           size_t num_chunksets, const uint8_t *blob_root, uint8_t *digests, uint8_t *valid,
                           hipStream_t stream) {
    if (n_rows == 0) return hipSuccess;
    hipLaunchKernelGGL(chunk_digest_kernel, dim3((uint32_t)n_rows), dim3(DG_WG), 0, stream, coded, pitch, (uint64_t)0,
                       ids, digests);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(validate_kernel, dim3((uint32_t)((n_rows + 63) / 64)), dim3(64), 0, stream, digests, n_rows,
                       ids, proofs, proof_len, chunkset_roots, num_chunksets, blob_root, valid);
    return hipGetLastError();
}

}  // namespace decds

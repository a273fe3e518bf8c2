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
#include "hip_status.h"
#include "rlnc_layout.h"

namespace decds {

constexpr uint32_t MSG_BYTES = 16 + (uint32_t)F;                   // ids || coded piece
constexpr uint32_t FULL_CHUNKS = MSG_BYTES / b3::CHUNK;            // 1024
constexpr uint32_t LAST_BYTES = MSG_BYTES - FULL_CHUNKS * b3::CHUNK;  // 27
static_assert(FULL_CHUNKS == 1024 && LAST_BYTES == 27, "BLAKE3 tree shape of a coded chunk message");

constexpr uint32_t DG_WG = FULL_CHUNKS / 4;  // 256 threads per row, 4 consecutive chunks each
constexpr uint32_t BLOB_GROUP_BYTES = FULL_CHUNKS * b3::CHUNK;  // 1 MiB: blob_group_kernel's unit
static_assert((uint64_t)CS % BLOB_GROUP_BYTES == 0, "a chunkset is whole blob-digest groups");
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Digest of one coded row per 256-thread workgroup: thread t hashes chunks 4t .. 4t+3 one after the
// other and folds them into their 4-chunk subtree in registers; the 256 subtree values fold in LDS
// (8 PARENT levels), then thread 0 adds the 27-byte 1025th chunk under the ROOT parent.
// ids == NULL: row = c*16 + j of a freshly encoded batch, chunkset_id = first + c and chunk_id =
// chunkset_id*16 + j (chunkset.rs:47); else the row's claimed (chunkset_id, chunk_id) = ids[2row..].
// Message blocks are staged through LDS (DG_LDS): a wave walks its 64 lanes' chunks in 32 steps of
// 128 message bytes (4 chunks x 8 steps per lane); per step it loads the 64 segments cooperatively —
// 8 lanes per 128-byte segment, 8 segments per load instruction, unaligned 16-byte buffer loads —
// writes them to one 128-byte LDS slot per lane and each lane reads its own two blocks back (slots
// XOR-swizzled: every ds_read_b128 group hits 16 distinct bank quads). The next step's loads are in
// flight across this step's compressions. (The lane-per-chunk form loaded 5 aligned words per block
// and funnel-shifted them: 64 distinct lines per load instruction, 0.68-0.75 ms at cfg2.)
constexpr uint32_t DG_STEP = 128;                       // message bytes per chunk per step
constexpr uint32_t DG_STEPS = 4 * b3::CHUNK / DG_STEP;  // 32: 4 chunks per lane
__device__ __forceinline__ uint32_t dg_slot(uint32_t t, uint32_t piece) {
    return t * DG_STEP + 16 * (piece ^ ((t >> 1) & 7u));
}

// The 1024-chunk BLAKE3 subtree (chaining value, not finalised) of the message at byte `bias` of rs's
// buffer (message byte m = buffer byte m + bias; a negative bias reads zeros before the buffer), chunk
// counters counter0 + 0 .. 1023: thread t hashes chunks 4t .. 4t+3 as described above and the 256 subtree
// values fold in LDS; the result is in cvs[0][0..7] of the returned LDS array for every thread. IDS:
// chunk 0's block 0 starts with the two ids (chunk.rs:40-46), patched over the zeros read at bias -16.
template <bool IDS>
__device__ __forceinline__ const uint32_t (*subtree_1024(__amdgpu_buffer_rsrc_t rs, int32_t bias, uint64_t counter0,
                                                        uint64_t cs_id, uint64_t chunk_id,
                                                        uint8_t *slots))[8] {
    const uint32_t t = threadIdx.x, l = t & 63u, wb = t & ~63u;
    // load k of this lane: segment of thread lt = wb + 8k + l/8, its 16-byte piece l % 8
    const uint32_t lt0 = wb + (l >> 3), lp = l & 7u;
    auto load_step = [&](u32x4 (&v)[8], uint32_t g) {  // step g: chunk 4 lt + g / 8, bytes 128 (g % 8) ..
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) {
            const uint32_t lt = lt0 + 8 * k;
            const uint32_t off = (4 * lt + (g >> 3)) * b3::CHUNK + (g & 7u) * DG_STEP + 16 * lp + (uint32_t)bias;
            v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
        }
    };
    u32x4 pf[8];
    load_step(pf, 0);
    uint32_t cv[8], first[8], lo[8], acc[8];
#pragma unroll 1
    for (uint32_t g = 0; g < DG_STEPS; g++) {
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) *reinterpret_cast<u32x4 *>(slots + dg_slot(lt0 + 8 * k, lp)) = pf[k];
        if (g + 1 < DG_STEPS) load_step(pf, g + 1);  // in flight across this step's compressions
        const uint32_t st = g & 7u, a = g >> 3;
        const uint64_t c = counter0 + 4 * t + a;
        if (st == 0)
#pragma unroll
            for (int i = 0; i < 8; i++) cv[i] = b3::K3.iv[i];
        // one wave: its LDS accesses complete in order, no barrier between the slot writes and reads
#pragma unroll
        for (uint32_t kb = 0; kb < 2; kb++) {
            uint32_t mw[16];
#pragma unroll
            for (uint32_t w = 0; w < 4; w++) {
                const u32x4 v = *reinterpret_cast<const u32x4 *>(slots + dg_slot(t, 4 * kb + w));
                mw[4 * w] = v.x, mw[4 * w + 1] = v.y, mw[4 * w + 2] = v.z, mw[4 * w + 3] = v.w;
            }
            if (IDS && kb == 0 && g == 0) {  // chunk 0's block 0 starts with the two ids (chunk.rs:40-46)
                const bool c0 = t == 0;
                mw[0] = c0 ? (uint32_t)cs_id : mw[0];
                mw[1] = c0 ? (uint32_t)(cs_id >> 32) : mw[1];
                mw[2] = c0 ? (uint32_t)chunk_id : mw[2];
                mw[3] = c0 ? (uint32_t)(chunk_id >> 32) : mw[3];
            }
            const uint32_t k = 2 * st + kb;
            b3::compress(cv, mw, c, b3::BLOCK, (k == 0 ? b3::CHUNK_START : 0u) | (k == 15 ? b3::CHUNK_END : 0u), cv);
        }
        if (st == 7) {  // chunk 4t + a done: fold into the 4-chunk subtree
            if (a == 0 || a == 2) {
#pragma unroll
                for (int i = 0; i < 8; i++) first[i] = cv[i];
            } else if (a == 1) {
                b3::parent(first, cv, 0, lo);
            } else {
                uint32_t hi[8];
                b3::parent(first, cv, 0, hi);
                b3::parent(lo, hi, 0, acc);
            }
        }
    }
    __syncthreads();  // every wave is done with its slots
    uint32_t(*cvs)[8] = reinterpret_cast<uint32_t(*)[8]>(slots);
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
    return cvs;
}

__global__ __launch_bounds__(DG_WG) void chunk_digest_kernel(const uint8_t *__restrict__ coded, size_t pitch,
                                                             uint64_t first_chunkset_id,
                                                             const uint64_t *__restrict__ ids,
                                                             uint8_t *__restrict__ digests) {
    __shared__ __attribute__((aligned(16))) uint8_t slots[DG_WG * DG_STEP];  // 32 KiB; the fold reuses it
    const uint32_t row = blockIdx.x;
    const uint64_t cs_id = ids ? ids[2 * (size_t)row] : first_chunkset_id + row / N;
    const uint64_t chunk_id = ids ? ids[2 * (size_t)row + 1] : cs_id * N + row % N;
    const uint8_t *piece = coded + (size_t)row * pitch;
    // message byte m is piece byte m - 16 (block 0 of chunk 0 reads offset -16: out of range, zeros,
    // ids patched in)
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(piece), 0, (int)F, 0x00020000);
    const uint32_t(*cvs)[8] = subtree_1024<true>(rs, -16, 0, cs_id, chunk_id, slots);
    if (threadIdx.x == 0) {
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

// Blob::new's whole-blob digest (blake3::hash(&data), blob.rs:249), group part: workgroup g hashes the
// 1 MiB at data + g MiB — BLAKE3 chunks first_chunk + 1024 g .. + 1023, all full — into its 1024-chunk
// subtree chaining value at cvs + 32 g. A chunkset is 10 such groups, so groups never straddle the
// batches or shards of the blob paths; the host folds the groups' values (and the last partial group's,
// hashed on the host) pairwise into the root (decds_blob_new).
__global__ __launch_bounds__(DG_WG) void blob_group_kernel(const uint8_t *__restrict__ data, uint64_t first_chunk,
                                                           uint8_t *__restrict__ cvs_out) {
    __shared__ __attribute__((aligned(16))) uint8_t slots[DG_WG * DG_STEP];
    const uint32_t g = blockIdx.x;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(data + (size_t)g * BLOB_GROUP_BYTES), 0, (int)BLOB_GROUP_BYTES, 0x00020000);
    const uint32_t(*cvs)[8] = subtree_1024<false>(rs, 0, first_chunk + (uint64_t)g * FULL_CHUNKS, 0, 0, slots);
    if (threadIdx.x < 8) reinterpret_cast<uint32_t *>(cvs_out + (size_t)g * 32)[threadIdx.x] = cvs[0][threadIdx.x];
}

// Digest of each coded row from the fused encode's 256 aligned 4-chunk subtree values
// (rlnc_encode_hash_kernel). One wave per row: lane i folds subtrees 4i .. 4i+3 (two independent
// parents, then theirs) into the 16-chunk subtree i, six PARENT levels fold those into the 1024-chunk
// left tree, then the 27-byte 1025th chunk joins under ROOT, as chunk_digest_kernel. Latency-bound
// (one wave, a chain of compressions), so the 1025th chunk rides along in cross-lane level 0: lane 63
// compresses it instead of the (62, 63) parent that lane 62 computes as well, and every later level
// reads a sibling group's value from its lowest lane, which lane 63 never is.
constexpr uint32_t FOLD_LANES = 64, SUB_PER_ROW = FULL_CHUNKS / 4;  // 256
__global__ __launch_bounds__(FOLD_LANES) void commit_fold_kernel(const uint8_t *__restrict__ coded, size_t pitch,
                                                                 const uint32_t *__restrict__ sub,
                                                                 uint8_t *__restrict__ digests) {
    const size_t row = blockIdx.x;
    const uint32_t i = threadIdx.x;
    const uint8_t *piece = coded + row * pitch;
    const bool tail = i == FOLD_LANES - 1;
    uint32_t tw[16];  // lane 63: the last chunk's 27 message bytes (the piece's final 27 bytes)
#pragma unroll
    for (int w = 0; w < 16; w++) {
        uint32_t x = 0;
        if (tail)
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (4 * w + k < (int)LAST_BYTES) x |= (uint32_t)piece[FULL_CHUNKS * b3::CHUNK - 16 + 4 * w + k] << (8 * k);
        tw[w] = x;
    }
    const uint32_t *p = sub + (row * SUB_PER_ROW + 4 * i) * 8;
    uint32_t m[16], lo[8], hi[8], cv[8], last[8];
#pragma unroll
    for (int w = 0; w < 16; w++) m[w] = p[w];
    b3::parent(m, m + 8, 0, lo);
#pragma unroll
    for (int w = 0; w < 16; w++) m[w] = p[16 + w];
    b3::parent(m, m + 8, 0, hi);
    b3::parent(lo, hi, 0, cv);
#pragma unroll
    for (uint32_t k = 0; k < 6; k++) {
        const uint32_t sl = (i ^ (1u << k)) & ~((1u << k) - 1);  // the sibling group's lowest lane
        const bool right = (i >> k) & 1u;
#pragma unroll
        for (int w = 0; w < 8; w++) {
            const uint32_t sib = __shfl(cv[w], sl, FOLD_LANES);
            m[w] = right ? sib : cv[w];
            m[w + 8] = right ? cv[w] : sib;
        }
        if (k == 0) {
#pragma unroll
            for (int w = 0; w < 16; w++) m[w] = tail ? tw[w] : m[w];
            b3::compress(b3::K3.iv, m, tail ? FULL_CHUNKS : 0u, tail ? LAST_BYTES : b3::BLOCK,
                         tail ? (b3::CHUNK_START | b3::CHUNK_END) : b3::PARENT, cv);
#pragma unroll
            for (int w = 0; w < 8; w++) last[w] = __shfl(cv[w], FOLD_LANES - 1, FOLD_LANES);
        } else {
            b3::parent(m, m + 8, 0, cv);
        }
    }
    if (i == 0) {
        uint32_t root[8];
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

hipError_t configure_commit_kernels() {
    const void *fns[] = {reinterpret_cast<const void *>(chunk_digest_kernel), reinterpret_cast<const void *>(chunkset_merkle_kernel),
                         reinterpret_cast<const void *>(commit_fold_kernel), reinterpret_cast<const void *>(validate_kernel),
                         reinterpret_cast<const void *>(blob_group_kernel)};
    for (const void *f : fns) {
        hipFuncAttributes a;
        hipError_t e = hipFuncGetAttributes(&a, f);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_blob_groups(const uint8_t *data, size_t n_groups, uint64_t first_chunk, uint8_t *cvs,
                              hipStream_t stream) {
    if (n_groups == 0) return hipSuccess;
    if (hipError_t p_ = hip_launch_begin("blob_group_kernel")) return p_;
    hipLaunchKernelGGL(blob_group_kernel, dim3((uint32_t)n_groups), dim3(DG_WG), 0, stream, data, first_chunk, cvs);
    return hipGetLastError();
}

hipError_t launch_commit(const uint8_t *coded, size_t pitch, size_t n, uint64_t first_chunkset_id, uint8_t *digests,
                         uint8_t *roots, uint8_t *proofs, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (hipError_t p_ = hip_launch_begin("chunk_digest_kernel")) return p_;
    hipLaunchKernelGGL(chunk_digest_kernel, dim3((uint32_t)(n * N)), dim3(DG_WG), 0, stream, coded, pitch,
                       first_chunkset_id, (const uint64_t *)nullptr, digests);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (hipError_t p_ = hip_launch_begin("chunkset_merkle_kernel")) return p_;
    hipLaunchKernelGGL(chunkset_merkle_kernel, dim3((uint32_t)((n * N + MK_WG - 1) / MK_WG)), dim3(MK_WG), 0, stream,
                       digests, n, roots, proofs);
    return hipGetLastError();
}

hipError_t launch_commit_fold(const uint8_t *coded, size_t pitch, size_t n, const uint32_t *sub, uint32_t per_row,
                              uint8_t *digests, uint8_t *roots, uint8_t *proofs, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (per_row != SUB_PER_ROW) return hipErrorInvalidValue;
    if (hipError_t p_ = hip_launch_begin("commit_fold_kernel")) return p_;
    hipLaunchKernelGGL(commit_fold_kernel, dim3((uint32_t)(n * N)), dim3(FOLD_LANES), 0, stream, coded, pitch, sub, digests);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (hipError_t p_ = hip_launch_begin("chunkset_merkle_kernel")) return p_;
    hipLaunchKernelGGL(chunkset_merkle_kernel, dim3((uint32_t)((n * N + MK_WG - 1) / MK_WG)), dim3(MK_WG), 0, stream,
                       digests, n, roots, proofs);
    return hipGetLastError();
}

hipError_t launch_validate(const uint8_t *coded, size_t pitch, size_t n_rows, const uint64_t *ids,
                           const uint8_t *proofs, size_t proof_len, const uint8_t *chunkset_roots,
                           size_t num_chunksets, const uint8_t *blob_root, uint8_t *digests, uint8_t *valid,
                           hipStream_t stream) {
    if (n_rows == 0) return hipSuccess;
    if (hipError_t p_ = hip_launch_begin("chunk_digest_kernel")) return p_;
    hipLaunchKernelGGL(chunk_digest_kernel, dim3((uint32_t)n_rows), dim3(DG_WG), 0, stream, coded, pitch, (uint64_t)0,
                       ids, digests);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (hipError_t p_ = hip_launch_begin("validate_kernel")) return p_;
    hipLaunchKernelGGL(validate_kernel, dim3((uint32_t)((n_rows + 63) / 64)), dim3(64), 0, stream, digests, n_rows,
                       ids, proofs, proof_len, chunkset_roots, num_chunksets, blob_root, valid);
    return hipGetLastError();
}

}  // namespace decds

/*
 * decds_rlnc.h — C-ABI of the MI355X-native RLNC chunkset codec (libdecds_rlnc.so, gfx950).
 *
 * Drop-in seam. decds-lib reaches its arithmetic through crate rlnc =0.4.0 from
 * decds-lib/src/chunkset.rs; these entry points replace those call sites and the chunkset
 * iteration around them in decds-lib/src/blob.rs. Each declaration names the reference interface
 * it replaces (file:line under /root/reference). Plain pointers and sizes only: no Rust, torch or
 * HIP types cross the boundary; a hipStream_t travels as `void *` (NULL = default stream).
 *
 * Memory ownership: the caller owns every buffer. The library borrows pointers for the duration
 * of the call (device calls: until the enqueued work on `stream` completes) and never frees
 * caller memory. A context owns only its device selection, field parameters and error text.
 *
 * Pointer kinds: *_batch functions take DEVICE pointers (hipMalloc'd or torch CUDA storage) and
 * are asynchronous on `stream`; decds_chunkset_* / decds_repairing_chunkset_* / decds_blob_* /
 * decds_repairing_blob_* take HOST pointers and are synchronous. The library never page-locks
 * caller memory behind the caller's back: host buffers inside a range registered with
 * decds_host_register or allocated with decds_host_alloc are DMA'd directly, any other host memory
 * is staged through the context's own page-locked buffers (correct, slower).
 *
 * Status codes map 1:1 onto decds-lib/src/errors.rs (DecdsError); negative codes are runtime
 * failures that the Rust side surfaces as ChunksetRepairingFailed — there is never a silent CPU
 * fallback: without a usable gfx950 device every compute entry point returns DECDS_ERR_NO_DEVICE.
 */
#ifndef DECDS_RLNC_H
#define DECDS_RLNC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DECDS_NUM_ORIGINAL_CHUNKS 10u        /* chunkset.rs:19 */
#define DECDS_NUM_ERASURE_CODED_CHUNKS 16u   /* chunkset.rs:21, consts.rs:5 */
#define DECDS_CHUNKSET_BYTES 10485760ull     /* chunkset.rs:20 */
#define DECDS_PIECE_BYTES 1048577ull         /* chunkset.rs:117 */
#define DECDS_CODED_PIECE_BYTES 1048587ull   /* rlnc full coded piece: coding vector || payload */
#define DECDS_REPAIR_PLAN_BYTES 128u
/* Recommended device layout of coded rows for the batch API: pitch 1,048,704 (= 8193 x 128) with
 * the first row starting 118 bytes past a 128-byte boundary, so every row's payload (row + 10) is
 * 128-byte aligned. The encoder's row stores are then line-aligned: +9-10 % encode throughput
 * against rows packed at 1,048,587. Any pitch >= 1,048,587 is accepted. */
#define DECDS_CODED_PITCH_ALIGNED 1048704ull
#define DECDS_CODED_ROW_OFFSET_ALIGNED 118u
#define DECDS_NO_CANDIDATE 0xFFu

/* ---- status codes (decds-lib/src/errors.rs:3-48) ------------------------------------------- */
#define DECDS_OK 0
#define DECDS_ERR_INVALID_CHUNKSET_SIZE 1          /* InvalidChunksetSize(len)        errors.rs:36 */
#define DECDS_ERR_INVALID_CHUNK_METADATA 2         /* InvalidChunkMetadata(id)        errors.rs:38 */
#define DECDS_ERR_CHUNKSET_READY_TO_REPAIR 3       /* ChunksetReadyToRepair(id)       errors.rs:23 */
#define DECDS_ERR_CHUNK_DECODING_FAILED 4          /* ChunkDecodingFailed(id, msg)    errors.rs:42 */
#define DECDS_ERR_CHUNKSET_NOT_YET_READY 5         /* ChunksetNotYetReadyToRepair(id) errors.rs:25 */
#define DECDS_ERR_CHUNKSET_REPAIRING_FAILED 6      /* ChunksetRepairingFailed(id,msg) errors.rs:29 */
#define DECDS_ERR_INVALID_SHARE_ID 7               /* InvalidErasureCodedShareId(id)  errors.rs:32 */
#define DECDS_ERR_EMPTY_DATA_FOR_BLOB 8            /* EmptyDataForBlob                errors.rs:6  */
#define DECDS_ERR_INVALID_CHUNKSET_ID 9            /* InvalidChunksetId(id, n)        errors.rs:34 */
#define DECDS_ERR_CHUNKSET_ALREADY_REPAIRED 10     /* ChunksetAlreadyRepaired(id)     errors.rs:27 */
#define DECDS_ERR_INVALID_PROOF_IN_CHUNK 11        /* InvalidProofInChunk(id)         errors.rs:40 */
#define DECDS_ERR_BLOB_HEADER_SERIALIZATION_FAILED 12    /* BlobHeaderSerializationFailed     errors.rs:13 */
#define DECDS_ERR_BLOB_HEADER_DESERIALIZATION_FAILED 13  /* BlobHeaderDeserializationFailed   errors.rs:15 */
#define DECDS_ERR_PCC_SERIALIZATION_FAILED 14            /* ProofCarryingChunkSerializationFailed   errors.rs:18 */
#define DECDS_ERR_PCC_DESERIALIZATION_FAILED 15          /* ProofCarryingChunkDeserializationFailed errors.rs:20 */
#define DECDS_ERR_INVALID_START_BOUND 16           /* InvalidStartBound               errors.rs:8 (byte-range queries, host) */
#define DECDS_ERR_INVALID_END_BOUND 17             /* InvalidEndBound(end)            errors.rs:10 (byte-range queries, host) */
#define DECDS_ERR_HIP (-1)                         /* HIP runtime failure (text: decds_last_error) */
#define DECDS_ERR_INVALID_ARGUMENT (-2)
#define DECDS_ERR_NO_DEVICE (-3)
#define DECDS_ERR_OUT_OF_DEVICE_MEMORY (-4)        /* a device allocation the call cannot do without failed */

typedef struct decds_ctx decds_ctx;

/* ---- context ---------------------------------------------------------------------------- */
int decds_ctx_create(int device, decds_ctx **out);
int decds_ctx_destroy(decds_ctx *ctx);
/* GF(2^8) polynomial (with the x^8 bit, e.g. 0x11D) and boundary marker used by rlnc 0.4.0.
 * Defaults 0x11D / 0x81. Exposed so an identification run can re-pin them. The
 * polynomial must be irreducible (a reducible one is no field: DECDS_ERR_INVALID_ARGUMENT). */
int decds_ctx_set_field(decds_ctx *ctx, uint32_t poly, uint8_t marker);
int decds_ctx_get_field(const decds_ctx *ctx, uint32_t *poly, uint8_t *marker);
const char *decds_status_string(int status);
const char *decds_last_error(void); /* thread-local text of the last failure */
int decds_device_count(void);
/* Waits for the context's device and reports a pending (sticky) device fault as DECDS_ERR_HIP, so a
 * fault is attributed to the work that caused it, not to the next call that happens to sync. */
int decds_device_status(const decds_ctx *ctx);

/* ---- batch codec over device-resident chunksets (the hot path) ---------------------------- */
/* Replaces ChunkSet::new's RLNC part for a batch of chunksets: Encoder::new(data, 10)
 * (chunkset.rs:43) + 16 x Encoder::code(&mut rng) (chunkset.rs:45-52), as driven by the rayon
 * loop in Blob::new (blob.rs:256-264).
 *   src    : n x DECDS_CHUNKSET_BYTES (chunkset c at src + c*CS)
 *   coeffs : n x 16 x 10 coding vectors (row j of chunkset c at coeffs + (c*16+j)*10)
 *   dst    : n*16 coded rows; row r = c*16+j at dst + r*dst_pitch, laid out exactly like rlnc's
 *            full coded piece: coding vector (10 B) || payload (L B). dst_pitch >= 1,048,587 and
 *            15*dst_pitch + 1,048,587 < 2^31 (every pitch argument below: a chunkset's rows sit in
 *            one 2 GiB buffer descriptor). */
int decds_encode_batch(decds_ctx *ctx, const uint8_t *src, size_t n_chunksets,
                       const uint8_t *coeffs, uint8_t *dst, size_t dst_pitch, void *stream);

/* name of the gfx950 kernel decds_encode_batch launches for n chunksets (for profiles and traces:
 * the persistent, tile-counter-fed sweep, rlnc_encode_sweep_kernel) */
const char *decds_encode_kernel_name(size_t n_chunksets);

/* Replaces the incremental rank logic of RepairingChunkSet::add_chunk_unvalidated ->
 * Decoder::decode (chunkset.rs:173-184) and is_ready_to_repair (chunkset.rs:187-189) for a batch:
 *   cand     : n x 16 coded-row indices in arrival order, DECDS_NO_CANDIDATE-terminated
 *   plan     : n x DECDS_REPAIR_PLAN_BYTES (accepted rows + inverse coding matrix)
 *   verdicts : n x 16 per-candidate results: DECDS_OK (useful), DECDS_ERR_CHUNK_DECODING_FAILED
 *              (did not raise the rank), DECDS_ERR_CHUNKSET_READY_TO_REPAIR (arrived after rank 10),
 *              -1 (no candidate)
 *   status   : n x int32: DECDS_OK (rank 10) or DECDS_ERR_CHUNKSET_NOT_YET_READY */
int decds_repair_plan_batch(decds_ctx *ctx, const uint8_t *coded, size_t coded_pitch,
                            size_t n_chunksets, const uint8_t *cand, uint8_t *plan,
                            int8_t *verdicts, int32_t *status, void *stream);

/* What rlnc's Decoder::get_decoded_data returns for one chunkset (chunkset.rs:202-204): the 10
 * decoded pieces concatenated (CS + 10 bytes) cut at the LAST boundary marker. An intact chunkset
 * (any set of validated chunks) ends in marker || 9 zeros, so decoded_len == DECDS_CHUNKSET_BYTES;
 * rows accepted unvalidated (add_chunk_unvalidated) can move the cut: below CS (the vector is the
 * first decoded_len bytes of dst) or up to CS + 9 (dst's CS bytes, then tail[0 .. decoded_len - CS)).
 * No marker anywhere is DECDS_ERR_CHUNKSET_REPAIRING_FAILED. */
typedef struct decds_repair_info {
    uint32_t decoded_len;  /* length of get_decoded_data's vector, <= DECDS_DECODED_MAX_BYTES */
    uint8_t tail[10];      /* decoded bytes [CS, CS + 10): marker || zeros when intact */
    uint8_t reserved[2];
} decds_repair_info;
#define DECDS_DECODED_MAX_BYTES (DECDS_CHUNKSET_BYTES + DECDS_NUM_ORIGINAL_CHUNKS - 1ull)

/* Replaces RepairingChunkSet::repair -> Decoder::get_decoded_data (chunkset.rs:200-208):
 * dst = n x DECDS_CHUNKSET_BYTES (the first CS decoded bytes of chunkset c at dst + c*CS);
 * chunksets whose status is not DECDS_OK are skipped. info (n x decds_repair_info, 4-byte aligned,
 * or NULL) receives each decoded chunkset's cut; status becomes DECDS_ERR_CHUNKSET_REPAIRING_FAILED
 * when the decoded data holds no marker. */
int decds_decode_batch(decds_ctx *ctx, const uint8_t *coded, size_t coded_pitch,
                       size_t n_chunksets, const uint8_t *plan, uint8_t *dst, int32_t *status,
                       decds_repair_info *info, void *stream);

/* name of the gfx950 kernel decds_decode_batch launches for n chunksets (for profiles and traces):
 * rlnc_decode_sweep_kernel from DECDS_DEC_SWEEP_MIN_N chunksets on, rlnc_decode_kernel below */
const char *decds_decode_kernel_name(size_t n_chunksets);
/* Launch-shape thresholds, process-wide (every form gives identical bytes; these only pick the faster
 * kernel form per batch size): "DECDS_DEC_SWEEP_MIN_N" (default 1536: persistent decode sweep from
 * that many chunksets on), "DECDS_ENC_SMALL_MAX_N" (default 2: encode batches up to that many
 * chunksets run 8-column tiles, twice as many workgroups), "DECDS_ENC_NT_MIN_N" (default 256: from
 * that many chunksets on the encode stores its coded rows non-temporal, below write-through) and
 * "DECDS_PLAN_DECODE_MAX_N" (default 2: decds_repair_batch runs plan + decode as one kernel,
 * rlnc_plan_decode_kernel, up to that many chunksets) and "DECDS_DEC_NARROW_MAX_N" (default 2: the
 * one-tile decode, fused or not, runs 8-column tiles up to that many chunksets). Each starts from the environment variable
 * of its name (read once, at first use) or the default. set != 0 sets it (value UINT64_MAX: back to
 * that start value). Returns the value in force, UINT64_MAX for an unknown name. */
uint64_t decds_tuning(const char *name, uint64_t value, int set);

/* plan + decode in one call (the RepairingBlob::add_chunk loop + get_repaired_chunkset,
 * blob.rs:373-394, 451-473, for candidates already resident on the device); the same outputs as
 * decds_repair_plan_batch followed by decds_decode_batch — up to DECDS_PLAN_DECODE_MAX_N chunksets
 * in one kernel launch (each decode workgroup runs its chunkset's plan first) */
int decds_repair_batch(decds_ctx *ctx, const uint8_t *coded, size_t coded_pitch,
                       size_t n_chunksets, const uint8_t *cand, uint8_t *plan, int8_t *verdicts,
                       uint8_t *dst, int32_t *status, decds_repair_info *info, void *stream);
/* name of the first gfx950 kernel decds_repair_batch launches for n chunksets: rlnc_plan_decode_kernel
 * (plan and decode in one launch) up to DECDS_PLAN_DECODE_MAX_N, else rlnc_plan_kernel (then the
 * decds_decode_kernel_name kernel) */
const char *decds_repair_kernel_name(size_t n_chunksets);

/* Counter-based SplitMix64 byte stream (seeded, reproducible on host and device) for synthetic
 * blobs and coding vectors; byte p = byte (p%8) of mix64(seed + (p/8 + 1) * 0x9E3779B97F4A7C15). */
int decds_fill_random_device(decds_ctx *ctx, uint64_t seed, uint64_t byte_offset, uint8_t *dst,
                             size_t nbytes, void *stream);
void decds_fill_random_host(uint64_t seed, uint64_t byte_offset, uint8_t *dst, size_t nbytes);

/* Host-side rank step over a 10-byte coding vector (rlnc Decoder's "is this piece useful").
 * basis: 10x10 RREF rows, pivots: 10, *rank in/out. Returns 1 useful (basis updated), 0 not. */
int decds_rank_push(uint8_t *basis, uint8_t *pivots, uint32_t *rank, const uint8_t *coeff,
                    uint32_t poly);

/* ---- chunkset-level mirror (decds-lib/src/chunkset.rs), host buffers ----------------------- */
typedef struct decds_chunkset decds_chunkset;
/* ChunkSet::new(chunkset_id, data) (chunkset.rs:37-69): RLNC encode + the commitment (16 chunk
 * digests, Merkle root, 16 proofs) on the device. len != 10 MiB -> DECDS_ERR_INVALID_CHUNKSET_SIZE.
 * coeffs: 16 x 10 coding vectors, or NULL to draw them from the library's RNG (the reference
 * draws from rand::rng(), chunkset.rs:42). Thread-safe: concurrent callers (Blob::new's rayon
 * workers, blob.rs:256-264) each take one of the context's lanes (stream, device buffers,
 * page-locked staging; at most DECDS_MAX_LANES, default 8, further callers wait for one), or with
 * env DECDS_CHUNKSET_COALESCE=1 are gathered into shared fused encode + hashing launches. */
int decds_chunkset_new(decds_ctx *ctx, size_t chunkset_id, const uint8_t *data, size_t len,
                       const uint8_t *coeffs, decds_chunkset **out);
/* ChunkSet::get_root_commitment (chunkset.rs:72-74): 32-byte Merkle root of the 16 chunk digests */
int decds_chunkset_get_root_commitment(const decds_chunkset *cs, uint8_t out[32]);
/* the proof carried by ProofCarryingChunk `chunk_id` (chunkset.rs:59-63, 98-102): 4 chunkset-level
 * hashes, then the blob-level hashes appended by decds_chunkset_append_blob_inclusion_proof.
 * Writes *proof_len hashes (32 B each) if out_len allows, else DECDS_ERR_INVALID_ARGUMENT. */
int decds_chunkset_get_chunk_proof(const decds_chunkset *cs, size_t chunk_id, uint8_t *out, size_t out_len,
                                   size_t *proof_len);
/* ChunkSet::append_blob_inclusion_proof (chunkset.rs:98-102): appended to every chunk's proof */
int decds_chunkset_append_blob_inclusion_proof(decds_chunkset *cs, const uint8_t *blob_proof, size_t len);
/* ChunkSet::get_chunk (chunkset.rs:87-89): copies the 1,048,587-byte erasure-coded data of local
 * chunk `chunk_id`; *global_chunk_id = chunkset_id*16 + chunk_id (chunkset.rs:47) */
int decds_chunkset_get_chunk(const decds_chunkset *cs, size_t chunk_id, uint8_t *out,
                             size_t out_len, size_t *global_chunk_id);
size_t decds_chunkset_id(const decds_chunkset *cs);
void decds_chunkset_free(decds_chunkset *cs);

typedef struct decds_repairing_chunkset decds_repairing_chunkset;
/* RepairingChunkSet::new(chunkset_id, commitment) (chunkset.rs:129-135). commitment: the chunkset's
 * 32-byte root, used by decds_repairing_chunkset_add_chunk; may be NULL if only
 * add_chunk_unvalidated is used. */
int decds_repairing_chunkset_new(decds_ctx *ctx, size_t chunkset_id, const uint8_t *commitment,
                                 decds_repairing_chunkset **out);
/* RepairingChunkSet::add_chunk (chunkset.rs:151-157): the chunk (chunkset_id, global chunk_id,
 * data, proof) must prove inclusion in the commitment (chunk.rs:103-110: leaf chunk_id % 16, the
 * first 4 proof hashes, digest over the ids and data) or DECDS_ERR_INVALID_PROOF_IN_CHUNK;
 * otherwise exactly add_chunk_unvalidated. A proof of fewer than 4 hashes is invalid (the
 * reference's slice would panic). */
int decds_repairing_chunkset_add_chunk(decds_repairing_chunkset *rcs, size_t chunk_chunkset_id, size_t chunk_id,
                                       const uint8_t *data, size_t len, const uint8_t *proof, size_t proof_len);
/* RepairingChunkSet::add_chunk_unvalidated (chunkset.rs:173-184): chunk_chunkset_id is the
 * chunk's get_chunkset_id(); data/len its get_erasure_coded_data() */
int decds_repairing_chunkset_add_chunk_unvalidated(decds_repairing_chunkset *rcs,
                                                   size_t chunk_chunkset_id, const uint8_t *data,
                                                   size_t len);
/* RepairingChunkSet::is_ready_to_repair (chunkset.rs:187-189) */
int decds_repairing_chunkset_is_ready_to_repair(const decds_repairing_chunkset *rcs);
/* RepairingChunkSet::repair (chunkset.rs:200-208): out receives get_decoded_data's vector, *out_len
 * its length — 10 MiB for any validated chunk set; rows accepted unvalidated can move rlnc's cut at
 * the last boundary marker (decds_repair_info), up to DECDS_DECODED_MAX_BYTES. No marker ->
 * DECDS_ERR_CHUNKSET_REPAIRING_FAILED. out_cap below the decoded length -> DECDS_ERR_INVALID_ARGUMENT
 * with *out_len set and the decoder kept, its result too (a retry with a larger buffer only copies
 * it out: no second transfer or decode; the kept result is CS + 10 bytes of host memory held by the
 * object until the repair completes or the object is freed — without memory for it the retry
 * decodes again). Consumes the decoder state on success (a second call
 * returns DECDS_ERR_CHUNKSET_ALREADY_REPAIRED). */
int decds_repairing_chunkset_repair(decds_repairing_chunkset *rcs, uint8_t *out, size_t out_cap, size_t *out_len);
void decds_repairing_chunkset_free(decds_repairing_chunkset *rcs);

/* ---- blob-level batching (decds-lib/src/blob.rs), host buffers ----------------------------- */
/* Blob::new's chunkset loop (blob.rs:252-264): zero-pads blob to n = ceil(len/CS) chunksets and
 * encodes them in device batches of `batch` chunksets (0 = 16; 8-32 measured best) with H2D,
 * kernels and D2H on one stream each over three slots, so PCIe carries both directions at once;
 * the slot buffers stay in ctx across calls (calls on one ctx are serialised). Register the
 * caller buffers once (decds_host_register, or allocate them with decds_host_alloc) for the full
 * rate. coded_host: n*16 rows of 1,048,587 bytes. coeffs_host: n x 16 x 10. */
int decds_blob_encode_host(decds_ctx *ctx, const uint8_t *blob, size_t blob_len,
                           const uint8_t *coeffs_host, uint8_t *coded_host, size_t batch);
/* RepairingBlob add_chunk/get_repaired_chunkset over all chunksets (blob.rs:373-394, 451-473):
 * coded_host: n*16 rows; cand_host: n x 16 arrival order; out: blob_len bytes (last chunkset
 * truncated as blob.rs:464; chunksets that cannot be repaired are zero-filled); status_host: n
 * per-chunkset status. */
int decds_blob_repair_host(decds_ctx *ctx, const uint8_t *coded_host, size_t n_chunksets,
                           const uint8_t *cand_host, size_t blob_len, uint8_t *out,
                           int32_t *status_host, size_t batch);
/* The same over n_ctx contexts (devices): chunksets sharded by contiguous index range, one host
 * thread and stream set per context, no collective (chunksets are independent, blob.rs:256-264).
 * Identical output to the single-context calls. */
int decds_blob_encode_host_multi(decds_ctx *const *ctxs, size_t n_ctx, const uint8_t *blob, size_t blob_len,
                                 const uint8_t *coeffs_host, uint8_t *coded_host, size_t batch);
int decds_blob_repair_host_multi(decds_ctx *const *ctxs, size_t n_ctx, const uint8_t *coded_host,
                                 size_t n_chunksets, const uint8_t *cand_host, size_t blob_len, uint8_t *out,
                                 int32_t *status_host, size_t batch);

/* ---- Blob (blob.rs:227-318) ------------------------------------------------------------------ */
typedef struct decds_blob decds_blob;
/* Blob::new(data) (blob.rs:244-285): empty -> DECDS_ERR_EMPTY_DATA_FOR_BLOB; whole-blob BLAKE3
 * digest (from the device: 1 MiB groups hashed from each batch's uploaded inputs, folded on the host;
 * blobs up to 1 MiB on the host); every chunkset RLNC-encoded with its commitment (digests, root, proofs) on
 * the devices of ctxs (sharded as the _multi calls); blob-level Merkle tree over the chunkset roots
 * with each chunk's blob-level path appended to its proof. coeffs: n x 16 x 10 or NULL (drawn from
 * the library's RNG, as the reference draws from rand::rng()). */
int decds_blob_new(decds_ctx *const *ctxs, size_t n_ctx, const uint8_t *data, size_t len, const uint8_t *coeffs,
                   decds_blob **out);
/* Blob::get_blob_header (blob.rs:288-290): BlobHeader fields; *chunkset_roots points into the blob */
int decds_blob_get_header(const decds_blob *blob, uint64_t *byte_length, uint64_t *num_chunksets, uint8_t *digest,
                          uint8_t *root, const uint8_t **chunkset_roots);
/* hashes in every chunk's proof: 4 chunkset-level + ceil(log2(num_chunksets)) blob-level */
size_t decds_blob_proof_len(const decds_blob *blob);
/* chunk (chunkset_id, share_id) of the blob: *data -> its 1,048,587 coded bytes (inside the blob),
 * proof <- decds_blob_proof_len hashes; share_id >= 16 -> DECDS_ERR_INVALID_SHARE_ID */
int decds_blob_get_chunk(const decds_blob *blob, size_t chunkset_id, size_t share_id, const uint8_t **data,
                         uint8_t *proof, size_t proof_cap);
/* Blob::get_share (blob.rs:306-317): share share_id of every chunkset, data n x 1,048,587 bytes,
 * proofs n x proof_len x 32; share_id >= 16 -> DECDS_ERR_INVALID_SHARE_ID */
int decds_blob_get_share(const decds_blob *blob, size_t share_id, uint8_t *data, size_t data_cap, uint8_t *proofs,
                         size_t proofs_cap);
void decds_blob_free(decds_blob *blob);

/* ---- RepairingBlob (blob.rs:321-473) ---------------------------------------------------------- */
typedef struct decds_repairing_blob decds_repairing_blob;
/* RepairingBlob::new(header) (blob.rs:341-353) from the BlobHeader fields it uses, on one context */
int decds_repairing_blob_new(decds_ctx *ctx, uint64_t byte_length, uint64_t num_chunksets, const uint8_t *root,
                             const uint8_t *chunkset_roots, decds_repairing_blob **out);
/* the same over n_ctx contexts (devices): chunkset c belongs to context c / ceil(num_chunksets / n_ctx),
 * the contiguous chunkset-index shards of decds_blob_new; every call below routes to the chunkset's
 * context, and decds_repairing_blob_add_chunks validates each context's rows on its own device (one
 * host thread per context). Statuses and repaired bytes are identical to the one-context object.
 * Memory: accepted rows (10 x 1,048,587 B per chunkset, as the reference's decoder keeps them,
 * chunkset.rs:129-135) stay on the device while the context is under its device budget and spill to
 * page-locked host memory past it; a device allocation the call cannot do without fails with
 * DECDS_ERR_OUT_OF_DEVICE_MEMORY instead of a HIP error. Default budget per context: env
 * DECDS_RB_DEVICE_MB, else half the device's free memory at creation, split over the contexts that
 * share the device. */
int decds_repairing_blob_new_multi(decds_ctx *const *ctxs, size_t n_ctx, uint64_t byte_length, uint64_t num_chunksets,
                                   const uint8_t *root, const uint8_t *chunkset_roots, decds_repairing_blob **out);
/* device budget per context from now on (a quarter of it, at least one 20.5 MiB decode area, for
 * decoding; the rest for row slots); memory already held is kept */
int decds_repairing_blob_set_device_budget(decds_repairing_blob *rb, uint64_t bytes_per_context);
/* stats[0..n_stats) of: device bytes held, chunksets with rows on the device, chunksets with rows
 * spilled to host memory, host spill bytes held, decode areas, contexts */
int decds_repairing_blob_memory(const decds_repairing_blob *rb, uint64_t *stats, size_t n_stats);
/* RepairingBlob::add_chunk (blob.rs:373-394), in the reference's order: chunkset id out of range ->
 * DECDS_ERR_INVALID_CHUNKSET_ID; chunkset already repaired -> DECDS_ERR_CHUNKSET_ALREADY_REPAIRED;
 * BlobHeader::validate_chunk fails -> DECDS_ERR_INVALID_PROOF_IN_CHUNK; chunkset ready ->
 * DECDS_ERR_CHUNKSET_READY_TO_REPAIR; then add_chunk_unvalidated (a piece that does not raise the
 * rank -> DECDS_ERR_CHUNK_DECODING_FAILED). Accepted rows are kept on the device (or spilled, above). */
int decds_repairing_blob_add_chunk(decds_repairing_blob *rb, uint64_t chunkset_id, uint64_t chunk_id,
                                   const uint8_t *data, size_t len, const uint8_t *proof, size_t proof_len);
/* add_chunk for n_rows chunks in arrival order, validated as one device batch: ids n x (chunkset_id,
 * chunk_id), rows n x 1,048,587, proofs n x proof_len x 32; status[i] = what the i-th add_chunk call
 * would have returned. */
int decds_repairing_blob_add_chunks(decds_repairing_blob *rb, size_t n_rows, const uint64_t *ids, const uint8_t *rows,
                                    const uint8_t *proofs, size_t proof_len, int32_t *status);
/* RepairingBlob::is_chunkset_ready_to_repair / is_chunkset_already_repaired (blob.rs:407-430) */
int decds_repairing_blob_is_chunkset_ready_to_repair(const decds_repairing_blob *rb, size_t chunkset_id, int *out);
int decds_repairing_blob_is_chunkset_already_repaired(const decds_repairing_blob *rb, size_t chunkset_id, int *out);
/* RepairingBlob::get_repaired_chunkset (blob.rs:451-473): out receives get_chunkset_size(id) bytes
 * (*out_len); the chunkset is consumed (also when its repair fails, as blob.rs:458-462). Ready
 * chunksets are decoded in device batches: the first call decodes up to 64 ready chunksets at once
 * and later calls for those only copy out. */
int decds_repairing_blob_get_repaired_chunkset(decds_repairing_blob *rb, size_t chunkset_id, uint8_t *out,
                                               size_t out_cap, size_t *out_len);
void decds_repairing_blob_free(decds_repairing_blob *rb);

/* ---- commitment layer (next row: chunk digests + Merkle trees) ------------ */
/* ChunkSet::new's commitment for a batch (chunkset.rs:54-63): for coded row r = c*16+j,
 * digests[r] = Chunk::digest = BLAKE3(chunkset_id u64 LE || chunk_id u64 LE || row) (chunk.rs:40-46)
 * with chunkset_id = first_chunkset_id + c, chunk_id = chunkset_id*16 + j (chunkset.rs:47);
 * roots[c] = MerkleTree root of the 16 digests (merkle_tree.rs:23-50); proofs[(c*16+j)*4 + k] =
 * leaf j's 4-hash inclusion proof (merkle_tree.rs:75-116). Device pointers; 32-byte hashes. */
int decds_commit_batch(decds_ctx *ctx, const uint8_t *coded, size_t pitch, size_t n_chunksets,
                       uint64_t first_chunkset_id, uint8_t *digests, uint8_t *roots, uint8_t *proofs,
                       void *stream);
/* ChunkSet::new for a batch (chunkset.rs:37-63): decds_encode_batch + decds_commit_batch with the
 * same arguments and results, but when the coded rows are 16-byte aligned (dst and dst_pitch
 * multiples of 16, e.g. DECDS_CODED_PITCH_ALIGNED rows at DECDS_CODED_ROW_OFFSET_ALIGNED) the
 * commitment's chunk hashing runs inside the encode kernel, right behind each workgroup's row stores,
 * so the VALU-bound hashing overlaps the HBM-bound encode instead of re-reading every row afterwards
 * (DESIGN.md §5.4). workspace: device memory of decds_encode_commit_workspace_bytes(n) bytes (unused
 * on the unfused path, may then be NULL). */
size_t decds_encode_commit_workspace_bytes(size_t n_chunksets);
int decds_encode_commit_batch(decds_ctx *ctx, const uint8_t *src, size_t n_chunksets, const uint8_t *coeffs,
                              uint8_t *dst, size_t dst_pitch, uint64_t first_chunkset_id, uint8_t *digests,
                              uint8_t *roots, uint8_t *proofs, void *workspace, void *stream);
/* host helpers: BLAKE3 (crate blake3 as used by decds), the Merkle tree over arbitrary n leaves
 * with decds' zero-hash padding (blob-level tree, blob.rs:266-273) and proof verification
 * (merkle_tree.rs:131-146). decds_merkle_tree returns the proof depth (proofs: n x depth x 32). */
void decds_blake3(const uint8_t *data, size_t len, uint8_t out[32]);
/* Chunk::digest (chunk.rs:40-46) on the host: BLAKE3(chunkset_id u64 LE || chunk_id u64 LE || data) */
void decds_chunk_digest(uint64_t chunkset_id, uint64_t chunk_id, const uint8_t *data, size_t len, uint8_t out[32]);
int decds_merkle_tree(const uint8_t *leaves, size_t n, uint8_t root[32], uint8_t *proofs);
int decds_merkle_verify(size_t leaf_index, const uint8_t leaf[32], const uint8_t *proof, size_t proof_len,
                        const uint8_t root[32]);

/* ---- repair-side validation (next row) ---------------------------------------- */
/* BlobHeader::validate_chunk (blob.rs:211-215) for a batch of received chunks, all device pointers.
 * Row r (coded + r*pitch, 1,048,587 B) claims ids[2r] = chunkset_id and ids[2r+1] = global chunk_id,
 * and carries proofs[r*proof_len .. (r+1)*proof_len) (32-byte hashes: 4 chunkset-level, then the
 * blob-level ones). digests[r] = Chunk::digest of the row under its claimed ids. valid[r] = 1 iff
 *   (blob_root == NULL or MerkleTree::verify_proof(chunk_id, digest, proof, blob_root))   chunk.rs:88-90
 *   and chunkset_id < num_chunksets                                                        blob.rs:213
 *   and verify_proof(chunk_id % 16, digest, proof[0..4], chunkset_roots[chunkset_id])     chunk.rs:103-110
 * else 0; proof_len < 4 makes every row invalid. */
int decds_validate_batch(decds_ctx *ctx, const uint8_t *coded, size_t pitch, size_t n_rows, const uint64_t *ids,
                         const uint8_t *proofs, size_t proof_len, const uint8_t *chunkset_roots,
                         size_t num_chunksets, const uint8_t *blob_root, uint8_t *digests, uint8_t *valid,
                         void *stream);

/* ---- wire / on-disk format (next row): bincode 2 standard(), consts.rs:2 ----- */
/* ProofCarryingChunk::to_bytes / from_bytes (chunk.rs:152-170): varint chunkset_id, varint chunk_id,
 * varint data length + data, varint proof length + 32-byte hashes. from_bytes is zero-copy: *data
 * and *proof point into `bytes`; *consumed = bytes read (the file flow rejects trailing bytes,
 * decds-bin utils.rs:60-70). Truncated or malformed input -> DECDS_ERR_PCC_DESERIALIZATION_FAILED. */
size_t decds_pcc_encoded_len(uint64_t chunkset_id, uint64_t chunk_id, size_t data_len, size_t proof_len);
int decds_pcc_to_bytes(uint64_t chunkset_id, uint64_t chunk_id, const uint8_t *data, size_t data_len,
                       const uint8_t *proof, size_t proof_len, uint8_t *out, size_t cap, size_t *written);
int decds_pcc_from_bytes(const uint8_t *bytes, size_t len, uint64_t *chunkset_id, uint64_t *chunk_id,
                         const uint8_t **data, size_t *data_len, const uint8_t **proof, size_t *proof_len,
                         size_t *consumed);
/* BlobHeader::to_bytes / from_bytes (blob.rs:168-197): varint byte_length, varint num_chunksets,
 * digest, root commitment, varint count + chunkset roots; from_bytes also rejects
 * num_chunksets != count (blob.rs:187-191). */
size_t decds_blob_header_encoded_len(uint64_t byte_length, uint64_t num_chunksets, size_t n_roots);
int decds_blob_header_to_bytes(uint64_t byte_length, uint64_t num_chunksets, const uint8_t digest[32],
                               const uint8_t root[32], const uint8_t *chunkset_roots, size_t n_roots, uint8_t *out,
                               size_t cap, size_t *written);
int decds_blob_header_from_bytes(const uint8_t *bytes, size_t len, uint64_t *byte_length, uint64_t *num_chunksets,
                                 uint8_t digest[32], uint8_t root[32], const uint8_t **chunkset_roots, size_t *n_roots,
                                 size_t *consumed);
/* blake3::hash of a whole blob (Blob::new's header digest, blob.rs:249) with BLAKE3's subtrees
 * split over up to nthreads host threads (same result as decds_blake3) */
void decds_blake3_parallel(const uint8_t *data, size_t len, uint8_t out[32], int nthreads);
/* the same hash over consecutive pieces of one message (blake3::Hasher update / finalize): complete
 * power-of-two subtrees of each piece are hashed on up to nthreads host threads as they arrive,
 * at most one chunk is held back; finalize does not consume the stream (free it separately). Any
 * split of the message gives decds_blake3's result. */
typedef struct decds_blake3_stream decds_blake3_stream;
decds_blake3_stream *decds_blake3_stream_new(void);
void decds_blake3_stream_update(decds_blake3_stream *s, const uint8_t *data, size_t len, int nthreads);
void decds_blake3_stream_finalize(const decds_blake3_stream *s, uint8_t out[32]);
void decds_blake3_stream_free(decds_blake3_stream *s);

/* Page-lock a caller buffer once for many host calls (unregistered memory is staged through the
 * context's page-locked buffers instead). Registrations are refcounted per exact range; a range
 * that partially overlaps a registered one is refused; an unregister while a call still uses the
 * range takes effect when that call returns. Pair with decds_host_unregister before freeing. */
int decds_host_register(const void *ptr, size_t len);
int decds_host_unregister(const void *ptr);
/* page-locked host memory the host paths DMA directly (hipHostMalloc + the same registry). Blocks
 * of 64 MiB and more (the library's own, e.g. a Blob's coded store, and these) go to a cache when
 * freed — up to DECDS_PINNED_CACHE_MB (default 8192; the blocks cached longest are released to make
 * room for a newly freed one; all of them are freed when the last context is destroyed) — and serve
 * later requests of 80-100 % of their size without page-locking again (~0.25 s per GiB);
 * decds_host_cache_trim releases them and
 * returns the bytes released. Memory from the cache is not zeroed. */
int decds_host_alloc(size_t len, void **out);
int decds_host_free(void *ptr);
size_t decds_host_cache_trim(void);
/* 1 if [ptr, ptr+len) lies inside one registered or allocated range, else 0 */
int decds_host_is_registered(const void *ptr, size_t len);

#ifdef __cplusplus
}
#endif
#endif /* DECDS_RLNC_H */

/*
 * rlnc_oracle.h — CPU restatement of the RLNC arithmetic that decds-lib's chunkset path calls.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing under oracle/ is linked into, loaded by or called from the
 * product library (decds_amd/libdecds_rlnc.so). Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py use it, and only as the checker.
 *
 * What it restates (reference = /root/reference, itzmeanjan/decds @ 2025-07-18):
 *   - decds-lib/src/chunkset.rs:37-52   ChunkSet::new -> rlnc Encoder::new(data, 10) + 16x code()
 *   - decds-lib/src/chunkset.rs:117     PADDED_CHUNK_BYTE_LEN = ceil((CS + 1) / 10) = 1,048,577
 *   - decds-lib/src/chunkset.rs:129-208 RepairingChunkSet: Decoder::new / decode / is_already_decoded
 *                                       / get_decoded_data and their error mapping
 *   - the arithmetic of crate rlnc =0.4.0 (decds Cargo.lock:482-488, checksum 50c3be80...dcbb).
 *     That crate is NOT vendored in /root/reference and cannot be fetched here (no network,
 *     no cargo). Its behaviour is restated from its published design:
 *       * GF(2^8) with irreducible polynomial 0x11D (x^8+x^4+x^3+x^2+1)      [recalled]
 *       * Encoder::new appends one boundary-marker byte 0x81, zero-pads to k*L [L pinned by
 *         chunkset.rs:117; marker value recalled]
 *       * code(): full coded piece = coding_vector(k) || sum_i c_i * piece_i  [recalled]
 *       * Decoder: incremental reduced-row-echelon elimination; a piece that does not raise the
 *         rank is rejected ("not useful") and leaves the state unchanged    [recalled]
 *       * get_decoded_data(): concatenate the k solved payload rows, truncate at the LAST
 *         occurrence of the boundary marker                                 [recalled]
 *     Polynomial and marker are run-time parameters so the identification test can re-pin them.
 *
 * PARITY STATUS: coded-piece bytes are "parity unpinned" against the reference — the reference
 * ships no golden vectors and its arithmetic crate is absent. Repair output IS pinned by the
 * reference's own round-trip properties (chunkset.rs:257-283, tests.rs:4-57): decode(encode(x))
 * must equal x for any field/marker choice. See DESIGN.md "Oracle and parity".
 */
#ifndef DECDS_RLNC_ORACLE_H
#define DECDS_RLNC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_K 10u                    /* ChunkSet::NUM_ORIGINAL_CHUNKS, chunkset.rs:19 */
#define ORC_N 16u                    /* ChunkSet::NUM_ERASURE_CODED_CHUNKS, chunkset.rs:21 */
#define ORC_CS 10485760u             /* ChunkSet::BYTE_LENGTH = 10 * Chunk::BYTE_LENGTH, chunkset.rs:20 */
#define ORC_L 1048577u               /* RepairingChunkSet::PADDED_CHUNK_BYTE_LEN, chunkset.rs:117 */
#define ORC_F (ORC_L + ORC_K)        /* full coded piece: coding vector || payload */
#define ORC_POLY_DEFAULT 0x11Du
#define ORC_MARKER_DEFAULT 0x81u

/* status codes of the oracle decoder (names follow rlnc's error kinds) */
#define ORC_OK 0
#define ORC_ERR_PIECE_NOT_USEFUL 1
#define ORC_ERR_RECEIVED_ALL_PIECES 2
#define ORC_ERR_INVALID_PIECE_LENGTH 3
#define ORC_ERR_NOT_ALL_PIECES_RECEIVED 4
#define ORC_ERR_INVALID_DECODED_DATA 5
#define ORC_ERR_INVALID_CHUNKSET_SIZE 6
#define ORC_ERR_ARGS 7

uint8_t orc_gf256_mul(uint8_t a, uint8_t b, uint32_t poly);
/* 1: AVX2 nibble-table row kernels where the CPU has AVX2 (same bytes); returns the mode in effect */
int orc_set_simd(int on);
uint8_t orc_gf256_inv(uint8_t a, uint32_t poly);
/* full 256x256 product table, row-major: out[a*256+b] = a*b */
void orc_gf256_mul_table(uint32_t poly, uint8_t *out);

/* counter-based SplitMix64 byte stream: byte p = little-endian byte (p%8) of mix(seed + (p/8+1)*golden) */
uint64_t orc_splitmix64_word(uint64_t seed, uint64_t w);
void orc_fill_random(uint64_t seed, uint64_t byte_offset, uint8_t *out, size_t len);

/* rlnc Encoder::new: piece length L = ceil((len+1)/k); out must hold k*L bytes */
size_t orc_piece_len(size_t data_len, size_t k);
int orc_encoder_pad(const uint8_t *data, size_t len, size_t k, uint8_t marker, uint8_t *out);
/* rlnc Encoder::code with an explicit coding vector; out holds k + L bytes */
void orc_code_with_coding_vector(const uint8_t *padded, size_t piece_len, size_t k,
                                 const uint8_t *coding_vector, uint8_t *out_full_piece,
                                 uint32_t poly);
/* ChunkSet::new's RLNC part: data (len must be ORC_CS) + coeffs[16][10] -> out[16][ORC_F].
 * nthreads > 1 splits the 16 coded pieces over POSIX threads (cpu_baseline only). */
int orc_chunkset_encode(const uint8_t *data, size_t len, const uint8_t *coeffs, uint8_t *out,
                        uint32_t poly, uint8_t marker, int nthreads);

/* rlnc Decoder restatement */
typedef struct orc_decoder orc_decoder;
orc_decoder *orc_decoder_new(size_t piece_len, size_t k, uint32_t poly, uint8_t marker);
void orc_decoder_free(orc_decoder *d);
int orc_decoder_decode(orc_decoder *d, const uint8_t *full_piece, size_t len);
int orc_decoder_is_decoded(const orc_decoder *d);
size_t orc_decoder_rank(const orc_decoder *d);
/* writes at most cap bytes; *out_len = decoded length (rposition of the marker) */
int orc_decoder_get_decoded_data(const orc_decoder *d, uint8_t *out, size_t cap, size_t *out_len);

/* rank-tracking over coefficient vectors only (used to cross-check the product's host/device plan) */
int orc_rank_push(uint8_t *basis /* k*k, RREF rows */, uint8_t *pivots /* k */, size_t *rank,
                  const uint8_t *coeff, size_t k, uint32_t poly);

/* Gauss-Jordan inverse of a k x k matrix; returns 0 if invertible */
int orc_matrix_inverse(const uint8_t *m, uint8_t *inv, size_t k, uint32_t poly);

/* commitment layer (blake3_oracle.c): BLAKE3, Chunk::digest, MerkleTree root/proofs/verify */
void orc_blake3(const uint8_t *in, size_t len, uint8_t out[32]);
void orc_chunk_digest(uint64_t chunkset_id, uint64_t chunk_id, const uint8_t *data, size_t len, uint8_t out[32]);
void orc_chunk_digest_rows(const uint8_t *rows, size_t n_rows, size_t pitch, uint64_t first_row, uint8_t *out);
int orc_merkle(const uint8_t *leaves, size_t n, uint8_t root[32], uint8_t *proofs);
int orc_merkle_verify(size_t leaf_index, const uint8_t leaf[32], const uint8_t *proof, size_t plen,
                      const uint8_t root[32]);

#ifdef __cplusplus
}
#endif
#endif

// wire.cpp — decds' on-disk / wire format: bincode 2 `standard()` encoding
// (consts.rs:2) of ProofCarryingChunk (chunk.rs:152-170) and BlobHeader (blob.rs:168-197), as
// zero-copy host encoders/decoders.
//
// bincode 2 standard(): little endian, variable-length integers. A u64/usize v is one byte if
// v < 251, else a tag byte 251/252/253 followed by v as u16/u32/u64 LE. Structs are their fields
// in declaration order; Vec<T> is a varint length then the elements; u8 is one raw byte;
// blake3::Hash (serde derive over [u8; 32]) is its 32 bytes with no length prefix [recalled: the
// reference ships no serialized fixture, so the layout is pinned only by round trips].
//   ProofCarryingChunk = { chunk: { chunkset_id: usize, chunk_id: usize, erasure_coded_data: Vec<u8> },
//                          proof: Vec<blake3::Hash> }                                  chunk.rs:7-11, 51-55
//   BlobHeader = { byte_length: usize, num_chunksets: usize, digest: Hash, root_commitment: Hash,
//                  chunkset_root_commitments: Vec<Hash> }                                  blob.rs:15-21
#include <cstring>

#include "../../include/decds_rlnc.h"
#include "capi_internal.h"

namespace {

size_t varint_len(uint64_t v) { return v < 251 ? 1 : v <= 0xFFFF ? 3 : v <= 0xFFFFFFFFull ? 5 : 9; }

uint8_t *put_varint(uint8_t *p, uint64_t v) {
    if (v < 251) {
        *p++ = (uint8_t)v;
        return p;
    }
    const int n = v <= 0xFFFF ? 2 : v <= 0xFFFFFFFFull ? 4 : 8;
    *p++ = n == 2 ? 251 : n == 4 ? 252 : 253;
    for (int i = 0; i < n; i++) *p++ = (uint8_t)(v >> (8 * i));
    return p;
}

// false on truncation or a tag this format cannot hold in a usize (254 = u128, 255 invalid)
bool get_varint(const uint8_t *&p, const uint8_t *end, uint64_t &v) {
    if (p >= end) return false;
    const uint8_t t = *p++;
    if (t < 251) {
        v = t;
        return true;
    }
    const int n = t == 251 ? 2 : t == 252 ? 4 : t == 253 ? 8 : 0;
    if (!n || end - p < n) return false;
    v = 0;
    for (int i = 0; i < n; i++) v |= (uint64_t)p[i] << (8 * i);
    p += n;
    return true;
}

}  // namespace

extern "C" {

size_t decds_pcc_encoded_len(uint64_t chunkset_id, uint64_t chunk_id, size_t data_len, size_t proof_len) {
    return varint_len(chunkset_id) + varint_len(chunk_id) + varint_len(data_len) + data_len + varint_len(proof_len) +
           32 * proof_len;
}

int decds_pcc_to_bytes(uint64_t chunkset_id, uint64_t chunk_id, const uint8_t *data, size_t data_len,
                       const uint8_t *proof, size_t proof_len, uint8_t *out, size_t cap, size_t *written) {
    const size_t need = decds_pcc_encoded_len(chunkset_id, chunk_id, data_len, proof_len);
    if (!out || cap < need || (data_len && !data) || (proof_len && !proof))
        return decds_set_error(DECDS_ERR_PCC_SERIALIZATION_FAILED, "failed to serialize proof carrying chunk: %zu-byte buffer, %zu needed",
                               cap, need);
    uint8_t *p = put_varint(out, chunkset_id);
    p = put_varint(p, chunk_id);
    p = put_varint(p, data_len);
    if (data_len) std::memcpy(p, data, data_len);
    p = put_varint(p + data_len, proof_len);
    if (proof_len) std::memcpy(p, proof, 32 * proof_len);
    if (written) *written = need;
    return DECDS_OK;
}

int decds_pcc_from_bytes(const uint8_t *bytes, size_t len, uint64_t *chunkset_id, uint64_t *chunk_id,
                         const uint8_t **data, size_t *data_len, const uint8_t **proof, size_t *proof_len,
                         size_t *consumed) {
    const uint8_t *p = bytes, *end = bytes + (bytes ? len : 0);
    uint64_t cs = 0, ch = 0, dl = 0, pl = 0;
    bool ok = bytes && get_varint(p, end, cs) && get_varint(p, end, ch) && get_varint(p, end, dl) &&
              (uint64_t)(end - p) >= dl;
    const uint8_t *d = p;
    if (ok) p += dl;
    ok = ok && get_varint(p, end, pl) && pl <= (uint64_t)(end - p) / 32;
    if (!ok)
        return decds_set_error(DECDS_ERR_PCC_DESERIALIZATION_FAILED,
                               "failed to deserialize proof carrying chunk: unexpected end of input or invalid length");
    if (chunkset_id) *chunkset_id = cs;
    if (chunk_id) *chunk_id = ch;
    if (data) *data = d;
    if (data_len) *data_len = dl;
    if (proof) *proof = p;
    if (proof_len) *proof_len = pl;
    if (consumed) *consumed = (size_t)(p + 32 * pl - bytes);
    return DECDS_OK;
}

size_t decds_blob_header_encoded_len(uint64_t byte_length, uint64_t num_chunksets, size_t n_roots) {
    return varint_len(byte_length) + varint_len(num_chunksets) + 64 + varint_len(n_roots) + 32 * n_roots;
}

int decds_blob_header_to_bytes(uint64_t byte_length, uint64_t num_chunksets, const uint8_t digest[32],
                               const uint8_t root[32], const uint8_t *chunkset_roots, size_t n_roots, uint8_t *out,
                               size_t cap, size_t *written) {
    const size_t need = decds_blob_header_encoded_len(byte_length, num_chunksets, n_roots);
    if (!out || cap < need || !digest || !root || (n_roots && !chunkset_roots))
        return decds_set_error(DECDS_ERR_BLOB_HEADER_SERIALIZATION_FAILED, "failed to serialize blob header: %zu-byte buffer, %zu needed",
                               cap, need);
    uint8_t *p = put_varint(out, byte_length);
    p = put_varint(p, num_chunksets);
    std::memcpy(p, digest, 32);
    std::memcpy(p + 32, root, 32);
    p = put_varint(p + 64, n_roots);
    if (n_roots) std::memcpy(p, chunkset_roots, 32 * n_roots);
    if (written) *written = need;
    return DECDS_OK;
}

int decds_blob_header_from_bytes(const uint8_t *bytes, size_t len, uint64_t *byte_length, uint64_t *num_chunksets,
                                 uint8_t digest[32], uint8_t root[32], const uint8_t **chunkset_roots, size_t *n_roots,
                                 size_t *consumed) {
    const uint8_t *p = bytes, *end = bytes + (bytes ? len : 0);
    uint64_t bl = 0, nc = 0, nr = 0;
    bool ok = bytes && get_varint(p, end, bl) && get_varint(p, end, nc) && end - p >= 64;
    const uint8_t *h = p;
    if (ok) p += 64;
    ok = ok && get_varint(p, end, nr) && nr <= (uint64_t)(end - p) / 32;
    if (!ok)
        return decds_set_error(DECDS_ERR_BLOB_HEADER_DESERIALIZATION_FAILED,
                               "failed to deserialize blob header: unexpected end of input or invalid length");
    // blob.rs:187-191
    if (nc != nr)
        return decds_set_error(DECDS_ERR_BLOB_HEADER_DESERIALIZATION_FAILED, "number of chunksets and root commitments do not match");
    if (byte_length) *byte_length = bl;
    if (num_chunksets) *num_chunksets = nc;
    if (digest) std::memcpy(digest, h, 32);
    if (root) std::memcpy(root, h + 32, 32);
    if (chunkset_roots) *chunkset_roots = p;
    if (n_roots) *n_roots = nr;
    if (consumed) *consumed = (size_t)(p + 32 * nr - bytes);
    return DECDS_OK;
}

}  // extern "C"

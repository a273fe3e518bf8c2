/*
 * blake3_oracle.c — CPU restatement of the commitment layer around decds' chunkset codec.
 * TEST INFRASTRUCTURE ONLY (same rules as rlnc_oracle.h): used by tests/ as the checker of the
 * device commitment kernels, never linked into the product library.
 *
 * BLAKE3 (crate blake3 =1.8.2, decds Cargo.lock; not vendored here) restated from the published
 * BLAKE3 specification in the structure of its reference implementation: a chunk state that
 * compresses 64-byte blocks with CHUNK_START / CHUNK_END flags, and an incremental chaining-value
 * stack that merges completed subtrees (PARENT) and finalises the root with the ROOT flag.
 * Pinned by the specification's published known answers (tests/test_commit_cpu.py).
 *
 * decds usage restated:
 *   chunk.rs:40-46        Chunk::digest = BLAKE3(chunkset_id as u64 LE || chunk_id as u64 LE || data)
 *   merkle_tree.rs:23-50  MerkleTree::new: pairwise parents, odd node paired with a zero hash that
 *                         is itself re-hashed (z = H(z || z)) at every level
 *   merkle_tree.rs:75-116 generate_proof: sibling per level (the level's zero hash when missing)
 *   merkle_tree.rs:158-160 parent_hash = BLAKE3(left || right)
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "rlnc_oracle.h"

#define B3_OUT 32
#define B3_BLOCK 64
#define B3_CHUNK 1024
enum { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8 };

static const uint32_t IV[8] = {0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A,
                               0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19};
static const uint8_t PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};

static uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

static void g(uint32_t *s, int a, int b, int c, int d, uint32_t mx, uint32_t my) {
    s[a] = s[a] + s[b] + mx;
    s[d] = rotr(s[d] ^ s[a], 16);
    s[c] = s[c] + s[d];
    s[b] = rotr(s[b] ^ s[c], 12);
    s[a] = s[a] + s[b] + my;
    s[d] = rotr(s[d] ^ s[a], 8);
    s[c] = s[c] + s[d];
    s[b] = rotr(s[b] ^ s[c], 7);
}

static void compress(const uint32_t cv[8], const uint32_t block[16], uint64_t counter, uint32_t block_len,
                     uint32_t flags, uint32_t out[16]) {
    uint32_t s[16] = {cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7],
                      IV[0], IV[1], IV[2], IV[3], (uint32_t)counter, (uint32_t)(counter >> 32), block_len, flags};
    uint32_t m[16], t[16];
    memcpy(m, block, sizeof m);
    for (int r = 0; r < 7; r++) {
        g(s, 0, 4, 8, 12, m[0], m[1]);
        g(s, 1, 5, 9, 13, m[2], m[3]);
        g(s, 2, 6, 10, 14, m[4], m[5]);
        g(s, 3, 7, 11, 15, m[6], m[7]);
        g(s, 0, 5, 10, 15, m[8], m[9]);
        g(s, 1, 6, 11, 12, m[10], m[11]);
        g(s, 2, 7, 8, 13, m[12], m[13]);
        g(s, 3, 4, 9, 14, m[14], m[15]);
        if (r < 6) {
            for (int i = 0; i < 16; i++) t[i] = m[PERM[i]];
            memcpy(m, t, sizeof m);
        }
    }
    for (int i = 0; i < 8; i++) {
        out[i] = s[i] ^ s[i + 8];
        out[i + 8] = s[i + 8] ^ cv[i];
    }
}

static void words_from_bytes(const uint8_t *b, size_t len, uint32_t w[16]) {
    uint8_t blk[B3_BLOCK] = {0};
    memcpy(blk, b, len);
    for (int i = 0; i < 16; i++)
        w[i] = (uint32_t)blk[4 * i] | (uint32_t)blk[4 * i + 1] << 8 | (uint32_t)blk[4 * i + 2] << 16 |
               (uint32_t)blk[4 * i + 3] << 24;
}

/* ---- reference-implementation-shaped incremental hasher ---------------------------------------- */
struct output {
    uint32_t cv[8], block[16];
    uint64_t counter;
    uint32_t block_len, flags;
};

struct chunk_state {
    uint32_t cv[8];
    uint64_t counter;
    uint8_t block[B3_BLOCK];
    size_t block_len, blocks_compressed;
};

static void chunk_init(struct chunk_state *c, uint64_t counter) {
    memcpy(c->cv, IV, sizeof IV);
    c->counter = counter;
    c->block_len = 0;
    c->blocks_compressed = 0;
}

static size_t chunk_len(const struct chunk_state *c) { return B3_BLOCK * c->blocks_compressed + c->block_len; }
static uint32_t chunk_start_flag(const struct chunk_state *c) { return c->blocks_compressed == 0 ? CHUNK_START : 0; }

static void chunk_update(struct chunk_state *c, const uint8_t *in, size_t len) {
    while (len) {
        if (c->block_len == B3_BLOCK) {
            uint32_t w[16], o[16];
            words_from_bytes(c->block, B3_BLOCK, w);
            compress(c->cv, w, c->counter, B3_BLOCK, chunk_start_flag(c), o);
            memcpy(c->cv, o, 32);
            c->blocks_compressed++;
            c->block_len = 0;
        }
        size_t take = B3_BLOCK - c->block_len;
        if (take > len) take = len;
        memcpy(c->block + c->block_len, in, take);
        c->block_len += take;
        in += take;
        len -= take;
    }
}

static struct output chunk_output(const struct chunk_state *c) {
    struct output o;
    memcpy(o.cv, c->cv, 32);
    words_from_bytes(c->block, c->block_len, o.block);
    o.counter = c->counter;
    o.block_len = (uint32_t)c->block_len;
    o.flags = chunk_start_flag(c) | CHUNK_END;
    return o;
}

static void output_cv(const struct output *o, uint32_t cv[8]) {
    uint32_t t[16];
    compress(o->cv, o->block, o->counter, o->block_len, o->flags, t);
    memcpy(cv, t, 32);
}

static struct output parent_output(const uint32_t l[8], const uint32_t r[8]) {
    struct output o;
    memcpy(o.cv, IV, 32);
    memcpy(o.block, l, 32);
    memcpy(o.block + 8, r, 32);
    o.counter = 0;
    o.block_len = B3_BLOCK;
    o.flags = PARENT;
    return o;
}

void orc_blake3(const uint8_t *in, size_t len, uint8_t out[32]) {
    struct chunk_state c;
    uint32_t stack[64][8];
    int depth = 0;
    uint64_t chunks = 0;
    chunk_init(&c, 0);
    while (len) {
        if (chunk_len(&c) == B3_CHUNK) {
            uint32_t cv[8];
            struct output o = chunk_output(&c);
            output_cv(&o, cv);
            uint64_t total = ++chunks;
            /* merge completed subtrees: one merge per trailing zero bit of the chunk count */
            while ((total & 1) == 0) {
                struct output p = parent_output(stack[--depth], cv);
                output_cv(&p, cv);
                total >>= 1;
            }
            memcpy(stack[depth++], cv, 32);
            chunk_init(&c, chunks);
        }
        size_t take = B3_CHUNK - chunk_len(&c);
        if (take > len) take = len;
        chunk_update(&c, in, take);
        in += take;
        len -= take;
    }
    struct output o = chunk_output(&c);
    while (depth > 0) {
        uint32_t cv[8];
        output_cv(&o, cv);
        o = parent_output(stack[--depth], cv);
    }
    uint32_t w[16];
    compress(o.cv, o.block, o.counter, o.block_len, o.flags | ROOT, w);
    for (int i = 0; i < 8; i++)
        for (int b = 0; b < 4; b++) out[4 * i + b] = (uint8_t)(w[i] >> (8 * b));
}

/* chunk.rs:40-46 */
void orc_chunk_digest(uint64_t chunkset_id, uint64_t chunk_id, const uint8_t *data, size_t len, uint8_t out[32]) {
    uint8_t *buf = (uint8_t *)malloc(len + 16);
    for (int b = 0; b < 8; b++) {
        buf[b] = (uint8_t)(chunkset_id >> (8 * b));
        buf[8 + b] = (uint8_t)(chunk_id >> (8 * b));
    }
    memcpy(buf + 16, data, len);
    orc_blake3(buf, len + 16, out);
    free(buf);
}

/* chunk.rs:40-46 over n_rows coded rows at `pitch` bytes apart, each ORC_F bytes long: row r is chunk
 * first_row + r of chunkset (first_row + r) / 16 (chunkset.rs:47: chunk id = chunkset_id * 16 + i).
 * One thread; tests/fullcheck.py runs batches of rows on a thread pool. */
void orc_chunk_digest_rows(const uint8_t *rows, size_t n_rows, size_t pitch, uint64_t first_row, uint8_t *out) {
    for (size_t r = 0; r < n_rows; r++) {
        const uint64_t id = first_row + r;
        orc_chunk_digest(id / ORC_N, id, rows + r * pitch, ORC_F, out + 32 * r);
    }
}

/* merkle_tree.rs:158-160 */
static void parent_hash(const uint8_t *l, const uint8_t *r, uint8_t out[32]) {
    uint8_t b[64];
    memcpy(b, l, 32);
    memcpy(b + 32, r, 32);
    orc_blake3(b, 64, out);
}

/* merkle_tree.rs:23-50 (root) and 75-116 (proof of every leaf). proofs: n x depth x 32 where
 * depth = ceil(log2(n)) (n.next_power_of_two().ilog2()); returns depth, or -1 for n == 0. */
int orc_merkle(const uint8_t *leaves, size_t n, uint8_t root[32], uint8_t *proofs) {
    if (n == 0) return -1;
    int depth = 0;
    while (((size_t)1 << depth) < n) depth++;
    uint8_t *cur = (uint8_t *)malloc(n * 32), *nxt = (uint8_t *)malloc(n * 32 + 32);
    memcpy(cur, leaves, n * 32);
    size_t *idx = (size_t *)malloc(n * sizeof(size_t));
    for (size_t i = 0; i < n; i++) idx[i] = i;
    uint8_t zero[32] = {0};
    size_t len = n;
    for (int lvl = 0; len > 1; lvl++) {
        size_t plen = (len + 1) / 2;
        for (size_t p = 0; p < plen; p++) {
            const uint8_t *l = cur + 2 * p * 32;
            const uint8_t *r = 2 * p + 1 < len ? cur + (2 * p + 1) * 32 : zero;
            parent_hash(l, r, nxt + p * 32);
        }
        if (proofs)
            for (size_t i = 0; i < n; i++) {
                size_t s = idx[i] ^ 1;
                memcpy(proofs + (i * depth + lvl) * 32, s < len ? cur + s * 32 : zero, 32);
                idx[i] >>= 1;
            }
        uint8_t z2[32];
        parent_hash(zero, zero, z2);
        memcpy(zero, z2, 32);
        uint8_t *t = cur;
        cur = nxt;
        nxt = t;
        len = plen;
    }
    memcpy(root, cur, 32);
    free(cur);
    free(nxt);
    free(idx);
    return depth;
}

/* merkle_tree.rs:131-146 */
int orc_merkle_verify(size_t leaf_index, const uint8_t leaf[32], const uint8_t *proof, size_t plen,
                      const uint8_t root[32]) {
    uint8_t h[32], t[32];
    memcpy(h, leaf, 32);
    for (size_t k = 0; k < plen; k++) {
        if ((leaf_index & 1) == 0)
            parent_hash(h, proof + 32 * k, t);
        else
            parent_hash(proof + 32 * k, h, t);
        memcpy(h, t, 32);
        leaf_index >>= 1;
    }
    return memcmp(h, root, 32) == 0;
}

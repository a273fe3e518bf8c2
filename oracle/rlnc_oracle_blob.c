/*
 * rlnc_oracle_blob.c — blob-level restatement (chunkset fan-out + repair driver). TEST
 * INFRASTRUCTURE ONLY: the parity checker and bench.py's cpu_baseline leg ("kind": "port").
 *
 *   orc_blob_encode  follows decds-lib/src/blob.rs:244-264 (zero-pad to a multiple of CS, then
 *                    ChunkSet::new per chunkset on a thread pool — rayon's into_par_iter there).
 *   orc_blob_repair  follows blob.rs:373-394 + 451-473 and chunkset.rs:173-208: feed candidate
 *                    chunks in arrival order to a per-chunkset decoder, stop at rank k, extract
 *                    (cut at the last boundary marker), truncate to the chunkset's real size.
 */
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

#include "rlnc_oracle.h"

int orc_blob_encode(const uint8_t *blob, size_t blob_len, const uint8_t *coeffs, uint8_t *out,
                    uint32_t poly, uint8_t marker, int nthreads);
int orc_blob_repair(const uint8_t *coded, size_t n_chunksets, const uint8_t *cand,
                    size_t blob_len, uint8_t *out, int32_t *status, uint32_t poly, uint8_t marker,
                    int nthreads);

struct blob_job {
    const uint8_t *blob;
    size_t blob_len, n;
    const uint8_t *coeffs;
    const uint8_t *cand;
    const uint8_t *coded;
    uint8_t *out;
    int32_t *status;
    uint32_t poly;
    uint8_t marker;
    atomic_size_t next;
};

static void *encode_worker(void *arg) {
    struct blob_job *j = (struct blob_job *)arg;
    uint8_t *cs = (uint8_t *)malloc(ORC_CS);
    for (;;) {
        size_t c = atomic_fetch_add(&j->next, 1);
        if (c >= j->n) break;
        /* blob.rs:252-262: the zero-padded blob sliced into CS-byte chunksets */
        size_t off = c * (size_t)ORC_CS, have = j->blob_len - off;
        if (have > ORC_CS) have = ORC_CS;
        memcpy(cs, j->blob + off, have);
        memset(cs + have, 0, ORC_CS - have);
        orc_chunkset_encode(cs, ORC_CS, j->coeffs + c * ORC_N * ORC_K,
                            j->out + c * (size_t)ORC_N * ORC_F, j->poly, j->marker, 1);
    }
    free(cs);
    return NULL;
}

static void run_pool(struct blob_job *j, void *(*fn)(void *), int nthreads) {
    if (nthreads < 1) nthreads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, fn, j);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
}

int orc_blob_encode(const uint8_t *blob, size_t blob_len, const uint8_t *coeffs, uint8_t *out,
                    uint32_t poly, uint8_t marker, int nthreads) {
    if (blob_len == 0) return ORC_ERR_ARGS; /* blob.rs:245-247 EmptyDataForBlob */
    struct blob_job j;
    memset(&j, 0, sizeof(j));
    j.blob = blob;
    j.blob_len = blob_len;
    j.n = (blob_len + ORC_CS - 1) / ORC_CS;
    j.coeffs = coeffs;
    j.out = out;
    j.poly = poly;
    j.marker = marker;
    atomic_init(&j.next, 0);
    run_pool(&j, encode_worker, nthreads);
    return ORC_OK;
}

static void *repair_worker(void *arg) {
    struct blob_job *j = (struct blob_job *)arg;
    uint8_t *tmp = (uint8_t *)malloc((size_t)ORC_K * ORC_L);
    for (;;) {
        size_t c = atomic_fetch_add(&j->next, 1);
        if (c >= j->n) break;
        orc_decoder *d = orc_decoder_new(ORC_L, ORC_K, j->poly, j->marker);
        for (unsigned a = 0; a < ORC_N && !orc_decoder_is_decoded(d); a++) {
            uint8_t row = j->cand[c * ORC_N + a];
            if (row >= ORC_N) break;
            orc_decoder_decode(d, j->coded + (c * ORC_N + row) * (size_t)ORC_F, ORC_F);
        }
        size_t len = 0;
        int st = orc_decoder_is_decoded(d) ? orc_decoder_get_decoded_data(d, tmp, (size_t)ORC_K * ORC_L, &len)
                                           : ORC_ERR_NOT_ALL_PIECES_RECEIVED;
        if (st == ORC_OK) {
            /* blob.rs:464 truncates get_decoded_data's vector to the chunkset's real size (blob.rs:84-94);
             * a vector cut short (rows accepted unvalidated) leaves zeros up to it in this contiguous layout */
            size_t off = c * (size_t)ORC_CS, keep = j->blob_len - off;
            if (keep > ORC_CS) keep = ORC_CS;
            memcpy(j->out + off, tmp, len < keep ? len : keep);
            if (len < keep) memset(j->out + off + len, 0, keep - len);
        }
        j->status[c] = st;
        orc_decoder_free(d);
    }
    free(tmp);
    return NULL;
}

int orc_blob_repair(const uint8_t *coded, size_t n_chunksets, const uint8_t *cand,
                    size_t blob_len, uint8_t *out, int32_t *status, uint32_t poly, uint8_t marker,
                    int nthreads) {
    struct blob_job j;
    memset(&j, 0, sizeof(j));
    j.coded = coded;
    j.n = n_chunksets;
    j.cand = cand;
    j.blob_len = blob_len;
    j.out = out;
    j.status = status;
    j.poly = poly;
    j.marker = marker;
    atomic_init(&j.next, 0);
    run_pool(&j, repair_worker, nthreads);
    return ORC_OK;
}

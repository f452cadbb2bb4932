/*
 * ORACLE — test infrastructure only (tests/ and bench.py's post-run check).
 *
 * Per-pair reference results for a whole batch, on threads: score, end
 * states, panic status and the first printed alignment as run-length CIGAR
 * words, for every pair of a CSR batch.  Each pair is ref_nw_fill (the
 * literal three-matrix fill, needleman_wunsch_affine.rs:169-237) followed by
 * ref_nw_dag_summary (the order-preserving memoised restatement of the DFS,
 * :242-334), both in refcpu.c; this file only spreads pairs over threads and
 * packs the op string into the product's CIGAR word encoding
 * ((len << 4) | op, op: '=' 7, 'X' 8, 'I' 1, 'D' 2).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>

#include "refcpu.h"

typedef struct {
    const uint8_t *qs, *ds;
    const uint64_t *qo, *dof, *cig_off;
    int32_t *score;
    uint8_t *end_states, *panics;
    int32_t *cig_len;
    uint32_t *cig;
    uint64_t lo, hi;
    int failed;
} CheckSlice;

static uint32_t op_code(char c) {
    switch (c) {
    case '=': return 7;
    case 'X': return 8;
    case 'I': return 1;
    default: return 2;
    }
}

static void *check_worker(void *arg) {
    CheckSlice *s = (CheckSlice *)arg;
    for (uint64_t p = s->lo; p < s->hi; ++p) {
        const uint8_t *q = s->qs + s->qo[p], *d = s->ds + s->dof[p];
        const size_t lq = s->qo[p + 1] - s->qo[p], ld = s->dof[p + 1] - s->dof[p];
        ref_nw_mats m;
        if (ref_nw_fill(q, lq, d, ld, &m) != 0) {
            s->failed = 1;
            return NULL;
        }
        uint8_t es = 0;
        s->score[p] = ref_nw_score(&m, &es);
        s->end_states[p] = es;
        uint64_t nb = 0;
        int pan = 0;
        int64_t olen = -1;
        char *ops = (char *)malloc(lq + ld + 1);
        ref_nw_dag_summary(q, d, &m, &nb, &pan, ops, lq + ld + 1, &olen);
        s->panics[p] = (uint8_t)pan;
        int32_t nw = -1;
        if (olen >= 0) {
            uint32_t *out = s->cig + s->cig_off[p];
            nw = 0;
            for (int64_t k = 0; k < olen;) {
                int64_t e = k;
                while (e < olen && ops[e] == ops[k]) ++e;
                out[nw++] = ((uint32_t)(e - k) << 4) | op_code(ops[k]);
                k = e;
            }
        }
        s->cig_len[p] = nw;
        free(ops);
        ref_nw_free(&m);
    }
    return NULL;
}

/* cig_off[p] = first word of pair p in cig (caller sizes it lq + ld words per
 * pair at most); cig_len[p] = -1 when the reference prints nothing.
 * Returns 0, or -1 if an allocation failed. */
int ref_nw_check_pairs_mt(const uint8_t *qs, const uint64_t *q_off, const uint8_t *ds,
                          const uint64_t *d_off, uint64_t n_pairs, const uint64_t *cig_off,
                          int32_t *score, uint8_t *end_states, uint8_t *panics, int32_t *cig_len,
                          uint32_t *cig, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    CheckSlice sl[256];
    for (int t = 0; t < threads; ++t) {
        CheckSlice c = {qs, ds, q_off, d_off, cig_off, score, end_states, panics, cig_len, cig,
                        n_pairs * (uint64_t)t / (uint64_t)threads,
                        n_pairs * (uint64_t)(t + 1) / (uint64_t)threads, 0};
        sl[t] = c;
        pthread_create(&th[t], NULL, check_worker, &sl[t]);
    }
    int rc = 0;
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL);
        if (sl[t].failed) rc = -1;
    }
    return rc;
}

/*
 * ORACLE — test infrastructure only (tests/, bench cpu_baseline).
 *
 * Gap-affine minimum penalty of a global alignment, the quantity a correct
 * gap-affine WFA computes (a *corrected* WFA with the
 * reference's penalties x = 4 mismatch, o = 2 gap open, e = 6 gap extend,
 * src/wfa.rs:14-21; a gap of length L costs o + L*e).  The reference's own
 * wfa_align (src/wfa.rs:23-42) does not compute this value for realistic
 * inputs (it panics in Ocean::trim at s = 20), so this row is
 * "parity unpinned" against the reference: the oracle is the textbook
 * three-state DP (Gotoh 1982), linear memory, restated here:
 *
 *   E[i][j] = min(E[i][j-1] + e, H[i][j-1] + o + e)      gap in the query
 *   F[i][j] = min(F[i-1][j] + e, H[i-1][j] + o + e)      gap in the db
 *   H[i][j] = min(H[i-1][j-1] + x*[q_j != d_i], E[i][j], F[i][j])
 *   H[0][0] = 0, H[0][j] = E[0][j] = o + e*j, H[i][0] = F[i][0] = o + e*i
 *
 * (i over the db, j over the query, like the NW oracle.)
 */
#include <stdint.h>
#include <stdlib.h>
#include <pthread.h>

#define BIG (INT64_MAX / 4)

static int64_t min64(int64_t a, int64_t b) { return a < b ? a : b; }

int64_t ref_affine_penalty(const uint8_t *q, size_t lq, const uint8_t *d, size_t ld, int32_t x,
                           int32_t o, int32_t e) {
    if (lq == 0 && ld == 0) return 0;
    if (lq == 0) return (int64_t)o + (int64_t)e * (int64_t)ld;
    if (ld == 0) return (int64_t)o + (int64_t)e * (int64_t)lq;
    int64_t *H = malloc((lq + 1) * sizeof(int64_t));
    int64_t *F = malloc((lq + 1) * sizeof(int64_t));
    if (!H || !F) {
        free(H);
        free(F);
        return -1;
    }
    H[0] = 0;
    for (size_t j = 1; j <= lq; ++j) {
        H[j] = (int64_t)o + (int64_t)e * (int64_t)j;
        F[j] = BIG;
    }
    for (size_t i = 1; i <= ld; ++i) {
        int64_t diag = H[0];
        H[0] = (int64_t)o + (int64_t)e * (int64_t)i;
        int64_t E = BIG;
        const uint8_t di = d[i - 1];
        for (size_t j = 1; j <= lq; ++j) {
            E = min64(E + e, H[j - 1] + o + e);
            F[j] = min64(F[j] + e, H[j] + o + e);
            const int64_t m = diag + (q[j - 1] == di ? 0 : x);
            diag = H[j];
            H[j] = min64(m, min64(E, F[j]));
        }
    }
    const int64_t r = H[lq];
    free(H);
    free(F);
    return r;
}

/* Batch over (query, db) index pairs on `threads` POSIX threads (CPU
 * baseline of the corrected-WFA measurement). */
typedef struct {
    const uint8_t *qs, *ds;
    const uint64_t *qo, *dof;
    const uint32_t *pq, *pd;
    uint64_t n, next;
    int32_t x, o, e;
    int64_t *out;
    pthread_mutex_t mu;
} AffJob;

static void *aff_worker(void *arg) {
    AffJob *j = (AffJob *)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        const uint64_t k = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (k >= j->n) break;
        const uint32_t a = j->pq[k], b = j->pd[k];
        j->out[k] = ref_affine_penalty(j->qs + j->qo[a], j->qo[a + 1] - j->qo[a], j->ds + j->dof[b],
                                       j->dof[b + 1] - j->dof[b], j->x, j->o, j->e);
    }
    return NULL;
}

void ref_affine_run_pairs(const uint8_t *qs, const uint64_t *qo, const uint8_t *ds,
                          const uint64_t *dof, const uint32_t *pq, const uint32_t *pd, uint64_t n,
                          int32_t x, int32_t o, int32_t e, int threads, int64_t *out) {
    AffJob job = {qs, ds, qo, dof, pq, pd, n, 0, x, o, e, out, PTHREAD_MUTEX_INITIALIZER};
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, aff_worker, &job);
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
}

/*
 * ORACLE — test infrastructure only (bench.py's cpu_baseline leg).
 *
 * The reference's pair loop (src/main.rs:61-67) is sequential; SURVEY.md
 * §8(d) also asks for the CPU port on all host cores.  This runs
 * ref_nw_run_pairs (refcpu.c: literal fill + DFS per pair) over contiguous
 * slices of the pair list on POSIX threads; the per-pair work is unchanged.
 */
#include <pthread.h>
#include <stdint.h>

#include "refcpu.h"

typedef struct {
    const uint8_t *qs, *ds;
    const uint64_t *qo, *dof;
    uint64_t lo, hi, max_pops, max_blocks, cells, capped;
} MtSlice;

static void *mt_worker(void *arg) {
    MtSlice *s = (MtSlice *)arg;
    /* ref_nw_run_pairs indexes pair p by q_off[p] / d_off[p]: pass the
       slice's offsets (absolute into qs / ds) */
    s->cells = ref_nw_run_pairs_capped(s->qs, s->qo + s->lo, s->ds, s->dof + s->lo,
                                       s->hi - s->lo, s->max_pops, s->max_blocks, &s->capped);
    return NULL;
}

uint64_t ref_nw_run_pairs_mt_capped(const uint8_t *qs, const uint64_t *q_off, const uint8_t *ds,
                                    const uint64_t *d_off, uint64_t n_pairs, uint64_t max_pops,
                                    uint64_t max_blocks, int threads, uint64_t *capped) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    MtSlice sl[256];
    for (int t = 0; t < threads; ++t) {
        sl[t].qs = qs;
        sl[t].ds = ds;
        sl[t].qo = q_off;
        sl[t].dof = d_off;
        sl[t].lo = n_pairs * (uint64_t)t / (uint64_t)threads;
        sl[t].hi = n_pairs * (uint64_t)(t + 1) / (uint64_t)threads;
        sl[t].max_pops = max_pops;
        sl[t].max_blocks = max_blocks;
        sl[t].cells = 0;
        sl[t].capped = 0;
        pthread_create(&th[t], NULL, mt_worker, &sl[t]);
    }
    uint64_t cells = 0, nc = 0;
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL);
        cells += sl[t].cells;
        nc += sl[t].capped;
    }
    if (capped) *capped = nc;
    return cells;
}

uint64_t ref_nw_run_pairs_mt(const uint8_t *qs, const uint64_t *q_off, const uint8_t *ds,
                             const uint64_t *d_off, uint64_t n_pairs, uint64_t max_pops,
                             int threads) {
    return ref_nw_run_pairs_mt_capped(qs, q_off, ds, d_off, n_pairs, max_pops, 0, threads, NULL);
}

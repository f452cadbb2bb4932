/*
 * ORACLE — test infrastructure only (bench.py's cpu_baseline leg).
 *
 * The reference's pair loop (src/main.rs:61-67) is sequential; SURVEY.md
 * §8(d) also asks for the CPU port on all host cores.  This runs
 * ref_nw_run_pairs (refcpu.c: literal fill + DFS per pair) over contiguous
 * slices of the pair list on POSIX threads; the per-pair work is unchanged.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <string.h>

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

/* The same pair loop with the reference's text (TraceBackInfo Display,
 * needleman_wunsch_affine.rs:390-411, printed per block at :283-286) written
 * to `fd` in the reference's pair order (main.rs:61-74): bench.py's
 * text-inclusive CPU baseline for the drop-in CLI.  Pairs go through in
 * chunks of `chunk`: the threads take pairs one by one (their DFS cost varies
 * by orders of magnitude) and format each pair's blocks into its own buffer;
 * then the chunk's buffers are written in order.  Returns the cells; *bytes =
 * the text written, *capped = pairs whose DFS stopped at max_pops. */
#include <stdlib.h>
#include <unistd.h>

typedef struct {
    const uint8_t *qs, *ds;
    const uint64_t *qo, *dof;
    uint64_t base, n, max_pops, max_blocks;
    char **buf;
    size_t *len;
    uint64_t *next; /* shared: the chunk's next pair (atomic) */
    uint64_t capped;
} TxSlice;

static void *tx_worker(void *arg) {
    TxSlice *s = (TxSlice *)arg;
    size_t cap = 1 << 16;
    char *tmp = (char *)malloc(cap);
    for (;;) {
        const uint64_t i = __atomic_fetch_add(s->next, 1, __ATOMIC_RELAXED);
        if (i >= s->n) break;
        const uint64_t p = s->base + i;
        const uint8_t *q = s->qs + s->qo[p], *d = s->ds + s->dof[p];
        const size_t lq = s->qo[p + 1] - s->qo[p], ld = s->dof[p + 1] - s->dof[p];
        ref_nw_mats m;
        if (ref_nw_fill(q, lq, d, ld, &m) != 0) {
            s->len[i] = 0;
            s->buf[i] = NULL;
            continue;
        }
        size_t olen = 0;
        uint64_t nb = 0;
        int rc = ref_nw_traceback_dfs_blocks(q, d, &m, tmp, cap, &olen, s->max_pops, s->max_blocks, &nb);
        if (olen > cap) { /* the text outgrew the buffer: again with room for it */
            while (cap < olen) cap *= 2;
            free(tmp);
            tmp = (char *)malloc(cap);
            rc = ref_nw_traceback_dfs_blocks(q, d, &m, tmp, cap, &olen, s->max_pops, s->max_blocks, &nb);
        }
        if (rc == 2) ++s->capped;
        ref_nw_free(&m);
        s->buf[i] = (char *)malloc(olen ? olen : 1);
        memcpy(s->buf[i], tmp, olen);
        s->len[i] = olen;
    }
    free(tmp);
    return NULL;
}

uint64_t ref_nw_run_pairs_text_mt(const uint8_t *qs, const uint64_t *q_off, const uint8_t *ds,
                                  const uint64_t *d_off, uint64_t n_pairs, uint64_t max_pops,
                                  uint64_t max_blocks, int threads, int fd, uint64_t chunk,
                                  uint64_t *bytes, uint64_t *capped) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    if (chunk < 1) chunk = 4096;
    pthread_t th[256];
    TxSlice sl[256];
    char **buf = (char **)malloc(chunk * sizeof(char *));
    size_t *len = (size_t *)malloc(chunk * sizeof(size_t));
    uint64_t cells = 0, nb = 0, nc = 0;
    for (uint64_t base = 0; base < n_pairs; base += chunk) {
        const uint64_t n = n_pairs - base < chunk ? n_pairs - base : chunk;
        uint64_t next = 0;
        for (int t = 0; t < threads; ++t) {
            TxSlice s = {qs, ds, q_off, d_off, base, n, max_pops, max_blocks, buf, len, &next, 0};
            sl[t] = s;
            pthread_create(&th[t], NULL, tx_worker, &sl[t]);
        }
        for (int t = 0; t < threads; ++t) {
            pthread_join(th[t], NULL);
            nc += sl[t].capped;
        }
        for (uint64_t i = 0; i < n; ++i) {
            const uint64_t p = base + i;
            cells += (q_off[p + 1] - q_off[p]) * (d_off[p + 1] - d_off[p]);
            size_t off = 0;
            while (off < len[i]) {
                const ssize_t w = write(fd, buf[i] + off, len[i] - off);
                if (w <= 0) break;
                off += (size_t)w;
            }
            nb += len[i];
            free(buf[i]);
        }
    }
    free(buf);
    free(len);
    if (bytes) *bytes = nb;
    if (capped) *capped = nc;
    return cells;
}

/*
 * ORACLE — test infrastructure only (see refcpu.h).  Linear-memory restatement
 * of the reference NW-affine fill for pairs whose three full matrices do not
 * fit (100 kbp x 100 kbp is 3e10 Rc cells in the
 * reference).  Same recurrences and boundaries as ref_nw_fill
 * (needleman_wunsch_affine.rs:169-236, parent sets :96-153); instead of the
 * parent lists each (cell, state) carries one bit: "a reference panic node
 * (D[0][j>=1] :299, I[i>=1][0] :303) is reachable from here through parent
 * pointers", OR-ed over the parents that tie the maximum.  Because the DFS
 * (:246-329) visits every node reachable from the end states unless it panics
 * first, the pair panics iff that bit is set on an end state (the same
 * statement ref_nw_dag_summary makes with its explicit DAG).
 *
 * Parallel form: the query columns are cut into T stripes, one thread each;
 * stripe t consumes the (M, I, D, bits) of the column left of it row by row
 * as stripe t-1 publishes them (a pipeline down the rows).
 *
 * ref_nw_first_linear additionally keeps every cell's parent sets (one byte:
 * the refcpu.h pM / pI / pD bits, 1 B per cell, 10 GB at configs[3]) and runs
 * the reference DFS (:246-329) over them with a "no terminal below" memo per
 * (cell, state): the first event in DFS order (a printed block at the origin,
 * or a boundary panic) and the first printed alignment, for pairs whose
 * three full i32 matrices would not fit (ref_nw_dag_summary's statement).
 */
#define _POSIX_C_SOURCE 200809L
#include "refcpu.h"

#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

#define GO (-8)
#define GE (-6)
#define MIS (-4)
#define MAT 5

typedef struct {
    int32_t m, i, d;
    uint8_t f; /* bit0 M, bit1 I, bit2 D: panic reachable */
} lin_cell;

typedef struct {
    const uint8_t *q, *d;
    size_t lq, ld;
    int nt;
    size_t w;               /* stripe width */
    lin_cell **col;         /* col[t][i]: column c0(t)-1 at row i, written by stripe t-1 */
    _Atomic size_t *prog;   /* prog[t]: rows of col[t] published */
    lin_cell end;           /* (ld, lq) */
    uint8_t *codes;         /* optional: parent sets per cell, row-major (ld+1) x (lq+1) */
} lin_job;

typedef struct {
    lin_job *job;
    int t;
} lin_arg;

static inline int32_t mx2(int32_t a, int32_t b) { return a > b ? a : b; }

/* column 0 at row i (:200-216), origin (:172-182) */
static lin_cell col0(size_t i) {
    lin_cell c;
    if (i == 0) {
        c.m = 0;
        c.i = REF_SENTINEL;
        c.d = REF_SENTINEL;
        c.f = 0;
    } else {
        c.m = REF_SENTINEL;
        c.i = GO + ((int32_t)i + 1) * GE;
        c.d = REF_SENTINEL;
        c.f = 2; /* I[i>=1][0] is itself a panic node */
    }
    return c;
}

static void *lin_stripe(void *vp) {
    lin_arg *a = (lin_arg *)vp;
    lin_job *J = a->job;
    const int t = a->t;
    const size_t c0 = 1 + (size_t)t * J->w;
    size_t c1 = c0 + J->w;
    if (c1 > J->lq + 1) c1 = J->lq + 1;
    const size_t n = c1 - c0;
    lin_cell *prev = (lin_cell *)malloc((n + 1) * sizeof(lin_cell));
    lin_cell *cur = (lin_cell *)malloc((n + 1) * sizeof(lin_cell));
    lin_cell *left = t ? J->col[t] : NULL;
    lin_cell *out = (t + 1 < J->nt) ? J->col[t + 1] : NULL;
    /* row 0 (:183-199): M = I = sentinel, D[0][j] = GO + (j+1) GE, a panic node */
    size_t avail = 0;
    if (t) {
        while ((avail = atomic_load_explicit(&J->prog[t], memory_order_acquire)) < 1) sched_yield();
        prev[0] = left[0];
    } else {
        prev[0] = col0(0);
    }
    for (size_t k = 0; k < n; ++k) {
        const size_t j = c0 + k;
        prev[k + 1].m = REF_SENTINEL;
        prev[k + 1].i = REF_SENTINEL;
        prev[k + 1].d = ((int32_t)j + 1) * GE + GO;
        prev[k + 1].f = 4;
    }
    if (out) {
        out[0] = prev[n];
        atomic_store_explicit(&J->prog[t + 1], 1, memory_order_release);
    }
    for (size_t i = 1; i <= J->ld; ++i) {
        if (t) {
            while (avail <= i) {
                avail = atomic_load_explicit(&J->prog[t], memory_order_acquire);
                if (avail <= i) sched_yield();
            }
            cur[0] = left[i];
        } else {
            cur[0] = col0(i);
        }
        const uint8_t di = J->d[i - 1];
        for (size_t k = 1; k <= n; ++k) {
            const int32_t s = (J->q[c0 + k - 2] == di) ? MAT : MIS;
            const lin_cell dg = prev[k - 1], up = prev[k], lf = cur[k - 1];
            lin_cell c;
            /* m_score :76-86 / m_pointer :120-153 */
            c.m = mx2(mx2(dg.m, dg.i), dg.d) + s;
            uint8_t f = 0;
            if (c.m == dg.m + s && (dg.f & 1)) f |= 1;
            if (c.m == dg.i + s && (dg.f & 2)) f |= 1;
            if (c.m == dg.d + s && (dg.f & 4)) f |= 1;
            /* i_score :91-94 / i_pointer :108-119 */
            c.i = mx2(lf.m + GO, lf.i) + GE;
            if (c.i == lf.i + GE && (lf.f & 2)) f |= 2;
            if (c.i == lf.m + GO + GE && (lf.f & 1)) f |= 2;
            /* d_score :87-90 / d_pointer :96-107 */
            c.d = mx2(up.m + GO, up.d) + GE;
            if (c.d == up.d + GE && (up.f & 4)) f |= 4;
            if (c.d == up.m + GO + GE && (up.f & 1)) f |= 4;
            c.f = f;
            cur[k] = c;
            if (J->codes) { /* refcpu.h bit conventions, push order */
                uint8_t b = 0;
                if (c.m == dg.m + s) b |= 1;
                if (c.m == dg.i + s) b |= 2;
                if (c.m == dg.d + s) b |= 4;
                if (c.i == lf.i + GE) b |= 8;
                if (c.i == lf.m + GO + GE) b |= 16;
                if (c.d == up.d + GE) b |= 32;
                if (c.d == up.m + GO + GE) b |= 64;
                J->codes[i * (J->lq + 1) + c0 + k - 1] = b;
            }
        }
        if (out) {
            out[i] = cur[n];
            if ((i & 31) == 0 || i == J->ld)
                atomic_store_explicit(&J->prog[t + 1], i + 1, memory_order_release);
        }
        lin_cell *tmp = prev;
        prev = cur;
        cur = tmp;
    }
    if (t + 1 == J->nt) J->end = prev[n];
    free(prev);
    free(cur);
    return NULL;
}

static int lin_run(lin_job *Jp, const uint8_t *q, size_t lq, const uint8_t *d, size_t ld,
                   int threads, uint8_t *codes, int32_t *score, uint8_t *end_states, int *panics) {
    lin_job J;
    memset(&J, 0, sizeof(J));
    J.q = q;
    J.d = d;
    J.lq = lq;
    J.ld = ld;
    J.codes = codes;
    if (codes) { /* boundary parent sets (:183-216): D[0][j] <- D[0][j-1], I[i][0] <- I[i-1][0] */
        codes[0] = 0;
        for (size_t j = 1; j <= lq; ++j) codes[j] = 32;
        for (size_t i = 1; i <= ld; ++i) codes[i * (lq + 1)] = 8;
    }
    if (threads < 1) threads = 1;
    size_t w = (lq + (size_t)threads - 1) / (size_t)threads;
    if (w < 256) w = 256;
    int nt = lq ? (int)((lq + w - 1) / w) : 1;
    J.nt = nt;
    J.w = w;
    lin_cell end;
    if (lq == 0) {
        end = col0(ld);
    } else {
        J.col = (lin_cell **)calloc((size_t)nt, sizeof(lin_cell *));
        J.prog = (_Atomic size_t *)calloc((size_t)nt + 1, sizeof(_Atomic size_t));
        for (int t = 1; t < nt; ++t) {
            J.col[t] = (lin_cell *)malloc((ld + 1) * sizeof(lin_cell));
            if (!J.col[t]) return -1;
            atomic_init(&J.prog[t], 0);
        }
        pthread_t *th = (pthread_t *)calloc((size_t)nt, sizeof(pthread_t));
        lin_arg *args = (lin_arg *)calloc((size_t)nt, sizeof(lin_arg));
        for (int t = 0; t < nt; ++t) {
            args[t].job = &J;
            args[t].t = t;
            pthread_create(&th[t], NULL, lin_stripe, &args[t]);
        }
        for (int t = 0; t < nt; ++t) pthread_join(th[t], NULL);
        for (int t = 1; t < nt; ++t) free(J.col[t]);
        free(J.col);
        free((void *)J.prog);
        free(th);
        free(args);
        end = J.end;
    }
    /* end states :247-280; the DFS pops D, M, I and panics if any reaches a panic node */
    const int32_t h = mx2(mx2(end.i, end.d), end.m);
    uint8_t e = 0;
    int pan = 0;
    if (end.m == h) e |= 1, pan |= end.f & 1;
    if (end.i == h) e |= 2, pan |= (end.f >> 1) & 1;
    if (end.d == h) e |= 4, pan |= (end.f >> 2) & 1;
    *score = h;
    *end_states = e;
    *panics = pan;
    if (Jp) *Jp = J;
    return 0;
}

int ref_nw_score_linear(const uint8_t *q, size_t lq, const uint8_t *d, size_t ld, int threads,
                        int32_t *score, uint8_t *end_states, int *panics) {
    return lin_run(NULL, q, lq, d, ld, threads, NULL, score, end_states, panics);
}

/* ---- the reference DFS over stored parent sets, first event only ---- */
enum { LS_M = 0, LS_I = 1, LS_D = 2 };
typedef struct {
    uint32_t x, y;
    uint8_t st, np, next;
    uint8_t ps[3];
} lin_frame;

/* parents of (st, x, y) in pop order (reverse of the push order :287-328) */
static int lin_parents(const uint8_t *codes, size_t W, int st, size_t x, size_t y, uint8_t *ps) {
    const uint8_t b = codes[x * W + y];
    int n = 0;
    if (st == LS_M) { /* push M, I, D (:120-153) -> pop D, I, M */
        if (b & 4) ps[n++] = LS_D;
        if (b & 2) ps[n++] = LS_I;
        if (b & 1) ps[n++] = LS_M;
    } else if (st == LS_I) { /* push ext (I), open (M) (:108-119) -> pop open first */
        if (b & 16) ps[n++] = LS_M;
        if (b & 8) ps[n++] = LS_I;
    } else { /* push ext (D), open (M) (:96-107) */
        if (b & 64) ps[n++] = LS_M;
        if (b & 32) ps[n++] = LS_D;
    }
    return n;
}

int ref_nw_first_linear(const uint8_t *q, size_t lq, const uint8_t *d, size_t ld, int threads,
                        int32_t *score, uint8_t *end_states, int *panics, char *ops,
                        size_t ops_cap, int64_t *ops_len, uint64_t *dead_nodes) {
    const size_t W = lq + 1, n = (ld + 1) * W;
    uint8_t *codes = (uint8_t *)malloc(n);
    uint8_t *dead = (uint8_t *)calloc(n, 1); /* bit st: (cell, st) explored, no terminal */
    lin_frame *stk = (lin_frame *)malloc((lq + ld + 2) * sizeof(lin_frame));
    if (!codes || !dead || !stk) {
        free(codes);
        free(dead);
        free(stk);
        return -1;
    }
    int rc = lin_run(NULL, q, lq, d, ld, threads, codes, score, end_states, panics);
    *ops_len = -1;
    uint64_t ndead = 0;
    if (rc == 0) {
        const uint8_t es = *end_states;
        const int order[3] = {LS_D, LS_M, LS_I}; /* end states pop order (:251-280) */
        const uint8_t bit[3] = {4, 1, 2};
        int found = 0; /* 1 origin, 2 panic */
        size_t top = 0;
        for (int e = 0; e < 3 && !found; ++e) {
            if (!(es & bit[e])) continue;
            top = 0;
            lin_frame f0 = {(uint32_t)ld, (uint32_t)lq, (uint8_t)order[e], 0, 0, {0, 0, 0}};
            f0.np = 255; /* not yet visited */
            stk[top++] = f0;
            while (top && !found) {
                lin_frame *f = &stk[top - 1];
                if (f->np == 255) { /* first visit (:282-303) */
                    const size_t x = f->x, y = f->y;
                    if (x == 0 && y == 0) { found = 1; break; } /* printed block :283-286 */
                    if (dead[x * W + y] & (1u << f->st)) { --top; continue; }
                    f->np = (uint8_t)lin_parents(codes, W, f->st, x, y, f->ps);
                    f->next = 0;
                    /* a boundary parent access panics (:299 seq2[x-1], :303 seq1[y-1]) */
                    const int bad = f->st == LS_M ? (x == 0 || y == 0)
                                  : f->st == LS_D ? x == 0 : y == 0;
                    if (f->np && bad) { found = 2; break; }
                }
                if (f->next < f->np) {
                    const uint8_t ps = f->ps[f->next++];
                    lin_frame c = {f->x, f->y, ps, 255, 0, {0, 0, 0}};
                    if (f->st == LS_M) { c.x -= 1; c.y -= 1; }
                    else if (f->st == LS_I) c.y -= 1;
                    else c.x -= 1;
                    stk[top++] = c;
                } else {
                    dead[(size_t)f->x * W + f->y] |= (uint8_t)(1u << f->st);
                    ++ndead;
                    --top;
                }
            }
        }
        if (found == 1) { /* stack bottom = end cell = last column; the origin frame on top */
            const size_t len = top - 1;
            for (size_t k = 0; k < len && k < ops_cap; ++k) {
                const lin_frame *f = &stk[len - 1 - k];
                ops[k] = f->st == LS_M ? (q[f->y - 1] == d[f->x - 1] ? '=' : 'X')
                       : f->st == LS_I ? 'I' : 'D';
            }
            *ops_len = (int64_t)len;
        }
    }
    if (dead_nodes) *dead_nodes = ndead;
    free(codes);
    free(dead);
    free(stk);
    return rc;
}

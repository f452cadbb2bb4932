/*
 * ORACLE — test infrastructure only (see refcpu.h).  Literal CPU restatement
 * of the reference's NW-affine fill/traceback and FASTA parser.  Every
 * function cites the reference lines it follows.  Release-mode semantics
 * (README.md:8 runs `cargo run --release`): i32 arithmetic, index panics.
 */
#include "refcpu.h"

#include <stdlib.h>
#include <string.h>

/* SCHEME, needleman_wunsch_affine.rs:15-20 */
#define GO (-8)
#define GE (-6)
#define MIS (-4)
#define MAT 5

enum { ST_M = 0, ST_I = 1, ST_D = 2 }; /* State, :365-371 */

static inline int32_t max2(int32_t a, int32_t b) { return a > b ? a : b; }

int ref_nw_fill(const uint8_t *q, size_t lq, const uint8_t *d, size_t ld, ref_nw_mats *o) {
    const size_t W = lq + 1, H = ld + 1, n = W * H;
    memset(o, 0, sizeof(*o));
    o->lq = lq;
    o->ld = ld;
    o->M = (int32_t *)calloc(n, 4);
    o->I = (int32_t *)calloc(n, 4);
    o->D = (int32_t *)calloc(n, 4);
    o->pM = (uint8_t *)calloc(n, 1);
    o->pI = (uint8_t *)calloc(n, 1);
    o->pD = (uint8_t *)calloc(n, 1);
    if (!o->M || !o->I || !o->D || !o->pM || !o->pI || !o->pD) {
        ref_nw_free(o);
        return -1;
    }
#define IX(x, y) ((size_t)(x) * W + (size_t)(y))
    /* origin, :172-182 */
    o->M[IX(0, 0)] = 0;
    o->D[IX(0, 0)] = REF_SENTINEL;
    o->I[IX(0, 0)] = REF_SENTINEL;
    /* row x = 0 over the query, :183-199 */
    for (size_t i = 1; i <= lq; ++i) {
        o->M[IX(0, i)] = REF_SENTINEL;
        o->I[IX(0, i)] = REF_SENTINEL;
        o->D[IX(0, i)] = ((int32_t)i + 1) * GE + GO;
        o->pD[IX(0, i)] = 1; /* parent D[0][i-1] */
    }
    /* column y = 0 over the db, :200-216 */
    for (size_t i = 1; i <= ld; ++i) {
        o->M[IX(i, 0)] = REF_SENTINEL;
        o->I[IX(i, 0)] = GO + ((int32_t)i + 1) * GE;
        o->pI[IX(i, 0)] = 1; /* parent I[i-1][0] */
        o->D[IX(i, 0)] = REF_SENTINEL;
    }
    /* main loop :217-236, db outer (x = i), query inner (y = j) */
    for (size_t i = 1; i <= ld; ++i) {
        for (size_t j = 1; j <= lq; ++j) {
            const int32_t s = (q[j - 1] == d[i - 1]) ? MAT : MIS;
            /* m_score :76-86 and m_pointer :120-153 */
            const int32_t pm = o->M[IX(i - 1, j - 1)], pi = o->I[IX(i - 1, j - 1)],
                          pd = o->D[IX(i - 1, j - 1)];
            const int32_t m = max2(max2(pm, pi), pd) + s;
            uint8_t bm = 0;
            if (m == pm + s) bm |= 1;
            if (m == pi + s) bm |= 2;
            if (m == pd + s) bm |= 4;
            o->M[IX(i, j)] = m;
            o->pM[IX(i, j)] = bm;
            /* i_score :91-94 and i_pointer :108-119 (uses M[i][j-1]) */
            const int32_t lm = o->M[IX(i, j - 1)], li = o->I[IX(i, j - 1)];
            const int32_t iv = max2(lm + GO, li) + GE;
            uint8_t bi = 0;
            if (iv == li + GE) bi |= 1;
            if (iv == lm + GO + GE) bi |= 2;
            o->I[IX(i, j)] = iv;
            o->pI[IX(i, j)] = bi;
            /* d_score :87-90 and d_pointer :96-107 (uses row i-1) */
            const int32_t um = o->M[IX(i - 1, j)], ud = o->D[IX(i - 1, j)];
            const int32_t dv = max2(um + GO, ud) + GE;
            uint8_t bd = 0;
            if (dv == ud + GE) bd |= 1;
            if (dv == um + GO + GE) bd |= 2;
            o->D[IX(i, j)] = dv;
            o->pD[IX(i, j)] = bd;
        }
    }
    return 0;
}

void ref_nw_free(ref_nw_mats *m) {
    free(m->M);
    free(m->I);
    free(m->D);
    free(m->pM);
    free(m->pI);
    free(m->pD);
    memset(m, 0, sizeof(*m));
}

void ref_nw_dense_mask(const ref_nw_mats *m, uint8_t *out) {
    const size_t W = m->lq + 1, H = m->ld + 1;
    for (size_t k = 0; k < W * H; ++k) {
        const int32_t h = max2(max2(m->M[k], m->I[k]), m->D[k]);
        uint8_t b = 0;
        if (m->M[k] == h) b |= 1;
        if (m->I[k] == h) b |= 2;
        if (m->D[k] == h) b |= 4;
        b |= (uint8_t)((m->pI[k] & 3) << 3);
        b |= (uint8_t)((m->pD[k] & 3) << 5);
        out[k] = b;
    }
}

int32_t ref_nw_score(const ref_nw_mats *m, uint8_t *end_states) {
    const size_t k = m->ld * (m->lq + 1) + m->lq;
    const int32_t h = max2(max2(m->I[k], m->D[k]), m->M[k]); /* :247-250 */
    if (end_states) {
        uint8_t e = 0;
        if (m->M[k] == h) e |= 1;
        if (m->I[k] == h) e |= 2;
        if (m->D[k] == h) e |= 4;
        *end_states = e;
    }
    return h;
}

/* ---- literal DFS (TraceBackInfo stack), :246-329 ---- */
typedef struct {
    int state;
    size_t x, y;
    size_t len;   /* columns so far */
    char *s1, *s2; /* owned, len bytes each */
} frame;

typedef struct {
    char *out;
    size_t cap, len;
} sink;

static void sink_put(sink *s, const char *p, size_t n) {
    if (s->out && s->len < s->cap) {
        size_t k = s->cap - s->len < n ? s->cap - s->len : n;
        memcpy(s->out + s->len, p, k);
    }
    s->len += n;
}

/* TraceBackInfo Display, :390-411, printed via println! at :284-285 */
static void print_block(sink *s, const frame *f) {
    static const char hdr[] = "alignment found\n";
    sink_put(s, hdr, sizeof(hdr) - 1);
    sink_put(s, "\nseq1: ", 7);
    sink_put(s, f->s1, f->len);
    sink_put(s, "\n      ", 7);
    for (size_t k = 0; k < f->len; ++k) sink_put(s, f->s1[k] == f->s2[k] ? "|" : " ", 1);
    sink_put(s, "\nseq2: ", 7);
    sink_put(s, f->s2, f->len);
    sink_put(s, "\n", 1);
}

/* parent list of a cell in push order: returns count, fills st/x/y */
static int parents_of(const ref_nw_mats *m, int state, size_t x, size_t y, int *ps, size_t *px,
                      size_t *py) {
    const size_t W = m->lq + 1;
    const size_t k = x * W + y;
    int n = 0;
    if (state == ST_M) {
        const uint8_t b = m->pM[k];
        if (b & 1) { ps[n] = ST_M; px[n] = x - 1; py[n] = y - 1; ++n; }
        if (b & 2) { ps[n] = ST_I; px[n] = x - 1; py[n] = y - 1; ++n; }
        if (b & 4) { ps[n] = ST_D; px[n] = x - 1; py[n] = y - 1; ++n; }
    } else if (state == ST_I) {
        const uint8_t b = m->pI[k];
        if (b & 1) { ps[n] = ST_I; px[n] = x; py[n] = y - 1; ++n; }
        if (b & 2) { ps[n] = ST_M; px[n] = x; py[n] = y - 1; ++n; }
    } else {
        const uint8_t b = m->pD[k];
        if (b & 1) { ps[n] = ST_D; px[n] = x - 1; py[n] = y; ++n; }
        if (b & 2) { ps[n] = ST_M; px[n] = x - 1; py[n] = y; ++n; }
    }
    return n;
}

int ref_nw_traceback_dfs(const uint8_t *q, const uint8_t *d, const ref_nw_mats *m, char *out,
                         size_t out_cap, size_t *out_len, uint64_t max_pops, uint64_t *n_blocks) {
    return ref_nw_traceback_dfs_blocks(q, d, m, out, out_cap, out_len, max_pops, 0, n_blocks);
}

int ref_nw_traceback_dfs_blocks(const uint8_t *q, const uint8_t *d, const ref_nw_mats *m,
                                char *out, size_t out_cap, size_t *out_len, uint64_t max_pops,
                                uint64_t max_blocks, uint64_t *n_blocks) {
    const size_t W = m->lq + 1;
    const size_t ex = m->ld, ey = m->lq, ek = ex * W + ey;
    sink s = {out, out_cap, 0};
    uint64_t blocks = 0, pops = 0;
    size_t cap = 64, top = 0;
    frame *stk = (frame *)malloc(cap * sizeof(frame));
    int rc = 0;
    const int32_t mx = max2(max2(m->I[ek], m->D[ek]), m->M[ek]);
    /* push order I, M, D (:251-280) */
    const int order[3] = {ST_I, ST_M, ST_D};
    const int32_t *vals[3] = {m->I, m->M, m->D};
    for (int k = 0; k < 3; ++k) {
        if (mx == vals[k][ek]) {
            frame f = {order[k], ex, ey, 0, NULL, NULL};
            stk[top++] = f;
        }
    }
    while (top > 0) {
        frame e = stk[--top];
        ++pops;
        if (max_pops && pops > max_pops) {
            free(e.s1);
            free(e.s2);
            rc = 2;
            break;
        }
        if (e.x == 0 && e.y == 0) { /* :283-286 */
            if (max_blocks && blocks >= max_blocks) { /* caller's block cap (not the reference's) */
                free(e.s1);
                free(e.s2);
                rc = 3;
                break;
            }
            print_block(&s, &e);
            ++blocks;
        }
        int ps[3];
        size_t px[3], py[3];
        const int np = parents_of(m, e.state, e.x, e.y, ps, px, py);
        for (int p = 0; p < np; ++p) { /* :287-328 */
            char c1, c2;
            if (e.state == ST_M) {
                if (e.y == 0 || e.x == 0) { rc = 1; break; } /* index panic */
                c1 = (char)q[e.y - 1];
                c2 = (char)d[e.x - 1];
            } else if (e.state == ST_D) {
                if (e.x == 0) { rc = 1; break; } /* :299 seq2[x-1] */
                c1 = '-';
                c2 = (char)d[e.x - 1];
            } else {
                if (e.y == 0) { rc = 1; break; } /* :303 seq1[y-1] */
                c1 = (char)q[e.y - 1];
                c2 = '-';
            }
            frame f;
            f.state = ps[p];
            f.x = px[p];
            f.y = py[p];
            f.len = e.len + 1;
            f.s1 = (char *)malloc(f.len);
            f.s2 = (char *)malloc(f.len);
            f.s1[0] = c1;
            f.s2[0] = c2;
            if (e.len) {
                memcpy(f.s1 + 1, e.s1, e.len);
                memcpy(f.s2 + 1, e.s2, e.len);
            }
            if (top == cap) {
                cap *= 2;
                stk = (frame *)realloc(stk, cap * sizeof(frame));
            }
            stk[top++] = f;
        }
        free(e.s1);
        free(e.s2);
        if (rc == 1) break;
    }
    while (top > 0) {
        --top;
        free(stk[top].s1);
        free(stk[top].s2);
    }
    free(stk);
    if (out_len) *out_len = s.len;
    if (n_blocks) *n_blocks = blocks;
    return rc;
}

/* ---- memoised restatement of the same DFS ---- */
enum { FE_NONE = 0, FE_ORIGIN = 1, FE_PANIC = 2 };

typedef struct {
    const ref_nw_mats *m;
    uint64_t *cnt;
    uint8_t *pan, *fe, *done;
} dag;

static inline uint64_t sat_add(uint64_t a, uint64_t b) { return a + b < a ? UINT64_MAX : a + b; }

static int is_panic_node(int state, size_t x, size_t y, int np) {
    if (np == 0) return 0;
    if (state == ST_M) return x == 0 || y == 0;
    if (state == ST_D) return x == 0;
    return y == 0;
}

static void dag_eval(dag *g, int state, size_t x, size_t y) {
    const size_t W = g->m->lq + 1;
    const size_t id = (x * W + y) * 3 + (size_t)state;
    if (g->done[id]) return;
    int ps[3];
    size_t px[3], py[3];
    const int np = parents_of(g->m, state, x, y, ps, px, py);
    uint64_t c = 0;
    uint8_t pan = 0, fe = FE_NONE;
    if (x == 0 && y == 0) {
        c = 1;
        fe = FE_ORIGIN;
    }
    if (is_panic_node(state, x, y, np)) {
        pan = 1;
        if (fe == FE_NONE) fe = FE_PANIC;
    } else {
        for (int p = np - 1; p >= 0; --p) { /* DFS pops the last pushed first */
            dag_eval(g, ps[p], px[p], py[p]);
            const size_t cid = (px[p] * W + py[p]) * 3 + (size_t)ps[p];
            c = sat_add(c, g->cnt[cid]);
            if (fe == FE_NONE) fe = g->fe[cid];
            if (g->pan[cid]) {
                pan = 1;
                break;
            }
        }
    }
    g->cnt[id] = c;
    g->pan[id] = pan;
    g->fe[id] = fe;
    g->done[id] = 1;
}

int ref_nw_dag_summary(const uint8_t *q, const uint8_t *d, const ref_nw_mats *m, uint64_t *n_blocks,
                       int *panics, char *ops, size_t ops_cap, int64_t *ops_len) {
    const size_t W = m->lq + 1, H = m->ld + 1, n = W * H * 3;
    dag g = {m, (uint64_t *)calloc(n, 8), (uint8_t *)calloc(n, 1), (uint8_t *)calloc(n, 1),
             (uint8_t *)calloc(n, 1)};
    const size_t ex = m->ld, ey = m->lq, ek = ex * W + ey;
    const int32_t mx = max2(max2(m->I[ek], m->D[ek]), m->M[ek]);
    /* pop order of the end states: D, M, I */
    const int order[3] = {ST_D, ST_M, ST_I};
    const int32_t *vals[3] = {m->D, m->M, m->I};
    uint64_t c = 0;
    int pan = 0, root_fe = FE_NONE, first_state = -1;
    for (int k = 0; k < 3; ++k) {
        if (mx != vals[k][ek]) continue;
        dag_eval(&g, order[k], ex, ey);
        const size_t id = ek * 3 + (size_t)order[k];
        c = sat_add(c, g.cnt[id]);
        if (root_fe == FE_NONE && g.fe[id] != FE_NONE) {
            root_fe = g.fe[id];
            first_state = order[k];
        }
        if (g.pan[id]) {
            pan = 1;
            break;
        }
    }
    *n_blocks = c;
    *panics = pan;
    *ops_len = -1;
    if (root_fe == FE_ORIGIN) {
        /* walk the first-event path, collecting columns back to front */
        size_t len = 0, x = ex, y = ey;
        int st = first_state;
        char *rev = (char *)malloc(m->lq + m->ld + 1);
        while (!(x == 0 && y == 0)) {
            int ps[3];
            size_t px[3], py[3];
            const int np = parents_of(m, st, x, y, ps, px, py);
            char op = st == ST_M ? (q[y - 1] == d[x - 1] ? '=' : 'X') : (st == ST_I ? 'I' : 'D');
            rev[len++] = op;
            int moved = 0;
            for (int p = np - 1; p >= 0; --p) {
                const size_t cid = (px[p] * W + py[p]) * 3 + (size_t)ps[p];
                if (g.fe[cid] != FE_NONE) {
                    st = ps[p];
                    x = px[p];
                    y = py[p];
                    moved = 1;
                    break;
                }
            }
            if (!moved) break; /* cannot happen when root_fe == ORIGIN */
        }
        for (size_t k = 0; k < len && k < ops_cap; ++k) ops[k] = rev[len - 1 - k];
        *ops_len = (int64_t)len;
        free(rev);
    }
    free(g.cnt);
    free(g.pan);
    free(g.fe);
    free(g.done);
    return 0;
}

uint64_t ref_nw_run_pairs_capped(const uint8_t *qs, const uint64_t *q_off, const uint8_t *ds,
                                 const uint64_t *d_off, uint64_t n_pairs, uint64_t max_pops,
                                 uint64_t max_blocks, uint64_t *capped) {
    uint64_t cells = 0, nc = 0;
    for (uint64_t p = 0; p < n_pairs; ++p) {
        const uint8_t *q = qs + q_off[p], *d = ds + d_off[p];
        const size_t lq = q_off[p + 1] - q_off[p], ld = d_off[p + 1] - d_off[p];
        ref_nw_mats m;
        if (ref_nw_fill(q, lq, d, ld, &m) != 0) break;
        size_t olen = 0;
        uint64_t nb = 0;
        /* rc 2: the DFS stopped at max_pops (the reference enumerates on) */
        if (ref_nw_traceback_dfs_blocks(q, d, &m, NULL, 0, &olen, max_pops, max_blocks, &nb) == 2)
            ++nc;
        ref_nw_free(&m);
        cells += (uint64_t)lq * ld;
    }
    if (capped) *capped = nc;
    return cells;
}

uint64_t ref_nw_run_pairs(const uint8_t *qs, const uint64_t *q_off, const uint8_t *ds,
                          const uint64_t *d_off, uint64_t n_pairs, uint64_t max_pops) {
    return ref_nw_run_pairs_capped(qs, q_off, ds, d_off, n_pairs, max_pops, 0, NULL);
}

/* ---- FASTA parser, parse.rs:52-99 ---- */
static int allowed(uint8_t c) { return c == 'A' || c == 'G' || c == 'C' || c == 'T' || c == 'N'; }

typedef struct {
    uint8_t *name, *seq;
    size_t nl, sl, ncap, scap;
} rec_t;

static void push_byte(uint8_t **p, size_t *n, size_t *cap, uint8_t c) {
    if (*n == *cap) {
        *cap = *cap ? *cap * 2 : 64;
        *p = (uint8_t *)realloc(*p, *cap);
    }
    (*p)[(*n)++] = c;
}

int64_t ref_parse_fasta(const uint8_t *buf, size_t len, int has_valid_ext, uint8_t *rec_out,
                        size_t rec_cap, size_t *rec_len, uint8_t *bad_chars, size_t bad_cap,
                        size_t *n_bad_chars) {
    if (!has_valid_ext) return -1; /* :55-60 FastaError(InvalidInput) */
    size_t nrec = 0, rcap = 16, nbad = 0;
    rec_t *recs = (rec_t *)calloc(rcap, sizeof(rec_t));
    rec_t cur;
    memset(&cur, 0, sizeof(cur));
    int in_name = 0;
    for (size_t k = 0; k < len; ++k) {
        const uint8_t c = buf[k];
        if (c == '>') { /* :67-74 */
            if (nrec == rcap) {
                rcap *= 2;
                recs = (rec_t *)realloc(recs, rcap * sizeof(rec_t));
            }
            recs[nrec++] = cur;
            memset(&cur, 0, sizeof(cur));
            push_byte(&cur.name, &cur.nl, &cur.ncap, c);
            in_name = 1;
            continue;
        }
        if (in_name) { /* :76-81 */
            if (c == '\n') {
                in_name = 0;
                continue;
            }
            push_byte(&cur.name, &cur.nl, &cur.ncap, c);
        } else if (c == '\n') {
            continue;
        } else if (!allowed(c)) { /* :84-85 */
            if (nbad < bad_cap) bad_chars[nbad] = c;
            ++nbad;
        } else {
            push_byte(&cur.seq, &cur.sl, &cur.scap, c);
        }
    }
    if (nrec == rcap) {
        rcap *= 2;
        recs = (rec_t *)realloc(recs, rcap * sizeof(rec_t));
    }
    recs[nrec++] = cur; /* :90 */
    /* :91 remove(0): drop the implicit first record */
    size_t w = 0;
    for (size_t r = 1; r < nrec; ++r) {
        const uint32_t nl = (uint32_t)recs[r].nl, sl = (uint32_t)recs[r].sl;
        if (rec_out && w + 8 + nl + sl <= rec_cap) {
            memcpy(rec_out + w, &nl, 4);
            memcpy(rec_out + w + 4, recs[r].name, nl);
            memcpy(rec_out + w + 4 + nl, &sl, 4);
            memcpy(rec_out + w + 8 + nl, recs[r].seq, sl);
        }
        w += 8 + nl + sl;
    }
    for (size_t r = 0; r < nrec; ++r) {
        free(recs[r].name);
        free(recs[r].seq);
    }
    free(recs);
    if (rec_len) *rec_len = w;
    if (n_bad_chars) *n_bad_chars = nbad;
    return (int64_t)(nrec - 1);
}

uint64_t ref_splitmix64(uint64_t *state) {
    uint64_t z = (*state += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/*
 * ORACLE — test infrastructure only (see refcpu.h).
 *
 * Plain-C restatement of the reference WFA, src/wfa.rs (snapshot 2025-02-13),
 * with release-build semantics (wrapping usize subtraction; panics of
 * rotate_left / slice indexing / unwrap still fire and end the pair):
 *   constants            :14-21
 *   wfa_align            :23-42
 *   WaveFrontElement x/y :85-90, get_distance :96-101
 *   WaveFront::expand    :127-139, get_element/get_offset :154-175,
 *                        is_converged :180-191
 *   get_parents          :201-209
 *   WaveFrontTensor::new :225-420, is_converged :422-439
 *   Ocean::global        :450-465, expand :467-488, trim :490-623,
 *                        is_converged :625-632, traceback :634-652,
 *                        rec_tr :654-853
 *   Alignment Display    :950-980 (+ the derived Debug of Alignment)
 * Pinned by the reference's own tests: test_wavefront_tensor_new_all_none
 * (:994-1000), recurrance_eq (:1003-1102), test_initial (:1105-1186),
 * test_converge (:1289-1294) — tests/test_wfa_oracle.py.
 */
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "refcpu.h"

enum { ST_M = 0, ST_D = 1, ST_I = 2 }; /* enum State { M, D, I } :44-50 */

typedef struct {
    int some;          /* Option<WaveFrontElement> */
    int32_t offset;
    uint8_t state;
    uint8_t np;        /* parents: Vec<State>, at most 3 */
    uint8_t parents[3];
} welem;

typedef struct {
    int some;          /* Option<WaveFront> */
    int32_t lo, hi;
    size_t len, cap;
    welem *el;
} wfront;

typedef struct {
    int some;          /* Option<WaveFrontTensor> */
    wfront i, d, m;
} wtensor;

typedef struct {
    char *p;
    size_t n, cap;
} tsink;

static void tput(tsink *s, const char *fmt, ...) {
    char tmp[512];
    va_list ap;
    va_start(ap, fmt);
    int k = vsnprintf(tmp, sizeof tmp, fmt, ap);
    va_end(ap);
    if (k < 0) return;
    if (s->n + (size_t)k + 1 > s->cap) {
        size_t nc = s->cap ? s->cap * 2 : 4096;
        while (nc < s->n + (size_t)k + 1) nc *= 2;
        s->p = (char *)realloc(s->p, nc);
        s->cap = nc;
    }
    memcpy(s->p + s->n, tmp, (size_t)k);
    s->n += (size_t)k;
    s->p[s->n] = 0;
}

/* ------------------------------------------------------------- WaveFront */
static void wf_push(wfront *f, const welem *e) {
    if (f->len == f->cap) {
        f->cap = f->cap ? 2 * f->cap : 8;
        f->el = (welem *)realloc(f->el, f->cap * sizeof(welem));
    }
    f->el[f->len++] = *e;
}
static void wf_free(wfront *f) {
    free(f->el);
    memset(f, 0, sizeof *f);
}
/* get_element :154-158: elements.get((idx - lo) as usize) */
static const welem *wf_get(const wfront *f, int32_t idx) {
    if (!f || !f->some) return NULL;
    const int64_t k = (int64_t)idx - f->lo;
    if (k < 0 || (uint64_t)k >= f->len) return NULL;
    return f->el[k].some ? &f->el[k] : NULL;
}
/* x(diag) / y(diag) :85-90 as usize (sign-extended i32) */
static uint64_t ex(const welem *e, int32_t diag) {
    return (uint64_t)(int64_t)(int32_t)(e->offset - (diag < 0 ? diag : 0));
}
static uint64_t ey(const welem *e, int32_t diag) {
    return (uint64_t)(int64_t)(int32_t)(e->offset + (diag > 0 ? diag : 0));
}
/* get_distance :96-101 */
static int32_t dist(const welem *e, size_t l1, size_t l2, int32_t diag) {
    const int32_t lv = (int32_t)l1 - e->offset - diag;
    const int32_t lh = (int32_t)l2 - e->offset;
    return lv > lh ? lv : lh;
}
/* WaveFront::expand :127-139 (seq1 = query indexed by y, seq2 = db by x) */
static void wf_extend(wfront *f, const uint8_t *s1, size_t l1, const uint8_t *s2, size_t l2) {
    for (size_t i = 0; i < f->len; ++i) {
        welem *e = &f->el[i];
        if (!e->some) continue;
        const int32_t diag = f->lo + (int32_t)i;
        while (ey(e, diag) < l1 && ex(e, diag) < l2 && s1[ey(e, diag)] == s2[ex(e, diag)])
            e->offset += 1;
    }
}
/* WaveFront::is_converged :180-191 */
static const welem *wf_converged(const wfront *f, size_t l1, size_t l2) {
    if (!f->some) return NULL;
    for (size_t i = 0; i < f->len; ++i) {
        const welem *e = &f->el[i];
        if (!e->some) continue;
        const int32_t diag = f->lo + (int32_t)i;
        if (ex(e, diag) == (uint64_t)l2 - 1 && ey(e, diag) == (uint64_t)l1 - 1) return e;
    }
    return NULL;
}
static void rotate_left(welem *a, size_t n, size_t mid) {
    if (!n || !mid) return;
    welem *tmp = (welem *)malloc(mid * sizeof(welem));
    memcpy(tmp, a, mid * sizeof(welem));
    memmove(a, a + mid, (n - mid) * sizeof(welem));
    memcpy(a + n - mid, tmp, mid * sizeof(welem));
    free(tmp);
}
static void truncate_to(wfront *f, size_t n) {
    if (n < f->len) f->len = n;
}
static uint32_t absdiff(int32_t a, int32_t b) {
    return a > b ? (uint32_t)((int64_t)a - b) : (uint32_t)((int64_t)b - a);
}

/* get_parents :201-209 */
static void parents_of(welem *out, int32_t offset, const welem **c, int nc) {
    out->np = 0;
    for (int k = 0; k < nc; ++k)
        if (c[k] && c[k]->offset == offset) out->parents[out->np++] = c[k]->state;
}

static int opt_max(int *have, int32_t *v, int hv, int32_t x) {
    /* Option max: None < Some */
    if (!hv) return 0;
    if (!*have || x > *v) {
        *v = x;
        *have = 1;
    }
    return 1;
}

/* WaveFrontTensor::new :225-420.  o = s-o-e, e = s-e, x = s-x sources.
 * Returns 0 (None) when no source front exists. */
static int tensor_new(const wtensor *o, const wtensor *e, const wtensor *x, wtensor *out,
                      tsink *txt) {
    memset(out, 0, sizeof *out);
    const wfront *om = o && o->some && o->m.some ? &o->m : NULL;
    const wfront *xm = x && x->some && x->m.some ? &x->m : NULL;
    const wfront *ei = e && e->some && e->i.some ? &e->i : NULL;
    const wfront *ed = e && e->some && e->d.some ? &e->d : NULL;
    const wfront *src[4] = {om, xm, ei, ed};
    int have = 0;
    int32_t hi = 0, lo = 0;
    for (int k = 0; k < 4; ++k)
        if (src[k]) {
            if (!have || src[k]->hi > hi) hi = src[k]->hi;
            if (!have || src[k]->lo < lo) lo = src[k]->lo;
            have = 1;
        }
    if (!have) return 0;
    hi += 1;
    lo -= 1;
    if (txt) tput(txt, "lo: %d, hi: %d\n", lo, hi);
    wfront I = {1, lo, hi, 0, 0, NULL}, D = {1, lo, hi, 0, 0, NULL}, M = {1, lo, hi, 0, 0, NULL};
    int32_t il = lo, ih = hi, dl = lo, dh = hi, ml = lo, mh = hi;
    int iset = 0, dset = 0, mset = 0;
    for (int32_t idx = lo; lo <= hi; ++idx) { /* `for idx in lo..=hi` */
        /* D: max(O.m[idx+1], E.d[idx+1]) :268-306 */
        {
            const welem *a = wf_get(om, idx + 1), *b = wf_get(ed, idx + 1);
            int h = 0;
            int32_t v = 0;
            opt_max(&h, &v, a != NULL, a ? a->offset : 0);
            opt_max(&h, &v, b != NULL, b ? b->offset : 0);
            welem w = {0, 0, 0, 0, {0, 0, 0}};
            if (h) {
                const welem *c[2] = {a, b};
                w.some = 1;
                w.offset = v;
                w.state = ST_D;
                parents_of(&w, v, c, 2);
                dh = idx;
                if (!dset) dl = idx, dset = 1;
            }
            wf_push(&D, &w);
        }
        /* I: max(O.m[idx-1], E.i[idx-1]) + 1 :308-347 */
        {
            const welem *a = wf_get(om, idx - 1), *b = wf_get(ei, idx - 1);
            int h = 0;
            int32_t v = 0;
            opt_max(&h, &v, a != NULL, a ? a->offset : 0);
            opt_max(&h, &v, b != NULL, b ? b->offset : 0);
            welem w = {0, 0, 0, 0, {0, 0, 0}};
            if (h) {
                const welem *c[2] = {a, b};
                w.some = 1;
                w.offset = v + 1;
                w.state = ST_I;
                parents_of(&w, v, c, 2);
                ih = idx;
                if (!iset) il = idx, iset = 1;
            }
            wf_push(&I, &w);
        }
        /* M: max(X.m[idx]+1, I[idx], D[idx]) :348-395.  I/D are the fronts
         * being built, still with lo = the constructor's lo. */
        {
            const welem *xa = wf_get(xm, idx);
            welem xc;
            if (xa) {
                xc = *xa;
                xc.offset += 1;
                xc.state = ST_M;
                xc.np = 0;
            }
            const welem *ib = wf_get(&I, idx), *db = wf_get(&D, idx);
            int h = 0;
            int32_t v = 0;
            opt_max(&h, &v, xa != NULL, xa ? xa->offset + 1 : 0);
            opt_max(&h, &v, ib != NULL, ib ? ib->offset : 0);
            opt_max(&h, &v, db != NULL, db ? db->offset : 0);
            if (h) {
                const welem *c[3] = {xa ? &xc : NULL, ib, db};
                welem w = {1, v, ST_M, 0, {0, 0, 0}};
                parents_of(&w, v, c, 3);
                wf_push(&M, &w);
                mh = idx;
                if (!mset) ml = idx, mset = 1;
            } else if (mset) {
                welem w = {0, 0, 0, 0, {0, 0, 0}};
                wf_push(&M, &w);
            }
        }
        if (idx == hi) break;
    }
    I.lo = il, I.hi = ih, D.lo = dl, D.hi = dh, M.lo = ml, M.hi = mh;
    rotate_left(I.el, I.len, absdiff(lo, I.lo));
    truncate_to(&I, absdiff(I.hi, I.lo) + 1);
    rotate_left(D.el, D.len, absdiff(lo, D.lo));
    truncate_to(&D, absdiff(D.hi, D.lo) + 1);
    truncate_to(&M, absdiff(M.hi, M.lo) + 1);
    out->some = 1;
    if (iset) out->i = I; else wf_free(&I);
    if (dset) out->d = D; else wf_free(&D);
    if (mset) out->m = M; else wf_free(&M);
    return 1;
}

static void tensor_free(wtensor *t) {
    wf_free(&t->i);
    wf_free(&t->d);
    wf_free(&t->m);
    t->some = 0;
}

/* ------------------------------------------------------------------ Ocean */
typedef struct {
    size_t n, cap;
    wtensor *t;
} wocean;

static void ocean_push(wocean *oc, const wtensor *t) {
    if (oc->n == oc->cap) {
        oc->cap = oc->cap ? 2 * oc->cap : 32;
        oc->t = (wtensor *)realloc(oc->t, oc->cap * sizeof(wtensor));
    }
    oc->t[oc->n++] = *t;
}
static const wtensor *ocean_get(const wocean *oc, int64_t s) {
    if (s < 0 || (uint64_t)s >= oc->n) return NULL;
    return oc->t[s].some ? &oc->t[s] : NULL;
}

/* trim :490-623.  Returns 0, or REF_WFA_PANIC_TRIM. */
static int ocean_trim(wocean *oc, const uint8_t *s1, size_t l1, const uint8_t *s2, size_t l2) {
    (void)s1;
    (void)s2;
    if (!oc->n || !oc->t[oc->n - 1].some) return 0;
    wtensor *cur = &oc->t[oc->n - 1];
    if (!cur->m.some) return 0;
    wfront *m = &cur->m;
    if (absdiff(m->lo, m->hi) <= 5) return 0; /* MINLENGTH */
    int32_t min_d = 0;
    for (int32_t dg = m->lo; m->lo <= m->hi; ++dg) {
        const welem *e = wf_get(m, dg);
        if (e) {
            const int32_t dd = dist(e, l1, l2, dg);
            if (dd < min_d) min_d = dd;
        }
        if (dg == m->hi) break;
    }
#define FIRST_OR_PANIC(E)                                                   \
    do {                                                                    \
        if (!m->len || !m->el[0].some) return REF_WFA_PANIC_TRIM;           \
        (E) = &m->el[0];                                                    \
    } while (0)
#define LAST_OR_PANIC(E)                                                    \
    do {                                                                    \
        if (!m->len || !m->el[m->len - 1].some) return REF_WFA_PANIC_TRIM;  \
        (E) = &m->el[m->len - 1];                                           \
    } while (0)
#define REMOVE_FRONT()                                                      \
    do {                                                                    \
        if (!m->len) return REF_WFA_PANIC_TRIM;                             \
        memmove(m->el, m->el + 1, (m->len - 1) * sizeof(welem));            \
        m->len--;                                                           \
    } while (0)
    const welem *fe;
    FIRST_OR_PANIC(fe);
    int32_t next_d = dist(fe, l1, l2, m->lo);
    while (m->lo < m->hi && absdiff(next_d, min_d) > 20) { /* MAXDIFF */
        m->lo += 1;
        REMOVE_FRONT();
        while (!wf_get(m, m->lo)) {
            if (m->lo == m->hi) break;
            m->lo += 1;
            REMOVE_FRONT();
        }
        FIRST_OR_PANIC(fe);
        next_d = dist(fe, l1, l2, m->lo);
    }
    LAST_OR_PANIC(fe);
    next_d = dist(fe, l1, l2, m->hi);
    while (m->hi > m->lo && absdiff(next_d, min_d) > 20) {
        m->hi -= 1;
        if (m->len) m->len--; /* pop */
        while (!wf_get(m, m->hi)) {
            if (m->lo == m->hi) break;
            m->hi -= 1;
            if (m->len) m->len--;
        }
        LAST_OR_PANIC(fe);
        next_d = dist(fe, l1, l2, m->hi);
    }
#undef FIRST_OR_PANIC
#undef LAST_OR_PANIC
#undef REMOVE_FRONT
    /* clamp I then D to M :574-622 (release: len - t wraps; truncate no-op) */
    wfront *g[2] = {cur->i.some ? &cur->i : NULL, cur->d.some ? &cur->d : NULL};
    for (int k = 0; k < 2; ++k) {
        wfront *f = g[k];
        if (!f) continue;
        size_t t;
        if (f->lo < m->lo) {
            const size_t mid = absdiff(f->lo, m->lo);
            if (mid > f->len) return REF_WFA_PANIC_TRIM; /* rotate_left assert */
            rotate_left(f->el, f->len, mid);
            t = mid + (f->hi > m->hi ? absdiff(f->hi, m->hi) : 0);
        } else if (f->hi > m->hi) {
            t = absdiff(f->hi, m->hi);
        } else {
            t = 0;
        }
        truncate_to(f, f->len - t); /* wrapping usize subtraction */
        if (m->hi < f->hi) f->hi = m->hi;
        if (m->lo > f->lo) f->lo = m->lo;
    }
    return 0;
}

/* Ocean::expand :467-488 */
static int ocean_expand(wocean *oc, const uint8_t *s1, size_t l1, const uint8_t *s2, size_t l2,
                        tsink *txt) {
    const int64_t s = (int64_t)oc->n;
    wtensor t;
    const int some = tensor_new(ocean_get(oc, s - 8), ocean_get(oc, s - 6), ocean_get(oc, s - 4),
                                &t, txt);
    if (!some) memset(&t, 0, sizeof t);
    ocean_push(oc, &t);
    wtensor *nt = &oc->t[oc->n - 1];
    if (nt->some && nt->m.some) wf_extend(&nt->m, s1, l1, s2, l2);
    return ocean_trim(oc, s1, l1, s2, l2);
}

/* WaveFrontTensor::is_converged :422-439 on the newest tensor */
static const welem *ocean_converged(const wocean *oc, size_t l1, size_t l2) {
    if (!oc->n || !oc->t[oc->n - 1].some) return NULL;
    const wtensor *t = &oc->t[oc->n - 1];
    const welem *e;
    if ((e = wf_converged(&t->i, l1, l2))) return e;
    if ((e = wf_converged(&t->d, l1, l2))) return e;
    if ((e = wf_converged(&t->m, l1, l2))) return e;
    return NULL;
}

static const char *state_name(int s) { return s == ST_M ? "M" : s == ST_D ? "D" : "I"; }

/* Debug for WaveFrontElement :103-116 (custom; `{:#?}` inner fields) */
static void put_elem_debug(tsink *t, const welem *e) {
    tput(t, "Element {\n");
    tput(t, "\tstate: %s\n\toffset: %d\n", state_name(e->state), e->offset);
    if (!e->np) {
        tput(t, "\tparents: []\n");
    } else {
        tput(t, "\tparents: [\n");
        for (int k = 0; k < e->np; ++k) tput(t, "    %s,\n", state_name(e->parents[k]));
        tput(t, "]\n");
    }
    tput(t, "}\n");
}

typedef struct {
    uint8_t *p;
    size_t n, cap;
} bytes_t;
static void bpush(bytes_t *b, uint8_t c) {
    if (b->n == b->cap) {
        b->cap = b->cap ? 2 * b->cap : 64;
        b->p = (uint8_t *)realloc(b->p, b->cap);
    }
    b->p[b->n++] = c;
}
/* current[0].seqK.extend(seq[a..b].iter().rev()) with slice bounds checks */
static int extend_rev(bytes_t *dst, const uint8_t *s, size_t len, uint64_t a, uint64_t b) {
    if (a > b || b > len) return REF_WFA_PANIC_SLICE;
    for (uint64_t k = b; k > a; --k) bpush(dst, s[k - 1]);
    return 0;
}

static int has_parent(const welem *e, int st) {
    for (int k = 0; k < e->np; ++k)
        if (e->parents[k] == st) return 1;
    return 0;
}

/* rec_tr :654-853 (iterative: every branch ends in `return rec_tr(..)`) */
static int rec_tr(const wocean *oc, int32_t diag, const uint8_t *s1, size_t l1, const uint8_t *s2,
                  size_t l2, bytes_t *a1, bytes_t *a2, welem ne, uint64_t score, tsink *txt) {
    for (;;) {
        if (diag == 0 && ne.offset == 0) {
            tput(txt, "ret\n");
            return 0;
        }
        const uint64_t dds[3] = {4, 6, 8};
        int moved = 0;
        for (int k = 0; k < 3 && !moved; ++k) {
            const uint64_t nd = dds[k];
            if (nd > score) {
                tput(txt, "well shit\n");
                continue;
            }
            const uint64_t ns = score - nd;
            tput(txt, "yeah, score: %llu\n", (unsigned long long)ns);
            if (ns >= oc->n) continue; /* wf_tensors.get(next_score) */
            const wtensor *t = oc->t[ns].some ? &oc->t[ns] : NULL;
            const welem *w = NULL;
            int32_t ndiag = diag;
            int kind = 0; /* 1 = M step, 2 = D-side (diag-1), 3 = I-side (diag+1), 4 = M->D quirk */
            if (nd == 4) {
                if (ne.state != ST_M && has_parent(&ne, ST_M) &&
                    (w = wf_get(t && t->m.some ? &t->m : NULL, diag))) {
                    tput(txt, "mismatch\n");
                    kind = 1;
                }
            } else if (nd == 6) {
                if (has_parent(&ne, ST_D) && (w = wf_get(t && t->d.some ? &t->d : NULL, diag - 1))) {
                    tput(txt, "extend\n");
                    kind = 2;
                } else if ((w = wf_get(t && t->i.some ? &t->i : NULL, diag + 1))) {
                    tput(txt, "extend\n");
                    kind = 3;
                }
            } else if (has_parent(&ne, ST_M)) {
                tput(txt, "open\n");
                const wfront *td = t && t->d.some ? &t->d : NULL;
                const wfront *ti = t && t->i.some ? &t->i : NULL;
                if (ne.state == ST_D) {
                    if ((w = wf_get(td, diag - 1))) kind = 2;
                } else if (ne.state == ST_I) {
                    if ((w = wf_get(ti, diag + 1))) kind = 3;
                } else {
                    if ((w = wf_get(ti, diag + 1))) kind = 3;
                    else if ((w = wf_get(td, diag - 1))) kind = 4;
                }
            }
            if (!kind) continue;
            int rc;
            if (kind == 1) {
                if ((rc = extend_rev(a1, s1, l1, ey(w, diag), ey(&ne, diag)))) return rc;
                if ((rc = extend_rev(a2, s2, l2, ex(w, diag), ex(&ne, diag)))) return rc;
            } else if (kind == 2) {
                if ((rc = extend_rev(a1, s1, l1, ey(w, diag), ey(&ne, diag)))) return rc;
                bpush(a2, '-');
                if ((rc = extend_rev(a2, s2, l2, ex(w, diag), ex(&ne, diag)))) return rc;
                ndiag = diag - 1;
            } else if (kind == 3) {
                bpush(a1, '-');
                if ((rc = extend_rev(a1, s1, l1, ey(w, diag), ey(&ne, diag)))) return rc;
                if ((rc = extend_rev(a2, s2, l2, ex(w, diag), ex(&ne, diag)))) return rc;
                ndiag = diag + 1;
            } else {
                if ((rc = extend_rev(a1, s1, l1, ey(w, diag), ey(&ne, diag)))) return rc;
                bpush(a1, '-');
                if ((rc = extend_rev(a2, s2, l2, ex(w, diag), ex(&ne, diag)))) return rc;
                ndiag = diag - 1;
            }
            ne = *w;
            diag = ndiag;
            score = ns;
            moved = 1;
        }
        if (!moved) {
            tput(txt, "huh\n");
            return 0;
        }
    }
}

static void put_vec_debug(tsink *t, const char *name, const bytes_t *b) {
    if (!b->n) {
        tput(t, "    %s: [],\n", name);
        return;
    }
    tput(t, "    %s: [\n", name);
    for (size_t k = 0; k < b->n; ++k) tput(t, "        %u,\n", (unsigned)b->p[k]);
    tput(t, "    ],\n");
}

int ref_wfa_align(const uint8_t *q, size_t lq, const uint8_t *d, size_t ld, int mode,
                  uint64_t max_steps, ref_wfa_result *res, char *out, size_t out_cap,
                  size_t *out_len) {
    memset(res, 0, sizeof *res);
    tsink txt = {NULL, 0, 0};
    tput(&txt, "%s", "");
    if (mode != 0) {
        res->status = REF_WFA_NOT_IMPLEMENTED;
    } else {
        wocean oc = {0, 0, NULL};
        /* Ocean::global :450-465 */
        wtensor t0;
        memset(&t0, 0, sizeof t0);
        t0.some = 1;
        t0.m.some = 1;
        welem e0 = {1, 0, ST_M, 0, {0, 0, 0}};
        wf_push(&t0.m, &e0);
        ocean_push(&oc, &t0);
        const uint8_t *s1 = q, *s2 = d;
        const size_t l1 = lq, l2 = ld;
        int rc = 0;
        uint64_t steps = 0;
        while (!ocean_converged(&oc, l1, l2)) {
            if (max_steps && steps >= max_steps) {
                rc = REF_WFA_NONCONVERGED;
                break;
            }
            rc = ocean_expand(&oc, s1, l1, s2, l2, &txt);
            ++steps;
            if (rc) break;
        }
        res->steps = steps;
        res->score = (int64_t)oc.n;
        if (!rc) {
            tput(&txt, "converged with score %llu: \n", (unsigned long long)oc.n);
            /* traceback :634-652 */
            const welem *last = ocean_converged(&oc, l1, l2);
            const int32_t diag = (int32_t)l1 - (int32_t)l2;
            tput(&txt, "huhu, diag: %d\n", diag);
            put_elem_debug(&txt, last);
            tput(&txt, "\nscore: %llu\n", (unsigned long long)oc.n);
            bytes_t a1 = {NULL, 0, 0}, a2 = {NULL, 0, 0};
            rc = rec_tr(&oc, diag, s1, l1, s2, l2, &a1, &a2, *last, oc.n, &txt);
            if (!rc) {
                /* Display :950-980, then println's newline */
                for (size_t k = a1.n; k > 0; --k) tput(&txt, "%c", a1.p[k - 1]);
                tput(&txt, "\n");
                const size_t nz = a1.n < a2.n ? a1.n : a2.n;
                for (size_t k = nz; k > 0; --k) tput(&txt, "%s", a1.p[k - 1] != a2.p[k - 1] ? " " : "|");
                for (size_t k = a2.n; k > 0; --k) tput(&txt, "%c", a2.p[k - 1]);
                tput(&txt, "\n\n");
                /* println!("{:#?}", t[0]) */
                tput(&txt, "Alignment {\n");
                put_vec_debug(&txt, "seq1", &a1);
                put_vec_debug(&txt, "seq2", &a2);
                tput(&txt, "}\n");
                res->aln_len1 = a1.n;
                res->aln_len2 = a2.n;
            }
            free(a1.p);
            free(a2.p);
        }
        res->status = rc;
        for (size_t k = 0; k < oc.n; ++k) tensor_free(&oc.t[k]);
        free(oc.t);
    }
    if (out_len) *out_len = txt.n;
    if (out && out_cap) {
        const size_t n = txt.n < out_cap - 1 ? txt.n : out_cap - 1;
        memcpy(out, txt.p, n);
        out[n] = 0;
    }
    free(txt.p);
    return res->status;
}

/* ---------------------------------------------------- tensor test hooks
 * Flat int32 encoding of an Option<WaveFrontTensor> for the reference's
 * tensor-level tests: [some, (front i, d, m)...]; front = [some, lo, hi, n,
 * n x (some, offset, state, np, p0, p1, p2)]. */
static const int32_t *dec_front(const int32_t *p, wfront *f) {
    memset(f, 0, sizeof *f);
    f->some = *p++;
    f->lo = *p++;
    f->hi = *p++;
    const int32_t n = *p++;
    for (int32_t k = 0; k < n; ++k) {
        welem e;
        e.some = *p++;
        e.offset = *p++;
        e.state = (uint8_t)*p++;
        e.np = (uint8_t)*p++;
        for (int j = 0; j < 3; ++j) e.parents[j] = (uint8_t)*p++;
        wf_push(f, &e);
    }
    return p;
}
static int32_t *enc_front(int32_t *p, const wfront *f) {
    *p++ = f->some;
    *p++ = f->some ? f->lo : 0;
    *p++ = f->some ? f->hi : 0;
    *p++ = f->some ? (int32_t)f->len : 0;
    if (f->some)
        for (size_t k = 0; k < f->len; ++k) {
            const welem *e = &f->el[k];
            *p++ = e->some;
            *p++ = e->some ? e->offset : 0;
            *p++ = e->some ? e->state : 0;
            *p++ = e->some ? e->np : 0;
            for (int j = 0; j < 3; ++j) *p++ = e->some && j < e->np ? e->parents[j] : 0;
        }
    return p;
}
static int dec_tensor(const int32_t *p, wtensor *t) {
    memset(t, 0, sizeof *t);
    if (!p || !p[0]) return 0;
    t->some = 1;
    p = dec_front(p + 1, &t->i);
    p = dec_front(p, &t->d);
    dec_front(p, &t->m);
    return 1;
}

int64_t ref_wfa_tensor_new(const int32_t *o, const int32_t *e, const int32_t *x, int32_t *out,
                           char *txt_out, size_t txt_cap) {
    wtensor to, te, tx, r;
    const int ho = dec_tensor(o, &to), he = dec_tensor(e, &te), hx = dec_tensor(x, &tx);
    tsink txt = {NULL, 0, 0};
    const int some = tensor_new(ho ? &to : NULL, he ? &te : NULL, hx ? &tx : NULL, &r, &txt);
    int32_t *p = out;
    *p++ = some;
    if (some) {
        p = enc_front(p, &r.i);
        p = enc_front(p, &r.d);
        p = enc_front(p, &r.m);
        tensor_free(&r);
    }
    if (txt_out && txt_cap) {
        const size_t n = txt.n < txt_cap - 1 ? txt.n : txt_cap - 1;
        if (n) memcpy(txt_out, txt.p, n);
        txt_out[n] = 0;
    }
    free(txt.p);
    tensor_free(&to);
    tensor_free(&te);
    tensor_free(&tx);
    return p - out;
}

/* Ocean::global() then is_converged (test_converge :1289-1294) */
int ref_wfa_initial_converged(const uint8_t *q, size_t lq, const uint8_t *d, size_t ld) {
    wocean oc = {0, 0, NULL};
    wtensor t0;
    memset(&t0, 0, sizeof t0);
    t0.some = 1;
    t0.m.some = 1;
    welem e0 = {1, 0, ST_M, 0, {0, 0, 0}};
    wf_push(&t0.m, &e0);
    ocean_push(&oc, &t0);
    (void)q;
    (void)d;
    const int c = ocean_converged(&oc, lq, ld) != NULL;
    tensor_free(&oc.t[0]);
    free(oc.t);
    return c;
}

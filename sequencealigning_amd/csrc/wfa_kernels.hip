// WFA with the reference's semantics (src/wfa.rs) on gfx950: one pair per
// lane.  The reference keeps every wavefront tensor of the score loop (the
// traceback walks back through all of them), so each lane owns a slice of a
// device arena holding its tensor history.  The arena is structure-of-arrays
// with the lane index fastest: the lanes of a wave are in the same score
// step and touch the same (tensor, front, element) at the same time, so the
// accesses coalesce.  Only even score steps can hold a tensor (every source
// of an odd step is odd, and step 0 is even), so slot = s / 2.
//
// Layout per launch (nl lanes, S slots, W elements per front):
//   hdr [S][3 fronts][4 fields: some, lo, hi, len][nl]   int32
//   off [S][3][W][nl]                                    int32 element offsets
//   meta[S][3][W][nl]   bit0 some, bits1-2 state, bits3-4 #parents,
//                       bits5-10 parents (2 bits each, push order)
//   tsome[S][nl]                                         tensor present
// Fronts are ordered i, d, m (WaveFrontTensor :212-216); states M = 0,
// D = 1, I = 2 (enum State :44-50).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "nw_host.hpp"
#include "saln.h"
#include "wfa_host.hpp"

namespace saln {

namespace {

enum { FI = 0, FD = 1, FM = 2 };
enum { SM = 0, SD = 1, SI = 2 };

struct Elem {
    bool some;
    int32_t offset;
    uint32_t meta;  // full meta word (state / parents)
};

__device__ __forceinline__ uint32_t mk_meta(uint32_t state, uint32_t np, uint32_t par) {
    return 1u | (state << 1) | (np << 3) | (par << 5);
}
__device__ __forceinline__ uint32_t m_state(uint32_t m) { return (m >> 1) & 3u; }
__device__ __forceinline__ uint32_t m_np(uint32_t m) { return (m >> 3) & 3u; }
__device__ __forceinline__ uint32_t m_par(uint32_t m, uint32_t k) { return (m >> (5 + 2 * k)) & 3u; }

struct LaneArena {
    WfaArena A;
    uint32_t l;
    __device__ int32_t &H(uint32_t slot, int f, int field) const {
        return A.hdr[((size_t)(slot * 3 + f) * 4 + field) * A.nl + l];
    }
    __device__ int32_t &O(uint32_t slot, int f, uint32_t k) const {
        return A.off[((size_t)(slot * 3 + f) * A.W + k) * A.nl + l];
    }
    __device__ uint32_t &Mt(uint32_t slot, int f, uint32_t k) const {
        return A.meta[((size_t)(slot * 3 + f) * A.W + k) * A.nl + l];
    }
    __device__ uint8_t &T(uint32_t slot) const { return A.tsome[(size_t)slot * A.nl + l]; }
    // get_element (:154-158) of front f of the tensor at slot (valid = slot exists)
    __device__ Elem get(bool valid, uint32_t slot, int f, int32_t idx) const {
        Elem e{false, 0, 0};
        if (!valid || !T(slot) || !H(slot, f, 0)) return e;
        const int64_t k = (int64_t)idx - H(slot, f, 1);
        if (k < 0 || k >= H(slot, f, 3)) return e;
        const uint32_t m = Mt(slot, f, (uint32_t)k);
        if (!(m & 1u)) return e;
        e.some = true;
        e.offset = O(slot, f, (uint32_t)k);
        e.meta = m;
        return e;
    }
    __device__ void put(uint32_t slot, int f, uint32_t k, const Elem &e) const {
        O(slot, f, k) = e.offset;
        Mt(slot, f, k) = e.some ? e.meta : 0u;
    }
    __device__ Elem at(uint32_t slot, int f, uint32_t k) const {
        const uint32_t m = Mt(slot, f, k);
        return Elem{(m & 1u) != 0, O(slot, f, k), m};
    }
};

// A source front's header read once per tensor (the arena is written while a
// tensor is built, so the compiler cannot keep these in registers itself):
// get_element (:154-158) against it needs only the element's own words.
struct SrcFront {
    bool ok;        // the tensor exists and the front is Some
    int32_t lo, n;  // first diagonal, element count
    uint32_t slot;
    int f;
    __device__ Elem get(const LaneArena &L, int32_t idx) const {
        Elem e{false, 0, 0};
        const int64_t k = (int64_t)idx - lo;
        if (!ok || k < 0 || k >= n) return e;
        const uint32_t m = L.Mt(slot, f, (uint32_t)k);
        if (!(m & 1u)) return e;
        e.some = true;
        e.offset = L.O(slot, f, (uint32_t)k);
        e.meta = m;
        return e;
    }
};
__device__ __forceinline__ SrcFront src_front(const LaneArena &L, bool ok, uint32_t slot, int f) {
    SrcFront r{ok, 0, 0, slot, f};
    if (ok) {
        r.lo = L.H(slot, f, 1);
        r.n = L.H(slot, f, 3);
    }
    return r;
}

// x(diag), y(diag) (:85-90) as sign-extended 64-bit (Rust `as usize`)
__device__ __forceinline__ int64_t ex(int32_t off, int32_t diag) { return (int64_t)(off - min(diag, 0)); }
__device__ __forceinline__ int64_t ey(int32_t off, int32_t diag) { return (int64_t)(off + max(diag, 0)); }
__device__ __forceinline__ uint32_t adiff(int32_t a, int32_t b) {
    return a > b ? (uint32_t)((int64_t)a - b) : (uint32_t)((int64_t)b - a);
}

// Option max (None < Some) folding
__device__ __forceinline__ void omax(bool &h, int32_t &v, bool s, int32_t x) {
    if (s && (!h || x > v)) {
        v = x;
        h = true;
    }
}

// reverse elements [a, b) of front (slot, f)
__device__ void rev_range(const LaneArena &L, uint32_t slot, int f, uint32_t a, uint32_t b) {
    while (a + 1 < b) {
        --b;
        const Elem x = L.at(slot, f, a), y = L.at(slot, f, b);
        L.put(slot, f, a, y);
        L.put(slot, f, b, x);
        ++a;
    }
}
__device__ void rotate_left(const LaneArena &L, uint32_t slot, int f, uint32_t n, uint32_t mid) {
    if (!n || !mid || mid == n) return;
    rev_range(L, slot, f, 0, mid);
    rev_range(L, slot, f, mid, n);
    rev_range(L, slot, f, 0, n);
}

// get_distance (:96-101)
__device__ __forceinline__ int32_t dist(int32_t off, int32_t l1, int32_t l2, int32_t diag) {
    const int32_t lv = l1 - off - diag, lh = l2 - off;
    return max(lv, lh);
}

struct Logs {
    int32_t *lohi;   // 2 per step: lo, hi (INT32_MIN = nothing printed)
    uint8_t *ev;     // rec_tr events
    uint32_t ev_cap;
    uint32_t nev;
};

// WaveFrontTensor::new (:225-420) into slot `ns`.  Returns false on width
// overflow (caller cap).
__device__ bool tensor_new(const LaneArena &L, int64_t s, uint32_t ns, int32_t *lohi_out,
                           bool &some) {
    const int64_t so = s - 8, se = s - 6, sx = s - 4;  // gap_opening + gap_extension, e, x
    const bool vo = so >= 0 && !(so & 1), ve = se >= 0 && !(se & 1), vx = sx >= 0 && !(sx & 1);
    const uint32_t po = vo ? (uint32_t)(so / 2) : 0, pe = ve ? (uint32_t)(se / 2) : 0,
                   px = vx ? (uint32_t)(sx / 2) : 0;
    const bool om = vo && L.T(po) && L.H(po, FM, 0);
    const bool xm = vx && L.T(px) && L.H(px, FM, 0);
    const bool ei = ve && L.T(pe) && L.H(pe, FI, 0);
    const bool ed = ve && L.T(pe) && L.H(pe, FD, 0);
    bool have = false;
    int32_t hi = 0, lo = 0;
#define SRC(ok, slot, f)                                                   \
    if (ok) {                                                              \
        const int32_t h = L.H(slot, f, 2), l = L.H(slot, f, 1);            \
        if (!have || h > hi) hi = h;                                       \
        if (!have || l < lo) lo = l;                                       \
        have = true;                                                       \
    }
    SRC(om, po, FM) SRC(xm, px, FM) SRC(ei, pe, FI) SRC(ed, pe, FD)
#undef SRC
    L.T(ns) = 0;
    some = false;
    if (!have) return true;
    hi += 1;
    lo -= 1;
    lohi_out[0] = lo;
    lohi_out[1] = hi;
    if (lo <= hi && (int64_t)hi - lo + 1 > (int64_t)L.A.W) return false;
    int32_t il = lo, ih = hi, dl = lo, dh = hi, ml = lo, mh = hi;
    bool iset = false, dset = false, mset = false;
    // Each front is written from its first Some element on (I, D as the
    // reference leaves them after rotate_left(lo.abs_diff(x.lo)): positions
    // past the truncated length are never read), so no rotation is needed.
    uint32_t mpos = 0, ipos = 0, dpos = 0;
    const SrcFront sm_o = src_front(L, om, po, FM), sd_e = src_front(L, ed, pe, FD);
    const SrcFront si_e = src_front(L, ei, pe, FI), sm_x = src_front(L, xm, px, FM);
    for (int32_t idx = lo; lo <= hi; ++idx) {
        Elem wd{false, 0, 0}, wi{false, 0, 0};
        {  // D (:268-306)
            const Elem a = sm_o.get(L, idx + 1), b = sd_e.get(L, idx + 1);
            bool h = false;
            int32_t v = 0;
            omax(h, v, a.some, a.offset);
            omax(h, v, b.some, b.offset);
            if (h) {
                uint32_t np = 0, par = 0;
                if (a.some && a.offset == v) par |= m_state(a.meta) << (2 * np++);
                if (b.some && b.offset == v) par |= m_state(b.meta) << (2 * np++);
                wd = Elem{true, v, mk_meta(SD, np, par)};
                dh = idx;
                if (!dset) dl = idx, dset = true;
            }
            if (dset) L.put(ns, FD, dpos++, wd);
        }
        {  // I (:308-347)
            const Elem a = sm_o.get(L, idx - 1), b = si_e.get(L, idx - 1);
            bool h = false;
            int32_t v = 0;
            omax(h, v, a.some, a.offset);
            omax(h, v, b.some, b.offset);
            if (h) {
                uint32_t np = 0, par = 0;
                if (a.some && a.offset == v) par |= m_state(a.meta) << (2 * np++);
                if (b.some && b.offset == v) par |= m_state(b.meta) << (2 * np++);
                wi = Elem{true, v + 1, mk_meta(SI, np, par)};
                ih = idx;
                if (!iset) il = idx, iset = true;
            }
            if (iset) L.put(ns, FI, ipos++, wi);
        }
        {  // M (:348-395): X.m[idx]+1 (as state M), I[idx], D[idx] of this tensor
            const Elem xa = sm_x.get(L, idx);
            bool h = false;
            int32_t v = 0;
            omax(h, v, xa.some, xa.offset + 1);
            omax(h, v, wi.some, wi.offset);
            omax(h, v, wd.some, wd.offset);
            if (h) {
                uint32_t np = 0, par = 0;
                if (xa.some && xa.offset + 1 == v) par |= (uint32_t)SM << (2 * np++);
                if (wi.some && wi.offset == v) par |= m_state(wi.meta) << (2 * np++);
                if (wd.some && wd.offset == v) par |= m_state(wd.meta) << (2 * np++);
                L.put(ns, FM, mpos++, Elem{true, v, mk_meta(SM, np, par)});
                mh = idx;
                if (!mset) ml = idx, mset = true;
            } else if (mset) {
                L.put(ns, FM, mpos++, Elem{false, 0, 0});
            }
        }
        if (idx == hi) break;
    }
    const uint32_t len = lo <= hi ? (uint32_t)(hi - lo + 1) : 0u;
    L.H(ns, FI, 0) = iset;
    L.H(ns, FI, 1) = il;
    L.H(ns, FI, 2) = ih;
    L.H(ns, FI, 3) = (int32_t)min(len, adiff(ih, il) + 1);
    L.H(ns, FD, 0) = dset;
    L.H(ns, FD, 1) = dl;
    L.H(ns, FD, 2) = dh;
    L.H(ns, FD, 3) = (int32_t)min(len, adiff(dh, dl) + 1);
    L.H(ns, FM, 0) = mset;
    L.H(ns, FM, 1) = ml;
    L.H(ns, FM, 2) = mh;
    L.H(ns, FM, 3) = (int32_t)min(mpos, adiff(mh, ml) + 1);
    L.T(ns) = 1;
    some = true;
    return true;
}

// Four sequence bytes from s + pos (pos + 4 <= length) as one word, byte 0
// lowest: two aligned dword loads and a byte funnel shift.  Each dword holds a
// byte of the range, so no load leaves the sequence's own aligned words.
__device__ __forceinline__ uint32_t load4(const uint8_t *s, int64_t pos) {
    const uintptr_t a = (uintptr_t)(s + pos);
    const uint32_t *w = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3u);
    const uint32_t lo = w[0], hi = sh ? w[1] : 0u;
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// WaveFront::expand (:127-139) on the M front of slot ns: the offset advances
// while s1[y] == s2[x] inside both sequences.  Compared four bytes per round
// trip (the first differing byte ends the run, as the byte loop would).
__device__ void extend_m(const LaneArena &L, uint32_t ns, const uint8_t *s1, int32_t l1,
                         const uint8_t *s2, int32_t l2) {
    if (!L.H(ns, FM, 0)) return;
    const int32_t lo = L.H(ns, FM, 1), n = L.H(ns, FM, 3);
    for (int32_t k = 0; k < n; ++k) {
        const uint32_t m = L.Mt(ns, FM, (uint32_t)k);
        if (!(m & 1u)) continue;
        const int32_t diag = lo + k;
        int32_t off = L.O(ns, FM, (uint32_t)k);
        for (;;) {
            const int64_t y = ey(off, diag), x = ex(off, diag);
            if (y < 0 || x < 0 || y >= l1 || x >= l2) break;
            if (y + 4 <= l1 && x + 4 <= l2) {
                const uint32_t d = load4(s1, y) ^ load4(s2, x);
                if (d == 0) {
                    off += 4;
                    continue;
                }
                off += (int32_t)(__builtin_ctz(d) >> 3);
                break;
            }
            if (s1[y] != s2[x]) break;
            ++off;
        }
        L.O(ns, FM, (uint32_t)k) = off;
    }
}

// Ocean::trim (:490-623) on slot ns.  Returns SALN_OK or SALN_REF_PANIC_TRIM.
__device__ int trim(const LaneArena &L, uint32_t ns, int32_t l1, int32_t l2) {
    if (!L.H(ns, FM, 0)) return SALN_OK;
    int32_t mlo = L.H(ns, FM, 1), mhi = L.H(ns, FM, 2);
    uint32_t mlen = (uint32_t)L.H(ns, FM, 3);
    if (adiff(mlo, mhi) <= 5) return SALN_OK;  // MINLENGTH
    int32_t min_d = 0;
    for (int32_t dg = mlo; mlo <= mhi; ++dg) {
        const int64_t k = (int64_t)dg - mlo;
        if (k >= 0 && k < mlen) {
            const Elem e = L.at(ns, FM, (uint32_t)k);
            if (e.some) min_d = min(min_d, dist(e.offset, l1, l2, dg));
        }
        if (dg == mhi) break;
    }
    auto remove_front = [&]() {
        for (uint32_t k = 0; k + 1 < mlen; ++k) L.put(ns, FM, k, L.at(ns, FM, k + 1));
        --mlen;
    };
    auto get_m = [&](int32_t idx) {
        const int64_t k = (int64_t)idx - mlo;
        return k >= 0 && k < mlen && (L.Mt(ns, FM, (uint32_t)k) & 1u);
    };
    if (!mlen || !(L.Mt(ns, FM, 0) & 1u)) return SALN_REF_PANIC_TRIM;
    int32_t next_d = dist(L.O(ns, FM, 0), l1, l2, mlo);
    while (mlo < mhi && adiff(next_d, min_d) > 20) {  // MAXDIFF
        ++mlo;
        if (!mlen) return SALN_REF_PANIC_TRIM;
        remove_front();
        while (!get_m(mlo)) {
            if (mlo == mhi) break;
            ++mlo;
            if (!mlen) return SALN_REF_PANIC_TRIM;
            remove_front();
        }
        if (!mlen || !(L.Mt(ns, FM, 0) & 1u)) return SALN_REF_PANIC_TRIM;
        next_d = dist(L.O(ns, FM, 0), l1, l2, mlo);
    }
    if (!mlen || !(L.Mt(ns, FM, mlen - 1) & 1u)) return SALN_REF_PANIC_TRIM;
    next_d = dist(L.O(ns, FM, mlen - 1), l1, l2, mhi);
    while (mhi > mlo && adiff(next_d, min_d) > 20) {
        --mhi;
        if (mlen) --mlen;
        while (!get_m(mhi)) {
            if (mlo == mhi) break;
            --mhi;
            if (mlen) --mlen;
        }
        if (!mlen || !(L.Mt(ns, FM, mlen - 1) & 1u)) return SALN_REF_PANIC_TRIM;
        next_d = dist(L.O(ns, FM, mlen - 1), l1, l2, mhi);
    }
    L.H(ns, FM, 1) = mlo;
    L.H(ns, FM, 2) = mhi;
    L.H(ns, FM, 3) = (int32_t)mlen;
    // clamp I then D to M (:574-622); `len - t` wraps in release (truncate no-op)
    for (int f = FI; f <= FD; ++f) {
        if (!L.H(ns, f, 0)) continue;
        const int32_t flo = L.H(ns, f, 1), fhi = L.H(ns, f, 2);
        const uint32_t flen = (uint32_t)L.H(ns, f, 3);
        uint64_t t;
        if (flo < mlo) {
            const uint32_t mid = adiff(flo, mlo);
            if (mid > flen) return SALN_REF_PANIC_TRIM;  // rotate_left assert
            rotate_left(L, ns, f, flen, mid);
            t = (uint64_t)mid + (fhi > mhi ? adiff(fhi, mhi) : 0u);
        } else if (fhi > mhi) {
            t = adiff(fhi, mhi);
        } else {
            t = 0;
        }
        if (t <= flen) L.H(ns, f, 3) = (int32_t)(flen - t);
        L.H(ns, f, 2) = min(fhi, mhi);
        L.H(ns, f, 1) = max(flo, mlo);
    }
    return SALN_OK;
}

// WaveFrontTensor::is_converged (:422-439) on slot ns, fronts i, d, m
__device__ bool converged(const LaneArena &L, uint32_t ns, int32_t l1, int32_t l2, Elem &out) {
    if (!L.T(ns)) return false;
    const int f_order[3] = {FI, FD, FM};
    for (int q = 0; q < 3; ++q) {
        const int f = f_order[q];
        if (!L.H(ns, f, 0)) continue;
        const int32_t lo = L.H(ns, f, 1), n = L.H(ns, f, 3);
        for (int32_t k = 0; k < n; ++k) {
            const Elem e = L.at(ns, f, (uint32_t)k);
            if (!e.some) continue;
            const int32_t diag = lo + k;
            if (ex(e.offset, diag) == (int64_t)l2 - 1 && ey(e.offset, diag) == (int64_t)l1 - 1) {
                out = e;
                return true;
            }
        }
    }
    return false;
}

enum { EV_WELL = 0, EV_YEAH = 1, EV_MISMATCH = 2, EV_EXTEND = 3, EV_OPEN = 4, EV_RET = 5, EV_HUH = 6 };

struct Row {
    uint8_t *p;
    uint32_t n, cap;
    bool over;
};
// row.extend(seq[a..b].iter().rev()); false = slice panic
__device__ bool extend_rev(Row &r, const uint8_t *s, int32_t len, int64_t a, int64_t b) {
    if (a < 0 || b < 0 || a > b || b > len) return false;
    for (int64_t k = b; k > a; --k) {
        if (r.n < r.cap) r.p[r.n] = s[k - 1];
        else r.over = true;
        ++r.n;
    }
    return true;
}
__device__ void push(Row &r, uint8_t c) {
    if (r.n < r.cap) r.p[r.n] = c;
    else r.over = true;
    ++r.n;
}
__device__ bool has_parent(uint32_t meta, uint32_t st) {
    for (uint32_t k = 0; k < m_np(meta); ++k)
        if (m_par(meta, k) == st) return true;
    return false;
}

}  // namespace

__global__ __launch_bounds__(256) void wfa_kernel(const WfaPairDesc *__restrict__ pairs,
                                                  uint32_t first, uint32_t n,
                                                  const uint8_t *__restrict__ qs,
                                                  const uint8_t *__restrict__ ds, WfaArena arena,
                                                  uint32_t max_steps, saln_wfa_result *results,
                                                  uint8_t *aln, int32_t *lohi_log, uint8_t *ev_log,
                                                  uint32_t ev_cap, WfaPairDesc *rerun,
                                                  uint32_t *rerun_cnt) {
    const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= n) return;
    const WfaPairDesc p = pairs[first + l];
    const LaneArena L{arena, l};
    const uint8_t *s1 = qs + p.q_off, *s2 = ds + p.db_off;  // seq1 = query, seq2 = db
    const int32_t l1 = (int32_t)p.len_q, l2 = (int32_t)p.len_db;
    saln_wfa_result r{};
    if (p.mode != SALN_MODE_GLOBAL) {
        r.status = SALN_NOT_IMPLEMENTED;
        results[p.pair_id] = r;
        return;
    }
    int32_t *lohi = lohi_log ? lohi_log + (size_t)p.pair_id * 2 * max_steps : nullptr;
    // Ocean::global (:450-465)
    for (uint32_t s = 0; s < arena.S; ++s) L.T(s) = 0;
    L.T(0) = 1;
    L.H(0, FI, 0) = 0;
    L.H(0, FD, 0) = 0;
    L.H(0, FM, 0) = 1;
    L.H(0, FM, 1) = 0;
    L.H(0, FM, 2) = 0;
    L.H(0, FM, 3) = 1;
    L.put(0, FM, 0, Elem{true, 0, mk_meta(SM, 0, 0)});
    int64_t len = 1;  // wfs.len()
    uint32_t steps = 0;
    int status = SALN_OK;
    Elem conv{false, 0, 0};
    for (;;) {
        const bool newest_even = !((len - 1) & 1);
        if (newest_even && converged(L, (uint32_t)((len - 1) / 2), l1, l2, conv)) break;
        if (steps >= max_steps) {
            if (rerun) {  // short first pass: hand the pair to the full-cap pass
                rerun[atomicAdd(rerun_cnt, 1u)] = p;
                return;
            }
            status = SALN_NONCONVERGED;
            break;
        }
        // Ocean::expand (:467-488)
        const int64_t s = len;
        int32_t lh[2] = {INT32_MIN, 0};
        if (!(s & 1)) {
            const uint32_t ns = (uint32_t)(s / 2);
            if (ns >= arena.S) {
                status = SALN_NONCONVERGED;
                break;
            }
            bool some = false;
            if (!tensor_new(L, s, ns, lh, some)) {
                if (lohi) lohi[2 * steps] = lh[0], lohi[2 * steps + 1] = lh[1];
                ++steps;
                status = SALN_NONCONVERGED;  // width cap
                break;
            }
            if (some) extend_m(L, ns, s1, l1, s2, l2);
            if (lohi) lohi[2 * steps] = lh[0], lohi[2 * steps + 1] = lh[1];
            ++len;
            ++steps;
            if (some && (status = trim(L, ns, l1, l2)) != SALN_OK) break;
        } else {
            if (lohi) lohi[2 * steps] = lh[0], lohi[2 * steps + 1] = lh[1];
            ++len;
            ++steps;
        }
    }
    r.steps = steps;
    r.score = (int32_t)len;
    if (status == SALN_OK) {
        r.conv_offset = conv.offset;
        r.conv_state = (uint8_t)m_state(conv.meta);
        r.conv_np = (uint8_t)m_np(conv.meta);
        for (uint32_t k = 0; k < 3; ++k) r.conv_parents[k] = (uint8_t)(k < r.conv_np ? m_par(conv.meta, k) : 0);
        // traceback / rec_tr (:634-853)
        uint8_t *ev = ev_log ? ev_log + (size_t)p.pair_id * ev_cap : nullptr;
        uint32_t nev = 0;
        auto log = [&](uint8_t c) {
            if (ev && nev < ev_cap) ev[nev] = c;
            ++nev;
        };
        Row a1{aln ? aln + p.aln_off : nullptr, 0, aln ? p.aln_cap : 0u, false};
        Row a2{aln ? aln + p.aln_off + p.aln_cap : nullptr, 0, aln ? p.aln_cap : 0u, false};
        int32_t diag = l1 - l2;
        Elem ne = conv;
        uint64_t score = (uint64_t)len;
        for (;;) {
            if (diag == 0 && ne.offset == 0) {
                log(EV_RET);
                break;
            }
            bool moved = false;
            for (int q = 0; q < 3 && !moved; ++q) {
                const uint64_t nd = q == 0 ? 4 : q == 1 ? 6 : 8;
                if (nd > score) {
                    log(EV_WELL);
                    continue;
                }
                const uint64_t nsc = score - nd;
                log(EV_YEAH);
                if (nsc >= (uint64_t)len) continue;
                const bool tv = !(nsc & 1) && L.T((uint32_t)(nsc / 2));
                const uint32_t ts = (uint32_t)(nsc / 2);
                Elem w{false, 0, 0};
                int kind = 0;
                if (nd == 4) {
                    if (m_state(ne.meta) != SM && has_parent(ne.meta, SM) &&
                        (w = L.get(tv, ts, FM, diag)).some) {
                        log(EV_MISMATCH);
                        kind = 1;
                    }
                } else if (nd == 6) {
                    if (has_parent(ne.meta, SD) && (w = L.get(tv, ts, FD, diag - 1)).some) {
                        log(EV_EXTEND);
                        kind = 2;
                    } else if ((w = L.get(tv, ts, FI, diag + 1)).some) {
                        log(EV_EXTEND);
                        kind = 3;
                    }
                } else if (has_parent(ne.meta, SM)) {
                    log(EV_OPEN);
                    const uint32_t st = m_state(ne.meta);
                    if (st == SD) {
                        if ((w = L.get(tv, ts, FD, diag - 1)).some) kind = 2;
                    } else if (st == SI) {
                        if ((w = L.get(tv, ts, FI, diag + 1)).some) kind = 3;
                    } else {
                        if ((w = L.get(tv, ts, FI, diag + 1)).some) kind = 3;
                        else if ((w = L.get(tv, ts, FD, diag - 1)).some) kind = 4;
                    }
                }
                if (!kind) continue;
                bool ok = true;
                const int64_t wy = ey(w.offset, diag), ny = ey(ne.offset, diag);
                const int64_t wx = ex(w.offset, diag), nx = ex(ne.offset, diag);
                int32_t ndiag = diag;
                if (kind == 1) {
                    ok = extend_rev(a1, s1, l1, wy, ny) && extend_rev(a2, s2, l2, wx, nx);
                } else if (kind == 2) {
                    ok = extend_rev(a1, s1, l1, wy, ny);
                    if (ok) push(a2, '-'), ok = extend_rev(a2, s2, l2, wx, nx);
                    ndiag = diag - 1;
                } else if (kind == 3) {
                    push(a1, '-');
                    ok = extend_rev(a1, s1, l1, wy, ny) && extend_rev(a2, s2, l2, wx, nx);
                    ndiag = diag + 1;
                } else {
                    ok = extend_rev(a1, s1, l1, wy, ny);
                    if (ok) push(a1, '-'), ok = extend_rev(a2, s2, l2, wx, nx);
                    ndiag = diag - 1;
                }
                if (!ok) {
                    status = SALN_REF_PANIC_SLICE;
                    break;
                }
                ne = w;
                diag = ndiag;
                score = nsc;
                moved = true;
            }
            if (status != SALN_OK) break;
            if (!moved) {
                log(EV_HUH);
                break;
            }
        }
        r.aln_len1 = a1.n;
        r.aln_len2 = a2.n;
        if (a1.over || a2.over || nev > ev_cap) r.reserved[0] = 1;  // a buffer was too small
    }
    r.status = status;
    results[p.pair_id] = r;
}

hipError_t launch_wfa(const WfaPairDesc *pairs, uint32_t first, uint32_t n, const uint8_t *qs,
                      const uint8_t *ds, const WfaArena &arena, uint32_t max_steps,
                      saln_wfa_result *results, uint8_t *aln, int32_t *lohi_log, uint8_t *ev_log,
                      uint32_t ev_cap, WfaPairDesc *rerun, uint32_t *rerun_cnt,
                      hipStream_t stream) {
    if (!n) return hipSuccess;
    wfa_kernel<<<dim3((n + 255) / 256), dim3(256), 0, stream>>>(
        pairs, first, n, qs, ds, arena, max_steps, results, aln, lohi_log, ev_log, ev_cap, rerun,
        rerun_cnt);
    return hipGetLastError();
}

}  // namespace saln

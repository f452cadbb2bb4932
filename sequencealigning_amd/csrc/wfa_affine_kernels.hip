// Corrected gap-affine WFA on gfx950.
//
// The reference's wfa_align (src/wfa.rs:23-42) keeps x = 4, o = 2, e = 6
// (wfa.rs:14-21) but defines no output for realistic inputs (Ocean::trim
// panics at s = 20); the engine for that path is
// wfa_kernels.hip, with the reference's exact semantics.  This file is a
// separately labelled engine that computes what a gap-affine WFA is meant to
// compute: the minimum penalty x * mismatches + sum(o + e * len) over gaps of
// a global alignment (checked against the Gotoh DP in oracle/refaffine.c).
//
// Wavefront recurrences (pattern = query, v; text = db, h; diagonal
// k = h - v; a wavefront entry is the furthest text offset h reaching score s
// on diagonal k):
//   I[s][k] = max(M[s-o-e][k-1], I[s-e][k-1]) + 1
//   D[s][k] = max(M[s-o-e][k+1], D[s-e][k+1])
//   M[s][k] = max(M[s-x][k] + 1, I[s][k], D[s][k]), then extended along
//             matching bases.
// The first s with M[s][ld - lq] == ld is the penalty.  Scores come in units
// of g = gcd(x, o+e, e); the wavefronts needed are the last (o+e)/g (M) and
// e/g (I, D) steps, kept in an LDS ring per wave.
//
// Geometry: one wave per pair (a persistent grid walks the pairs), lanes over
// the diagonals of a step in chunks of 64; the ring holds W (a power of two)
// diagonals per wavefront at index k & (W-1), with each slot's [lo, hi]
// range in LDS; reads outside a source's range are -inf.  Offsets are i16
// (pairs up to 32,000 bases; i32 above).  Extension compares 4 bases at a
// time from the sequences in global memory (L1/L2-resident per pair).
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <type_traits>

#include "wfa_affine.hpp"

namespace saln {

namespace {

constexpr int kRingMax = 16;
// An empty range is (kEmptyLo, -kEmptyLo): min / max of ranges and the +-1
// of the recurrences keep it empty without tests.
constexpr int32_t kEmptyLo = 1 << 29;
typedef __attribute__((address_space(3))) uint8_t lds_cu8_raw;
typedef const lds_cu8_raw lds_cu8;
typedef const __attribute__((address_space(3))) uint32_t lds_cu32;

template <typename OffT>
struct OffTraits;
template <>
struct OffTraits<int16_t> {
    static constexpr int32_t kNeg = -32768;
};
template <>
struct OffTraits<int32_t> {
    static constexpr int32_t kNeg = INT32_MIN / 4;
};

// 4 bytes at p (4-aligned or not) from the two aligned dwords covering them.
// Global sequences: both dwords hold a byte of the sequence (callers check 5
// readable bytes at p), so nothing past the sequence's last dword is read.
// LDS sequences: the staged copy is padded.
template <typename P>
__device__ __forceinline__ uint32_t load4(P p) {
    const uintptr_t a = (uintptr_t)p;
    typedef typename std::remove_pointer<P>::type cu8;
    typedef typename std::conditional<std::is_same<cu8, const lds_cu8>::value, const lds_cu32,
                                      const uint32_t>::type cu32;
    cu32 *w = (cu32 *)(a & ~(uintptr_t)3);
    return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(a & 3));
}

// Extend (v, h) along matching bases: returns the new text offset.
template <typename P>
__device__ __forceinline__ int32_t extend(P q, int32_t lq, P d, int32_t ld, int32_t v, int32_t h) {
    for (;;) {
        if (v + 5 <= lq && h + 5 <= ld) {
            const uint32_t x = load4(q + v) ^ load4(d + h);
            if (x) return h + (int32_t)(__builtin_ctz(x) >> 3);
            v += 4;
            h += 4;
        } else {
            while (v < lq && h < ld && q[v] == d[h]) {
                ++v;
                ++h;
            }
            return h;
        }
    }
}

// Score of one pair (q, d in global memory or staged in LDS): the first s
// whose M wavefront reaches (lq, ld); -1 above max_score, -2 ring too narrow.
// kSafe0: the sequences have >= 8 readable bytes at q and d (staged in LDS,
// or long enough), so a probe that is not taken may still load there.
template <typename OffT, int CM, bool kSafe0, typename P>
__device__ __forceinline__ int32_t wfa_pair(P q, int32_t lq, P d, int32_t ld, const WfaAffParams &prm,
                            int32_t *rng, OffT *Mr, OffT *Ir, OffT *Dr) {
    constexpr int32_t kNeg = OffTraits<OffT>::kNeg;
    const int32_t lane = (int32_t)threadIdx.x;
    const int32_t W = prm.W, wm = prm.W - 1;
    const int32_t tx = prm.x / prm.g, toe = (prm.o + prm.e) / prm.g, te = prm.e / prm.g;
    const int32_t kend = ld - lq;
    __builtin_amdgcn_wave_barrier();
    if (lane < 3 * kRingMax) {  // every slot empty
        rng[2 * lane] = kEmptyLo;
        rng[2 * lane + 1] = -kEmptyLo;
    }
    // s = 0: M[0][0] = 0, extended
    if (lane == 0) {
        Mr[0] = (OffT)extend(q, lq, d, ld, 0, 0);
        rng[0] = 0;
        rng[1] = 0;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    if (kend == 0 && (int32_t)Mr[0] >= ld) return 0;
    // ring slots of step t and of its sources, advanced without divisions
    auto wrap = [](int32_t v, int32_t r) { return v < 0 ? v + r : v; };
    int32_t sM = 0, sI = 0;  // slot of step t (t % RM, t % RI)
    for (int32_t t = 1;; ++t) {
        const int32_t s = t * prm.g;
        if (s > prm.max_score) return -1;
        sM = sM + 1 == prm.RM ? 0 : sM + 1;
        sI = sI + 1 == prm.RI ? 0 : sI + 1;
        // sources (slot, range); a negative step or an empty slot has lo > hi
        auto src = [&](int comp, int32_t ts, int32_t slot_now, int32_t back, int32_t ring,
                       int32_t &slot, int32_t &lo, int32_t &hi) __attribute__((always_inline)) {
            if (ts < 0) {
                slot = 0;
                lo = kEmptyLo;
                hi = -kEmptyLo;
                return;
            }
            slot = wrap(slot_now - back, ring);  // back < ring
            lo = rng[2 * (comp * kRingMax + slot)];
            hi = rng[2 * (comp * kRingMax + slot) + 1];
        };
        int32_t soe, loMo, hiMo, sx, loMx, hiMx, sie, loI, hiI, sde, loD, hiD;
        src(0, t - toe, sM, toe, prm.RM, soe, loMo, hiMo);
        src(0, t - tx, sM, tx, prm.RM, sx, loMx, hiMx);
        src(1, t - te, sI, te, prm.RI, sie, loI, hiI);
        src(2, t - te, sI, te, prm.RI, sde, loD, hiD);
        // new ranges (empty sources are (kEmptyLo, -kEmptyLo) and stay out of
        // every min / max below; a clamp that empties a range is re-marked)
        int32_t iLo = max(min(loMo, loI) + 1, -lq), iHi = min(max(hiMo, hiI) + 1, ld);
        int32_t dLo = max(min(loMo, loD) - 1, -lq), dHi = min(max(hiMo, hiD) - 1, ld);
        if (iLo > iHi) iLo = kEmptyLo, iHi = -kEmptyLo;
        if (dLo > dHi) dLo = kEmptyLo, dHi = -kEmptyLo;
        const int32_t xLo = max(loMx, -lq), xHi = min(hiMx, ld);
        int32_t mLo = min(min(iLo, dLo), xLo <= xHi ? xLo : kEmptyLo);
        int32_t mHi = max(max(iHi, dHi), xLo <= xHi ? xHi : -kEmptyLo);
        if (mLo > mHi) {  // nothing at this score
            if (lane == 0) {
                rng[2 * sM] = kEmptyLo, rng[2 * sM + 1] = -kEmptyLo;
                rng[2 * (kRingMax + sI)] = kEmptyLo, rng[2 * (kRingMax + sI) + 1] = -kEmptyLo;
                rng[2 * (2 * kRingMax + sI)] = kEmptyLo, rng[2 * (2 * kRingMax + sI) + 1] = -kEmptyLo;
            }
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_wave_barrier();
            continue;
        }
        if (mHi - mLo + 1 > W) return -2;  // the ring is too narrow: re-run with a wider one
        // LDS reads are always in bounds (k & wm), so a range test is a select.
        // Predicates are arithmetic (one unsigned compare, or one max3 and a
        // compare) so they cost VALU only, no SALU mask combining.  An empty
        // source gets lo = 2^30, span 0: k - lo never passes.
        auto span_of = [](int32_t &lo, int32_t hi) {  // empty: lo = 2^29, span 0
            return (uint32_t)max(hi - lo, 0);
        };
        const uint32_t spMo = span_of(loMo, hiMo), spMx = span_of(loMx, hiMx);
        const uint32_t spI = span_of(loI, hiI), spD = span_of(loD, hiD);
        auto rd = [&](const OffT *ring, int32_t slot, int32_t k, int32_t lo,
                      uint32_t sp) __attribute__((always_inline)) {
            const int32_t v = (int32_t)ring[slot * W + (k & wm)];
            return (uint32_t)(k - lo) <= sp ? v : kNeg;
        };
        // an offset h on diagonal k is a cell iff 0 <= h <= ld and h - k <= lq
        auto cell = [&](int32_t h, int32_t k) __attribute__((always_inline)) {
            return max(max(-h, h - ld), h - k - lq) <= 0;
        };
        // Target slots (t % RM, t % RI) differ from every source slot
        // (RM > max(toe, tx), RI > te), so chunks read and write freely.
        // Groups of 4 chunks (256 diagonals) are branch-free so the LDS / HBM
        // latencies of the 4 overlap: A) I, D and the pre-extension M (reads
        // only); B) the first 4-base comparison of every chunk; C) the rare
        // longer extensions and the writes.  Lanes past mHi compute -inf and
        // write it: entries outside a slot's stored range are never read, and
        // a group never spans more than W diagonals, so nothing valid is hit.
        // (I and D outside their own ranges read -inf from both sources.)
        const int32_t span = mHi - mLo;
#pragma unroll
        for (int g = 0; g < CM / 4; ++g) {
            if (256 * g > span) break;  // uniform
            int32_t Mv[4], Iv[4], Dv[4];
            bool slow[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int32_t k = mLo + 64 * (4 * g + c) + lane;
                int32_t I = max(rd(Mr, soe, k - 1, loMo, spMo), rd(Ir, sie, k - 1, loI, spI)) + 1;
                I = cell(I, k) ? I : kNeg;
                int32_t D = max(rd(Mr, soe, k + 1, loMo, spMo), rd(Dr, sde, k + 1, loD, spD));
                D = cell(D, k) ? D : kNeg;
                int32_t X = rd(Mr, sx, k, loMx, spMx) + 1;
                X = cell(X, k) ? X : kNeg;
                const int32_t M = max(X, max(I, D));
                Iv[c] = I;
                Dv[c] = D;
                Mv[c] = (uint32_t)(k - mLo) <= (uint32_t)span ? M : kNeg;
            }
            uint32_t more = 0;  // bit c: chunk c's lane matched 4 bases, keep extending
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int32_t k = mLo + 64 * (4 * g + c) + lane;
                const int32_t M = Mv[c];
                const int32_t v = M - k;
                const bool fast = kSafe0 && max(max(-M, v + 5 - lq), M + 5 - ld) <= 0;
                slow[c] = M >= 0 && !fast;
                if constexpr (kSafe0) {  // loads at a safe address when not fast
                    const uint32_t x = load4(q + (fast ? v : 0)) ^ load4(d + (fast ? M : 0));
                    const int32_t adv = x ? (int32_t)(__builtin_ctz(x) >> 3) : 4;
                    Mv[c] = fast ? M + adv : M;
                    more |= (fast && !x) ? 1u << c : 0u;
                }
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int32_t k = mLo + 64 * (4 * g + c) + lane;
                int32_t M = Mv[c];
                if (slow[c] || ((more >> c) & 1u)) M = extend(q, lq, d, ld, M - k, M);
                Mr[sM * W + (k & wm)] = (OffT)M;
                Ir[sI * W + (k & wm)] = (OffT)Iv[c];
                Dr[sI * W + (k & wm)] = (OffT)Dv[c];
            }
        }
        if (lane == 0) {  // I / D entries outside their own ranges were written as -inf
            rng[2 * sM] = mLo, rng[2 * sM + 1] = mHi;
            rng[2 * (kRingMax + sI)] = iLo, rng[2 * (kRingMax + sI) + 1] = iHi;
            rng[2 * (2 * kRingMax + sI)] = dLo, rng[2 * (2 * kRingMax + sI) + 1] = dHi;
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        if (kend >= mLo && kend <= mHi && (int32_t)Mr[sM * W + (kend & wm)] >= ld) return s;
    }
}

// Copy len bytes at src into LDS at dst (16-byte granules from src & ~15,
// so the copy starts at dst + (src & 15)); returns the staged pointer.
__device__ __forceinline__ lds_cu8 *stage(const uint8_t *src, int32_t len, lds_cu8_raw *dst) {
    const uintptr_t a = (uintptr_t)src, base = a & ~(uintptr_t)15;
    const int32_t nblk = (int32_t)((((a + (uintptr_t)len + 15) & ~(uintptr_t)15) - base) / 16);
    typedef __attribute__((address_space(3))) uint32_t lds_u32;
    for (int32_t i = (int32_t)threadIdx.x; i < nblk; i += 64) {
        const uint4 v = ((const uint4 *)base)[i];
        lds_u32 *w = (lds_u32 *)dst + 4 * i;
        w[0] = v.x, w[1] = v.y, w[2] = v.z, w[3] = v.w;
    }
    return dst + (a & 15);
}

template <typename OffT>
__global__ __launch_bounds__(64) void wfa_affine_kernel(const WfaAffPair *__restrict__ pairs,
                                                        uint32_t n_pairs,
                                                        const uint8_t *__restrict__ qs,
                                                        const uint8_t *__restrict__ ds,
                                                        WfaAffParams prm,
                                                        const uint32_t *__restrict__ n_dev,
                                                        int32_t *__restrict__ scores) {
    if (n_dev) n_pairs = *n_dev;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_raw[];
    // ranges: [component][slot] = (lo, hi); component 0 M, 1 I, 2 D
    int32_t *rng = (int32_t *)lds_raw;
    OffT *Mr = (OffT *)(lds_raw + 3 * kRingMax * 2 * sizeof(int32_t));
    OffT *Ir = Mr + prm.RM * prm.W;
    OffT *Dr = Ir + prm.RI * prm.W;
    // staged sequences (prm.seqcap bytes, 16-aligned after the rings)
    lds_cu8_raw *sbuf = (lds_cu8_raw *)(((uintptr_t)(Dr + prm.RI * prm.W) + 15) & ~(uintptr_t)15);
    const int32_t lane = (int32_t)threadIdx.x;

    for (uint32_t pi = blockIdx.x; pi < n_pairs; pi += gridDim.x) {
        const WfaAffPair p = pairs[pi];
        const int32_t lq = (int32_t)p.lq, ld = (int32_t)p.ld;
        const uint8_t *__restrict__ q = qs + p.q_off;
        const uint8_t *__restrict__ d = ds + p.d_off;
        int32_t result;
        if (lq == 0 || ld == 0) {  // one gap (or nothing)
            const int32_t len = lq + ld;
            result = len == 0 ? 0 : prm.o + prm.e * len;
            if (result > prm.max_score) result = -1;
        } else {
            const int32_t qspan = (lq + 47) & ~15;  // staged q: +15 lead, +16 tail pad
            if (qspan + ld + 48 <= prm.seqcap) {
                __builtin_amdgcn_wave_barrier();
                lds_cu8 *lq8 = stage(q, lq, sbuf);
                lds_cu8 *ld8 = stage(d, ld, sbuf + qspan);
                __builtin_amdgcn_s_waitcnt(0xC07F);
                __builtin_amdgcn_wave_barrier();
                result = prm.W == 512    ? wfa_pair<OffT, 8, true>(lq8, lq, ld8, ld, prm, rng, Mr, Ir, Dr)
                         : prm.W == 1024 ? wfa_pair<OffT, 16, true>(lq8, lq, ld8, ld, prm, rng, Mr, Ir, Dr)
                                         : wfa_pair<OffT, 32, true>(lq8, lq, ld8, ld, prm, rng, Mr, Ir, Dr);
            } else if (lq >= 8 && ld >= 8) {
                result = prm.W == 512    ? wfa_pair<OffT, 8, true>(q, lq, d, ld, prm, rng, Mr, Ir, Dr)
                         : prm.W == 1024 ? wfa_pair<OffT, 16, true>(q, lq, d, ld, prm, rng, Mr, Ir, Dr)
                                         : wfa_pair<OffT, 32, true>(q, lq, d, ld, prm, rng, Mr, Ir, Dr);
            } else {
                result = prm.W == 512    ? wfa_pair<OffT, 8, false>(q, lq, d, ld, prm, rng, Mr, Ir, Dr)
                         : prm.W == 1024 ? wfa_pair<OffT, 16, false>(q, lq, d, ld, prm, rng, Mr, Ir, Dr)
                                         : wfa_pair<OffT, 32, false>(q, lq, d, ld, prm, rng, Mr, Ir, Dr);
            }
        }
        if (lane == 0) scores[p.out] = result;
        __builtin_amdgcn_wave_barrier();
    }
}

}  // namespace

size_t wfa_affine_lds_bytes(const WfaAffParams &prm, bool wide) {
    const size_t rings = 3 * kRingMax * 2 * sizeof(int32_t) +
                         (size_t)(prm.RM + 2 * prm.RI) * prm.W *
                             (wide ? sizeof(int32_t) : sizeof(int16_t));
    return ((rings + 15) & ~(size_t)15) + (size_t)prm.seqcap;
}

hipError_t launch_wfa_affine(const WfaAffPair *pairs, uint32_t n, const uint8_t *qs,
                             const uint8_t *ds, const WfaAffParams &prm, bool wide,
                             uint32_t grid, const uint32_t *n_dev, int32_t *scores,
                             hipStream_t stream) {
    if (!n) return hipSuccess;
    const size_t lds = wfa_affine_lds_bytes(prm, wide);
    if (wide)
        wfa_affine_kernel<int32_t><<<dim3(grid), dim3(64), lds, stream>>>(pairs, n, qs, ds, prm,
                                                                          n_dev, scores);
    else
        wfa_affine_kernel<int16_t><<<dim3(grid), dim3(64), lds, stream>>>(pairs, n, qs, ds, prm,
                                                                          n_dev, scores);
    return hipGetLastError();
}

namespace {
// Pairs of pass 1 that outgrew the ring (score -2) -> rerun list.
__global__ void wfa_affine_compact_kernel(const WfaAffPair *__restrict__ pairs, uint32_t n,
                                          const int32_t *__restrict__ scores,
                                          WfaAffPair *__restrict__ out,
                                          uint32_t *__restrict__ count) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const WfaAffPair p = pairs[i];
    if (scores[p.out] == -2) out[atomicAdd(count, 1u)] = p;
}
}  // namespace

hipError_t launch_wfa_affine_compact(const WfaAffPair *pairs, uint32_t n, const int32_t *scores,
                                     WfaAffPair *out, uint32_t *count, hipStream_t stream) {
    if (!n) return hipSuccess;
    wfa_affine_compact_kernel<<<dim3((n + 255) / 256), dim3(256), 0, stream>>>(pairs, n, scores,
                                                                             out, count);
    return hipGetLastError();
}

}  // namespace saln

// NW-affine fill + canonical traceback kernels for gfx950 (MI355X).
//
// Reference path: src/needleman_wunsch_affine.rs — ScoreTensor::fill :169-237
// (recurrences m_score/i_score/d_score :76-94, parent lists :96-153) and
// ScoreTensor::traceback :242-334.
//
// Fill geometry ("skewed row pipeline"): a group of G lanes (G = 16: one DPP
// row; G = 64: the whole wave) owns one pair.  Lane l owns K consecutive
// query columns of the current chunk and walks the db rows; at step t it
// computes row r = t - l + 1, so the left neighbour finished the same row one
// step earlier.  The only cross-lane traffic per step is two DPP shifts
// (the row's I candidate leaving the lane's last column and the last
// column's H), fused as update_dpp moves.  Each lane keeps its previous-row
// H and next-row D for its K columns in registers; nothing else of the matrix
// is stored except the 7-bit parent code per cell (1 B/cell), written
// [step][lane][ceil(K/4) dwords] so every step is one contiguous store per
// group.
#include <hip/hip_runtime.h>

#include "nw_common.hpp"
#include "saln.h"

namespace saln {

// lane i <- lane i-1 within the group; the group's lane 0 keeps `old`.
template <int G>
__device__ __forceinline__ int32_t shr1(int32_t old, int32_t v) {
    static_assert(G == 16 || G == 64, "group must be a DPP row or the wave");
    if constexpr (G == 16)
        return __builtin_amdgcn_update_dpp(old, v, 0x111 /*row_shr:1*/, 0xf, 0xf, false);
    else
        return __builtin_amdgcn_update_dpp(old, v, 0x138 /*wave_shr:1*/, 0xf, 0xf, false);
}

template <int K>
struct MaskWords {
    uint32_t w[(K + 3) / 4];
};

template <int G, int K>
__global__ __launch_bounds__(256) void nw_fill_kernel(const NwPairDesc *__restrict__ pairs,
                                                      uint32_t first, uint32_t count,
                                                      const uint8_t *__restrict__ qs,
                                                      const uint8_t *__restrict__ ds,
                                                      uint8_t *__restrict__ mask,
                                                      int2 *__restrict__ scratch,
                                                      int32_t *__restrict__ end_h, Scoring sc) {
    constexpr int GPB = 256 / G;
    constexpr int KD = (K + 3) / 4;
    constexpr Geom geo{G, K};
    const int lane = threadIdx.x % G;
    const uint32_t gi = blockIdx.x * GPB + threadIdx.x / G;
    if (gi >= count) return;  // whole group (DPP never crosses groups)
    const NwPairDesc p = pairs[first + gi];
    const uint32_t lq = p.len_q, ld = p.len_db;
    const uint8_t *__restrict__ q = qs + p.q_off;
    const uint8_t *__restrict__ d = ds + p.db_off;
    uint8_t *__restrict__ mk = mask + p.mask_off;
    int2 *__restrict__ scr = scratch + p.scratch_off;
    const uint32_t nch = geo.n_chunks(lq);
    const int T = (int)ld + G - 1;
    const int32_t sM = 2 * sc.match, sX = 2 * sc.mismatch;
    const int32_t sO = 2 * sc.gap_open, sE = 2 * sc.gap_extend;
    // end cell owner
    const uint32_t jend = lq - 1;
    const uint32_t c_end = jend / geo.W(), l_end = (jend % geo.W()) / K, k_end = jend % K;

    for (uint32_t c = 0; c < nch; ++c) {
        const uint32_t col0 = c * geo.W() + (uint32_t)lane * K;  // my columns: col0+1 .. col0+K
        int32_t qc[K], Hp[K], Dn[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t j = col0 + k + 1;
            qc[k] = j <= lq ? (int32_t)q[j - 1] : -1;
            Hp[k] = hs_row0(sc, j);  // H'(0, j)
            Dn[k] = ds_row1(sc, j);  // D'(1, j)
        }
        int32_t hd = hs_row0(sc, col0);  // H'(r-1, col0): diagonal of my first column
        int32_t pubF = 0, pubH = 0;
        int32_t dnext = (lane == 0) ? (int32_t)d[0] : 0;
        int2 bnext = make_int2(0, 0);
        if (c > 0 && lane == 0) bnext = scr[1];
        uint8_t *mchunk = mk + (uint64_t)c * geo.chunk_bytes(ld);

        for (int t = 0; t < T; ++t) {
            const int r = t - lane + 1;
            const int32_t dch = dnext;
            if (r >= 0 && r < (int)ld) dnext = (int32_t)d[r];
            int32_t bF, bH;
            if (c == 0) {
                bF = is_col1(sc, (uint32_t)(t + 1));
                bH = hs_col0(sc, (uint32_t)(t + 1));
            } else {
                bH = bnext.x;
                bF = bnext.y;
                if (lane == 0 && t + 2 <= (int)ld) bnext = scr[t + 2];
            }
            const int32_t inF = shr1<G>(bF, pubF);  // I'(r, col0+1)
            const int32_t inH = shr1<G>(bH, pubH);  // H'(r, col0)
            if (r >= 1 && r <= (int)ld) {
                int32_t F = inF;
                MaskWords<K> mw;
#pragma unroll
                for (int k = 0; k < KD; ++k) mw.w[k] = 0;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const int32_t M = hd + (qc[k] == dch ? sM : sX);
                    const int32_t I = F, D = Dn[k];
                    const int32_t H = max(M, max(I, D));
                    const int32_t Hc = H & ~1;
                    const int32_t tO = M + sO;
                    uint32_t b = (M >= Hc ? kArgM : 0u) | (I >= Hc ? kArgI : 0u) |
                                 (D >= Hc ? kArgD : 0u);
                    b |= ((I | 1) >= tO ? kIExt : 0u) | ((tO | 1) >= I ? kIOpen : 0u);
                    b |= ((D | 1) >= tO ? kDExt : 0u) | ((tO | 1) >= D ? kDOpen : 0u);
                    mw.w[k / 4] |= b << (8 * (k % 4));
                    F = max(tO, I) + sE;
                    Dn[k] = max(tO, D) + sE;
                    hd = Hp[k];
                    Hp[k] = H;
                }
                hd = inH;
                pubF = F;
                pubH = Hp[K - 1];
                *reinterpret_cast<MaskWords<K> *>(mchunk + (uint64_t)t * geo.step_bytes() +
                                                  (uint32_t)lane * KD * 4) = mw;
                if (lane == G - 1 && c + 1 < nch) scr[r] = make_int2(pubH, pubF);
                if (c == c_end && (uint32_t)lane == l_end && r == (int)ld) {
                    int32_t e = 0;
#pragma unroll
                    for (int k = 0; k < K; ++k)
                        if ((uint32_t)k == k_end) e = Hp[k];
                    end_h[first + gi] = e;
                }
            }
        }
        if (c + 1 < nch) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
}

// --------------------------------------------------------------- traceback
struct GeomTable {
    Geom g[4];
};

struct MaskCell {
    const uint8_t *m;
    Geom g;
    uint32_t lq, ld;
    Scoring sc;
    __device__ uint8_t byte(uint32_t i, uint32_t j) const { return m[g.cell(i, j, ld)]; }
    __device__ uint8_t argmax(uint32_t i, uint32_t j) const {
        if (i == 0) return argmax_row0(sc, j);
        if (j == 0) return argmax_col0(sc, i);
        return byte(i, j) & 7;
    }
    __device__ uint8_t ibits(uint32_t i, uint32_t j) const {  // i, j >= 1
        return j == 1 ? ibits_col1(sc, i) : (byte(i, j - 1) >> 3) & 3;
    }
    __device__ uint8_t dbits(uint32_t i, uint32_t j) const {  // i, j >= 1
        return i == 1 ? dbits_row1(sc, j) : (byte(i - 1, j) >> 5) & 3;
    }
};

enum { kStM = 0, kStI = 1, kStD = 2 };
enum { kEvOrigin = 0, kEvPanic = 1, kEvDead = 2 };

// Canonical (first printed) alignment: the reference DFS pops end states in
// the order D, M, I (:251-280 push I, M, D) and parents in reverse push order
// (M: D>I>M; I: open>extend; D: open>extend).  While no sentinel cell is
// reachable every DFS path ends at the origin or at a boundary panic node,
// so the first path is this greedy walk.  A sentinel dead end (only possible
// once len_q+len_db >~ 5,450) sets flags bit0 and the host redoes the walk
// with backtracking.
__global__ __launch_bounds__(256) void nw_traceback_kernel(
    const NwPairDesc *__restrict__ pairs, uint32_t n, const uint8_t *__restrict__ qs,
    const uint8_t *__restrict__ ds, const uint8_t *__restrict__ mask,
    const int32_t *__restrict__ end_h, saln_nw_result *__restrict__ results,
    uint32_t *__restrict__ cigar, Scoring sc, GeomTable gt) {
    const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n) return;
    const NwPairDesc p = pairs[idx];
    const uint32_t lq = p.len_q, ld = p.len_db;
    const uint8_t *q = qs + p.q_off;
    const uint8_t *d = ds + p.db_off;
    const MaskCell mc{mask + p.mask_off, gt.g[p.variant & 3], lq, ld, sc};
    const int32_t hend = (lq && ld) ? end_h[idx] : hs_boundary_end(sc, lq, ld);
    const uint8_t am_end = mc.argmax(ld, lq);
    int st = (am_end & kArgD) ? kStD : ((am_end & kArgM) ? kStM : kStI);
    uint32_t i = ld, j = lq;
    uint32_t *out = cigar ? cigar + p.cigar_off : nullptr;
    uint32_t nops = 0, run_op = 0, run_len = 0;
    int ev;
    for (;;) {
        uint32_t op;
        if (st == kStM) {
            if (i == 0 && j == 0) { ev = kEvOrigin; break; }
            if (i == 0 || j == 0) { ev = kEvDead; break; }
            op = q[j - 1] == d[i - 1] ? SALN_CIGAR_EQ : SALN_CIGAR_X;
            const uint8_t a = mc.argmax(i - 1, j - 1);
            --i;
            --j;
            st = (a & kArgD) ? kStD : ((a & kArgI) ? kStI : kStM);
        } else if (st == kStI) {
            if (j == 0) { ev = i >= 1 ? kEvPanic : kEvDead; break; }
            if (i == 0) { ev = kEvDead; break; }
            op = SALN_CIGAR_I;
            const uint8_t b = mc.ibits(i, j);
            --j;
            st = (b & 2) ? kStM : kStI;
        } else {
            if (i == 0) { ev = j >= 1 ? kEvPanic : kEvDead; break; }
            if (j == 0) { ev = kEvDead; break; }
            op = SALN_CIGAR_D;
            const uint8_t b = mc.dbits(i, j);
            --i;
            st = (b & 2) ? kStM : kStD;
        }
        if (op == run_op && run_len) {
            ++run_len;
        } else {
            if (run_len && out) out[nops] = (run_len << 4) | run_op;
            nops += run_len ? 1 : 0;
            run_op = op;
            run_len = 1;
        }
    }
    if (run_len) {
        if (out) out[nops] = (run_len << 4) | run_op;
        ++nops;
    }
    if (ev != kEvOrigin) nops = 0;
    if (out) {  // ops were produced back to front
        for (uint32_t a = 0, b = nops ? nops - 1 : 0; a < b; ++a, --b) {
            const uint32_t tmp = out[a];
            out[a] = out[b];
            out[b] = tmp;
        }
    }
    saln_nw_result r;
    r.score = hend >> 1;
    r.status = (hend & 1) ? SALN_REF_PANIC_BOUNDARY : SALN_OK;
    r.cigar_len = nops;
    r.end_states = am_end;
    r.printed = ev == kEvOrigin ? 1 : 0;
    r.flags = (ev == kEvDead ? 1 : 0) | ((ev == kEvPanic && !(hend & 1)) ? 2 : 0);
    r.reserved = 0;
    results[p.pair_id] = r;
}

// ----------------------------------------------------------------- launchers
constexpr Geom kVariants[4] = {{16, 10}, {16, 16}, {64, 8}, {64, 16}};

hipError_t launch_fill(int variant, const NwPairDesc *pairs, uint32_t first, uint32_t count,
                       const uint8_t *qs, const uint8_t *ds, uint8_t *mask, int2 *scratch,
                       int32_t *end_h, Scoring sc, hipStream_t stream) {
    if (count == 0) return hipSuccess;
    const uint32_t gpb = 256 / kVariants[variant].G;
    const dim3 grid((count + gpb - 1) / gpb), block(256);
    switch (variant) {
        case 0:
            nw_fill_kernel<16, 10><<<grid, block, 0, stream>>>(pairs, first, count, qs, ds, mask,
                                                                scratch, end_h, sc);
            break;
        case 1:
            nw_fill_kernel<16, 16><<<grid, block, 0, stream>>>(pairs, first, count, qs, ds, mask,
                                                                scratch, end_h, sc);
            break;
        case 2:
            nw_fill_kernel<64, 8><<<grid, block, 0, stream>>>(pairs, first, count, qs, ds, mask,
                                                               scratch, end_h, sc);
            break;
        default:
            nw_fill_kernel<64, 16><<<grid, block, 0, stream>>>(pairs, first, count, qs, ds, mask,
                                                                scratch, end_h, sc);
            break;
    }
    return hipGetLastError();
}

hipError_t launch_traceback(const NwPairDesc *pairs, uint32_t n, const uint8_t *qs,
                            const uint8_t *ds, const uint8_t *mask, const int32_t *end_h,
                            saln_nw_result *results, uint32_t *cigar, Scoring sc,
                            hipStream_t stream) {
    if (n == 0) return hipSuccess;
    GeomTable gt;
    for (int v = 0; v < 4; ++v) gt.g[v] = kVariants[v];
    nw_traceback_kernel<<<dim3((n + 255) / 256), dim3(256), 0, stream>>>(
        pairs, n, qs, ds, mask, end_h, results, cigar, sc, gt);
    return hipGetLastError();
}

Geom variant_geom(int v) { return kVariants[v]; }

int choose_variant(uint32_t len_q) {
    if (len_q <= 160) return 0;
    if (len_q <= 256) return 1;
    if (len_q <= 512) return 2;
    return 3;
}

}  // namespace saln

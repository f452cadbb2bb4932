// Row-fill step floor: the score-only row step of a lone
// wave over a 128-column stripe, i32 lanes of two columns (the shipped
// nw_fill_rows_kernel<2, kCodesNone> recurrence) against i16 x 2 lanes with
// per-row frames (lane l: column l in the low half, column 64 + l in the high
// half; every value of row r held relative to B(r) = H~(r, c0)).
// Each wave fills its own stripe from a boundary column in memory (loaded in
// 8-row groups, as the stripe hand-off does) and publishes (H~, I~) leaving
// its last column per row; there is no neighbour to wait for, so the time is
// rows x row step: the floor the shipped C4 fill (rows x step + stripes x
// hand-off lag) sits on.  Transformed recurrence as nw_kernels.hip:1853:
//   M~ = H~(r-1, c-1) - pen,  I~(r, c+1) = max(I~(r, c), M~ + O),
//   D~(r+1, c) = max(M~ + O, D~) + Ds,  H~ = max(M~, I~, D~).
// Checked against a host i32 computation on every wave's last row and
// published column.  Build: hipcc -O3 --offload-arch=gfx950 row_pk_floor.hip
// -o row_pk_floor; run: ./row_pk_floor [waves] [rows] [reps] [waves per workgroup]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int W = 128;    // columns per stripe (one wave)
constexpr int kG = 8;     // boundary rows per group
constexpr int32_t P = 36, O = -32, Ds = -68;  // pen (mismatch), open, D step (x4 scale)

typedef short s16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t u(s16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ s16x2 v2(uint32_t x) { return __builtin_bit_cast(s16x2, x); }
__device__ __forceinline__ s16x2 pmax(s16x2 a, s16x2 b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ uint32_t pk(int32_t lo, int32_t hi) {
    return ((uint32_t)lo & 0xFFFFu) | ((uint32_t)hi << 16);
}
template <int kCtrl, int kRow = 0xf, int kBank = 0xf>
__device__ __forceinline__ uint32_t dpp(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, kCtrl, kRow, kBank, false);
}

struct Args {
    const uint8_t *q;     // [waves][128]
    const uint8_t *d;     // [rows] (all waves)
    const int2 *bound;    // [waves][rows + 1 + 2 kG]: (H~(r, 0), I~(r, 1)); row 0: (H~(0,0), -)
    const int32_t *h0;    // [waves][128]: H~(0, c)
    const int32_t *d1;    // [waves][128]: D~(1, c)
    int2 *pub;            // [waves][rows + 72]: (H~(r, 128), I~ leaving); pad slots
    int32_t *last;        // [waves][128]: H~(rows, c)
    int rows;
    int waves;
};

// db chars of rows r .. r+3 from one scalar dword load (rows 4-aligned)
__device__ __forceinline__ uint32_t dword4(const uint8_t *d, int r) {
    typedef const __attribute__((address_space(4))) uint32_t cu32;
    return ((cu32 *)d)[(r - 1) >> 2];
}

// ---------------------------------------------------------------- i32, K = 2
__global__ __launch_bounds__(256) void rows_i32(Args a) {
    const int lane = threadIdx.x & 63, wv = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    if (wv >= a.waves) return;
    const int R = a.rows;
    const int2 *bd = a.bound + (size_t)wv * (R + 1 + 2 * kG);
    int2 *pub = a.pub + (size_t)wv * (R + 72);
    uint32_t qc[2];
    int32_t Hp[2], Dn[2];
    for (int k = 0; k < 2; ++k) {
        const int c = 2 * lane + k;
        qc[k] = (uint32_t)a.q[wv * W + c] << 8;
        Hp[k] = a.h0[wv * W + c];
        Dn[k] = a.d1[wv * W + c];
    }
    int32_t Bprev = bd[0].x;
    int2 nv = lane < kG ? bd[1 + lane] : make_int2(0, 0);
    for (int r0 = 1; r0 <= R; r0 += kG) {
        const int2 cur = nv;
        if (lane < kG) nv = bd[r0 + kG + lane];
        const uint32_t voff = lane == 63 ? 0u : (uint32_t)(R + 1 + lane - r0) * 8u;  // next group (pad rows past R)
        uint32_t w4 = 0;
#pragma unroll
        for (int q = 0; q < kG; ++q) {
            const int r = r0 + q;
            if ((q & 3) == 0) w4 = dword4(a.d, r);
            const uint32_t dch = ((w4 >> (8 * (q & 3))) & 0xFFu) << 8;
            const int32_t bH = __builtin_amdgcn_readlane(cur.x, q);
            const int32_t bI = __builtin_amdgcn_readlane(cur.y, q);
            const int32_t diag = (int32_t)dpp<0x138>((uint32_t)Bprev, (uint32_t)Hp[1]);  // wave_shr:1
            int32_t M[2], tO[2], Pf[2], Dv[2];
            for (int k = 0; k < 2; ++k) {
                const int32_t pen = (int32_t)min(qc[k] ^ dch, (uint32_t)P);
                M[k] = (k == 0 ? diag : Hp[0]) - pen;
                tO[k] = M[k] + O;
                Pf[k] = k == 0 ? tO[0] : max(Pf[0], tO[1]);
                Dv[k] = Dn[k];
                Dn[k] = max(tO[k], Dv[k]) + Ds;
            }
            int32_t S = Pf[1];
            S = max(S, (int32_t)dpp<0x111>(0x80000000u, (uint32_t)S));
            S = max(S, (int32_t)dpp<0x112>(0x80000000u, (uint32_t)S));
            S = max(S, (int32_t)dpp<0x114>(0x80000000u, (uint32_t)S));
            S = max(S, (int32_t)dpp<0x118>(0x80000000u, (uint32_t)S));
            S = max(S, (int32_t)dpp<0x142, 0xa>(0x80000000u, (uint32_t)S));
            S = max(S, (int32_t)dpp<0x143, 0xc>(0x80000000u, (uint32_t)S));
            const int32_t Ein = max((int32_t)dpp<0x138>(0x80000000u, (uint32_t)S), bI);
            const int32_t I0 = Ein, I1 = max(Ein, Pf[0]);
            Hp[0] = max(M[0], max(I0, Dv[0]));
            Hp[1] = max(M[1], max(I1, Dv[1]));
            // every lane stores (no exec change): lane 63 at row r, the others
            // at pad slots past the column
            *(int2 *)((char *)(pub + r0) + voff + 8 * q) = make_int2(Hp[1], max(S, bI));
            Bprev = bH;
        }
    }
    for (int k = 0; k < 2; ++k) a.last[wv * W + 2 * lane + k] = Hp[k];
}

// ------------------------------------------------- i16 x 2, per-row frames
__global__ __launch_bounds__(256) void rows_pk(Args a) {
    const int lane = threadIdx.x & 63, wv = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    if (wv >= a.waves) return;
    const int R = a.rows;
    const int2 *bd = a.bound + (size_t)wv * (R + 1 + 2 * kG);
    int2 *pub = a.pub + (size_t)wv * (R + 72);
    const uint32_t kNeg = 0x80008000u;
    const bool l0 = lane == 0;
    const uint32_t qc = ((uint32_t)a.q[wv * W + lane] << 8) | ((uint32_t)a.q[wv * W + 64 + lane] << 24);
    int32_t Bprev = bd[0].x;
    // row-0 state relative to B(0)
    uint32_t Hp = pk(a.h0[wv * W + lane] - Bprev, a.h0[wv * W + 64 + lane] - Bprev);
    uint32_t Dn = pk(a.d1[wv * W + lane] - Bprev, a.d1[wv * W + 64 + lane] - Bprev);
    int2 nv = lane < kG ? bd[1 + lane] : make_int2(0, 0);
    for (int r0 = 1; r0 <= R; r0 += kG) {
        const int2 cur = nv;
        if (lane < kG) nv = bd[r0 + kG + lane];
        const uint32_t voff = lane == 63 ? 0u : (uint32_t)(R + 1 + lane - r0) * 8u;
        uint32_t w4 = 0;
#pragma unroll
        for (int q = 0; q < kG; ++q) {
            const int r = r0 + q;
            if ((q & 3) == 0) w4 = dword4(a.d, r);
            const uint32_t ch = (w4 >> (8 * (q & 3))) & 0xFFu;
            const uint32_t dch = (ch << 8) | (ch << 24);
            const int32_t bH = __builtin_amdgcn_readlane(cur.x, q);
            const int32_t bI = __builtin_amdgcn_readlane(cur.y, q);
            const int32_t dB = bH - Bprev;                      // frame step (scalar)
            const uint32_t dBp = pk(dB, dB), nBp = pk(-dB, -dB);
            // carried state into the frame of row r
            Hp = u(v2(Hp) - v2(dBp));
            const uint32_t Dv = u(v2(Dn) - v2(dBp));
            // diagonal: lane l-1's H (lane 0: low = H~(r-1, c0) = -dB, high = lane 63's low)
            const uint32_t ror = dpp<0x13C>(0u, Hp);  // wave_ror:1
            const uint32_t diag = l0 ? __builtin_amdgcn_perm(ror, nBp, 0x05040100u) : ror;
            const uint32_t x = qc ^ dch;
            const uint32_t pen = u(__builtin_bit_cast(s16x2, __builtin_elementwise_min(
                __builtin_bit_cast(unsigned short __attribute__((ext_vector_type(2))), x),
                __builtin_bit_cast(unsigned short __attribute__((ext_vector_type(2))), pk(P, P)))));
            const uint32_t M = u(v2(diag) - v2(pen));
            const uint32_t tO = u(v2(M) + v2(pk(O, O)));
            Dn = u(pmax(v2(tO), v2(Dv)) + v2(pk(Ds, Ds)));
            // inclusive prefix max of tO over lanes, both halves at once
            uint32_t S = tO;
            S = u(pmax(v2(S), v2(dpp<0x111>(kNeg, S))));
            S = u(pmax(v2(S), v2(dpp<0x112>(kNeg, S))));
            S = u(pmax(v2(S), v2(dpp<0x114>(kNeg, S))));
            S = u(pmax(v2(S), v2(dpp<0x118>(kNeg, S))));
            S = u(pmax(v2(S), v2(dpp<0x142, 0xa>(kNeg, S))));
            S = u(pmax(v2(S), v2(dpp<0x143, 0xc>(kNeg, S))));
            // exclusive: lane l-1's (lane 0: none); the high halves also see
            // the low halves' total (lane 63's low prefix) and both the
            // boundary's I~ (scalar side)
            const uint32_t ex = dpp<0x138>(kNeg, S);  // wave_shr:1
            const int32_t tot = (int16_t)(__builtin_amdgcn_readlane(S, 63) & 0xFFFFu);
            const int32_t bIr = bI - bH;
            const uint32_t I = u(pmax(v2(ex), v2(pk(bIr, max(bIr, tot)))));
            Hp = u(pmax(pmax(v2(M), v2(I)), v2(Dv)));
            {
                const int32_t h = (int32_t)Hp >> 16, s = max((int32_t)S >> 16, tot);
                *(int2 *)((char *)(pub + r0) + voff + 8 * q) = make_int2(h + bH, max(s + bH, bI));
            }
            Bprev = bH;
        }
    }
    a.last[wv * W + lane] = (int32_t)(int16_t)(Hp & 0xFFFFu) + Bprev;
    a.last[wv * W + 64 + lane] = ((int32_t)Hp >> 16) + Bprev;
}

// The same with values biased by 0x8000 (u16 order = i16 order, 0 = -inf):
// DPP moves zero-fill their out-of-row lanes (bound_ctrl), so no `old`
// operand has to be materialised per move, and u16 max ops compare.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 w2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t uw(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ uint32_t umax2(uint32_t a, uint32_t b) {
    return uw(__builtin_elementwise_max(w2(a), w2(b)));
}
template <int kCtrl>
__device__ __forceinline__ uint32_t dppz(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, 0xf, 0xf, true);
}
__global__ __launch_bounds__(256) void rows_pkz(Args a) {
    const int lane = threadIdx.x & 63, wv = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    if (wv >= a.waves) return;
    const int R = a.rows;
    const int2 *bd = a.bound + (size_t)wv * (R + 1 + 2 * kG);
    int2 *pub = a.pub + (size_t)wv * (R + 72);
    const uint32_t kB = 0x80008000u;  // bias of both halves
    const bool l0 = lane == 0;
    const uint32_t qc = ((uint32_t)a.q[wv * W + lane] << 8) | ((uint32_t)a.q[wv * W + 64 + lane] << 24);
    int32_t Bprev = bd[0].x;
    uint32_t Hp = pk(a.h0[wv * W + lane] - Bprev, a.h0[wv * W + 64 + lane] - Bprev) ^ kB;
    uint32_t Dn = pk(a.d1[wv * W + lane] - Bprev, a.d1[wv * W + 64 + lane] - Bprev) ^ kB;
    int2 nv = lane < kG ? bd[1 + lane] : make_int2(0, 0);
    for (int r0 = 1; r0 <= R; r0 += kG) {
        const int2 cur = nv;
        if (lane < kG) nv = bd[r0 + kG + lane];
        const uint32_t voff = lane == 63 ? 0u : (uint32_t)(R + 1 + lane - r0) * 8u;
        uint32_t w4 = 0;
#pragma unroll
        for (int q = 0; q < kG; ++q) {
            if ((q & 3) == 0) w4 = dword4(a.d, r0 + q);
            const uint32_t ch = (w4 >> (8 * (q & 3))) & 0xFFu;
            const uint32_t dch = (ch << 8) | (ch << 24);
            const int32_t bH = __builtin_amdgcn_readlane(cur.x, q);
            const int32_t bI = __builtin_amdgcn_readlane(cur.y, q);
            const int32_t dB = bH - Bprev;
            const uint32_t dBp = pk(dB, dB), nBp = pk(-dB, -dB) ^ kB;
            Hp = uw(w2(Hp) - w2(dBp));
            const uint32_t Dv = uw(w2(Dn) - w2(dBp));
            const uint32_t ror = dpp<0x13C>(0u, Hp);  // wave_ror:1
            const uint32_t diag = l0 ? __builtin_amdgcn_perm(ror, nBp, 0x05040100u) : ror;
            const uint32_t x = qc ^ dch;
            const uint32_t pen = uw(__builtin_elementwise_min(w2(x), w2(pk(P, P))));
            const uint32_t M = uw(w2(diag) - w2(pen));
            const uint32_t tO = uw(w2(M) + w2(pk(O, O)));
            Dn = uw(w2(umax2(tO, Dv)) + w2(pk(Ds, Ds)));
            uint32_t S = tO;
            S = umax2(S, dppz<0x111>(S));
            S = umax2(S, dppz<0x112>(S));
            S = umax2(S, dppz<0x114>(S));
            S = umax2(S, dppz<0x118>(S));
            S = umax2(S, dppz<0x142>(S));  // row_bcast:15 (row 0: zero-filled)
            S = umax2(S, dppz<0x143>(S));  // row_bcast:31 (rows 0, 1: zero-filled)
            const uint32_t ex = dppz<0x138>(S);  // wave_shr:1, lane 0 zero (-inf)
            const uint32_t tot = __builtin_amdgcn_readlane(S, 63) & 0xFFFFu;  // biased
            const uint32_t bIr = (uint32_t)(bI - bH + 0x8000) & 0xFFFFu;
            const uint32_t I = umax2(ex, bIr | (max(bIr, tot) << 16));
            Hp = umax2(umax2(M, I), Dv);
            {
                const int32_t h = (int32_t)(Hp >> 16) - 0x8000;
                const int32_t sv = (int32_t)max(S >> 16, tot) - 0x8000;
                *(int2 *)((char *)(pub + r0) + voff + 8 * q) = make_int2(h + bH, max(sv + bH, bI));
            }
            Bprev = bH;
        }
    }
    a.last[wv * W + lane] = (int32_t)(Hp & 0xFFFFu) - 0x8000 + Bprev;
    a.last[wv * W + 64 + lane] = (int32_t)(Hp >> 16) - 0x8000 + Bprev;
}

// ---------------------------------------------------------------------- host
static void host_ref(const uint8_t *q, const uint8_t *d, const int2 *bd, const int32_t *h0,
                     const int32_t *d1, int R, std::vector<int32_t> *last, std::vector<int2> *pub,
                     int32_t *maxrel) {
    std::vector<int32_t> H(h0, h0 + W), D(d1, d1 + W), Hn(W);
    for (int r = 1; r <= R; ++r) {
        const int32_t bH = bd[r].x, bI = bd[r].y, Bp = bd[r - 1].x;
        int32_t I = bI;
        for (int c = 0; c < W; ++c) {
            const int32_t pen = q[c] == d[r - 1] ? 0 : P;
            const int32_t M = (c ? H[c - 1] : Bp) - pen;
            const int32_t h = std::max(M, std::max(I, D[c]));
            D[c] = std::max(M + O, D[c]) + Ds;
            I = std::max(I, M + O);
            Hn[c] = h;
            *maxrel = std::max(*maxrel, std::abs(h - bH));
            *maxrel = std::max(*maxrel, std::abs(D[c] - bH));
        }
        H = Hn;
        (*pub)[r] = make_int2(H[W - 1], I);
    }
    *last = H;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char **argv) {
    const int waves = argc > 1 ? atoi(argv[1]) : 782;
    const int R = argc > 2 ? atoi(argv[2]) : 100000;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    const int wpb = argc > 4 ? atoi(argv[4]) : 1;  // waves per workgroup (1..4)
    if (waves < 1 || R < 8 || R % 8 || wpb < 1 || wpb > 4) { fprintf(stderr, "waves >= 1, rows >= 8, rows %% 8 == 0\n"); return 2; }
    srand(7);
    const char al[4] = {'A', 'C', 'G', 'T'};
    std::vector<uint8_t> q((size_t)waves * W), d(R);
    for (auto &c : q) c = al[rand() & 3];
    for (auto &c : d) c = al[rand() & 3];
    // boundary: H~(r, 0) a random walk drifting like a random pair's column,
    // I~(r, 1) an open below it; row 0 near zero
    const size_t bs = (size_t)R + 1 + 2 * kG;
    std::vector<int2> bd(waves * bs);
    std::vector<int32_t> h0((size_t)waves * W), d1((size_t)waves * W);
    for (int w = 0; w < waves; ++w) {
        int32_t b = 0;
        for (int r = 0; r < (int)bs; ++r) {
            if (r) b += (rand() % 41) - 24;
            bd[w * bs + r] = make_int2(b, b + O - (rand() % 16));
        }
        for (int c = 0; c < W; ++c) {
            h0[w * W + c] = -(rand() % 64) - 2 * c;
            d1[w * W + c] = h0[w * W + c] + O;
        }
    }
    uint8_t *dq, *dd;
    int2 *dbd, *dpub;
    int32_t *dh0, *dd1, *dlast;
    CK(hipMalloc(&dq, q.size()));
    CK(hipMalloc(&dd, d.size() + 16));
    CK(hipMalloc(&dbd, bd.size() * sizeof(int2)));
    CK(hipMalloc(&dh0, h0.size() * 4));
    CK(hipMalloc(&dd1, d1.size() * 4));
    CK(hipMalloc(&dpub, (size_t)waves * (R + 72) * sizeof(int2)));
    CK(hipMalloc(&dlast, (size_t)waves * W * 4));
    CK(hipMemcpy(dq, q.data(), q.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dd, d.data(), d.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dbd, bd.data(), bd.size() * sizeof(int2), hipMemcpyHostToDevice));
    CK(hipMemcpy(dh0, h0.data(), h0.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dd1, d1.data(), d1.size() * 4, hipMemcpyHostToDevice));
    Args a{dq, dd, dbd, dh0, dd1, dpub, dlast, R, waves};
    // host check of waves 0 and waves-1
    const int chk[2] = {0, waves - 1};
    std::vector<std::vector<int32_t>> want_last(2);
    std::vector<std::vector<int2>> want_pub(2, std::vector<int2>(R + 1));
    int32_t maxrel = 0;
    for (int i = 0; i < 2; ++i)
        host_ref(&q[chk[i] * W], d.data(), &bd[chk[i] * bs], &h0[chk[i] * W], &d1[chk[i] * W], R,
                 &want_last[i], &want_pub[i], &maxrel);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("{\"waves\": %d, \"waves_per_block\": %d, \"rows\": %d, \"max_rel\": %d", waves, wpb, R, maxrel);
    for (int v = 0; v < 3; ++v) {
        const char *name = v == 2 ? "pkz" : v ? "pk" : "i32";
        float best = 1e30f;
        for (int it = 0; it < reps + 1; ++it) {
            CK(hipMemset(dlast, 0, (size_t)waves * W * 4));
            CK(hipEventRecord(e0));
            const int nb = (waves + wpb - 1) / wpb;
            if (v == 2) rows_pkz<<<nb, 64 * wpb>>>(a);
            else if (v) rows_pk<<<nb, 64 * wpb>>>(a);
            else rows_i32<<<nb, 64 * wpb>>>(a);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (it) best = std::min(best, ms);
        }
        int bad = 0;
        std::vector<int32_t> got(W);
        std::vector<int2> gp(R + 1);
        for (int i = 0; i < 2; ++i) {
            CK(hipMemcpy(got.data(), dlast + (size_t)chk[i] * W, W * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(gp.data(), dpub + (size_t)chk[i] * (R + 72), (R + 1) * sizeof(int2),
                         hipMemcpyDeviceToHost));
            for (int c = 0; c < W; ++c) bad += got[c] != want_last[i][c];
            for (int r = 1; r <= R; ++r)
                bad += gp[r].x != want_pub[i][r].x || gp[r].y != want_pub[i][r].y;
        }
        printf(", \"%s\": {\"ms\": %.4f, \"us_per_row\": %.5f, \"mismatches\": %d}", name, best,
               best * 1e3 / R, bad);
    }
    printf("}\n");
    return 0;
}

// Row-fill chains per wave: does a lone wave's score-only
// row step (the shipped nw_fill_rows_kernel<K, kCodesNone> recurrence, i32
// lanes of K columns, DPP prefix max over the 64 lanes) get cheaper per
// stripe-row when the wave carries NC independent stripes and interleaves
// their rows, so that one chain's DPP hazard slots and latencies hold the
// other's instructions?  Each chain fills its own 64K-column stripe from a
// boundary column in memory (8-row groups, as the hand-off loads them) and
// publishes (H~, I~) leaving its last column per row; no neighbour to wait
// for, so the time is rows x step.  C4 needs 782 K = 2 stripes (one per
// SIMD): NC = 2 with K = 1 would hold 1,563 K = 1 stripes in 782 waves.
// Transformed recurrence as row_pk_floor.hip / nw_kernels.hip:
//   M~ = H~(r-1, c-1) - pen,  I~(r, c+1) = max(I~(r, c), M~ + O),
//   D~(r+1, c) = max(M~ + O, D~) + Ds,  H~ = max(M~, I~, D~).
// Checked against a host i32 computation on the first and last stripe.
// Build: hipcc -O3 --offload-arch=gfx950 row_chains.hip -o row_chains
// Run:   ./row_chains [stripes] [rows] [reps]  (prints one JSON line per (K, NC))
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kG = 8;                         // boundary rows per group
constexpr int32_t P = 36, O = -32, Ds = -68;  // pen (mismatch), open, D step (x4 scale)

template <int kCtrl, int kRow = 0xf, int kBank = 0xf>
__device__ __forceinline__ uint32_t dpp(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, kCtrl, kRow, kBank, false);
}

struct Args {
    const uint8_t *q;   // [stripes][W]
    const uint8_t *d;   // [rows] (all stripes)
    const int2 *bound;  // [stripes][rows + 1 + 2 kG]: (H~(r, 0), I~(r, 1))
    const int32_t *h0;  // [stripes][W]: H~(0, c)
    const int32_t *d1;  // [stripes][W]: D~(1, c)
    int2 *pub;          // [stripes][rows + 72]
    int32_t *last;      // [stripes][W]
    int rows;
    int stripes;
};

__device__ __forceinline__ uint32_t dword4(const uint8_t *d, int r) {
    typedef const __attribute__((address_space(4))) uint32_t cu32;
    return ((cu32 *)d)[(r - 1) >> 2];
}

template <int K, int NC>
__global__ __launch_bounds__(256) void rows_x(Args a) {
    constexpr int W = 64 * K;
    const int lane = threadIdx.x & 63, wv = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const int s0 = wv * NC;
    if (s0 >= a.stripes) return;
    const int R = a.rows;
    const int2 *bd[NC];
    int2 *pub[NC];
    uint32_t qc[NC][K];
    int32_t Hp[NC][K], Dn[NC][K], Bprev[NC];
    int2 nv[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int s = min(s0 + c, a.stripes - 1);
        bd[c] = a.bound + (size_t)s * (R + 1 + 2 * kG);
        pub[c] = a.pub + (size_t)s * (R + 72);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int col = K * lane + k;
            qc[c][k] = (uint32_t)a.q[s * W + col] << 8;
            Hp[c][k] = a.h0[s * W + col];
            Dn[c][k] = a.d1[s * W + col];
        }
        Bprev[c] = bd[c][0].x;
        nv[c] = lane < kG ? bd[c][1 + lane] : make_int2(0, 0);
    }
    for (int r0 = 1; r0 <= R; r0 += kG) {
        int2 cur[NC];
        uint32_t voff[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            cur[c] = nv[c];
            if (lane < kG) nv[c] = bd[c][r0 + kG + lane];
            voff[c] = lane == 63 ? 0u : (uint32_t)(R + 1 + lane - r0) * 8u;
        }
        uint32_t w4 = 0;
#pragma unroll
        for (int q = 0; q < kG; ++q) {
            const int r = r0 + q;
            if ((q & 3) == 0) w4 = dword4(a.d, r);
            const uint32_t dch = ((w4 >> (8 * (q & 3))) & 0xFFu) << 8;
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const int32_t bH = __builtin_amdgcn_readlane(cur[c].x, q);
                const int32_t bI = __builtin_amdgcn_readlane(cur[c].y, q);
                const int32_t diag = (int32_t)dpp<0x138>((uint32_t)Bprev[c], (uint32_t)Hp[c][K - 1]);
                int32_t M[K], tO[K], Pf[K], Dv[K];
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const int32_t pen = (int32_t)min(qc[c][k] ^ dch, (uint32_t)P);
                    M[k] = (k == 0 ? diag : Hp[c][k - 1]) - pen;
                    tO[k] = M[k] + O;
                    Pf[k] = k == 0 ? tO[0] : max(Pf[k - 1], tO[k]);
                    Dv[k] = Dn[c][k];
                    Dn[c][k] = max(tO[k], Dv[k]) + Ds;
                }
                int32_t S = Pf[K - 1];
                S = max(S, (int32_t)dpp<0x111>(0x80000000u, (uint32_t)S));
                S = max(S, (int32_t)dpp<0x112>(0x80000000u, (uint32_t)S));
                S = max(S, (int32_t)dpp<0x114>(0x80000000u, (uint32_t)S));
                S = max(S, (int32_t)dpp<0x118>(0x80000000u, (uint32_t)S));
                S = max(S, (int32_t)dpp<0x142, 0xa>(0x80000000u, (uint32_t)S));
                S = max(S, (int32_t)dpp<0x143, 0xc>(0x80000000u, (uint32_t)S));
                const int32_t Ein = max((int32_t)dpp<0x138>(0x80000000u, (uint32_t)S), bI);
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const int32_t Ik = k == 0 ? Ein : max(Ein, Pf[k - 1]);
                    Hp[c][k] = max(M[k], max(Ik, Dv[k]));
                }
                *(int2 *)((char *)(pub[c] + r0) + voff[c] + 8 * q) = make_int2(Hp[c][K - 1], max(S, bI));
                Bprev[c] = bH;
            }
        }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        if (s0 + c >= a.stripes) break;
#pragma unroll
        for (int k = 0; k < K; ++k) a.last[(size_t)(s0 + c) * W + K * lane + k] = Hp[c][k];
    }
}

static void host_ref(int W, const uint8_t *q, const uint8_t *d, const int2 *bd, const int32_t *h0,
                     const int32_t *d1, int R, std::vector<int32_t> *last, std::vector<int2> *pub) {
    std::vector<int32_t> H(h0, h0 + W), D(d1, d1 + W), Hn(W);
    for (int r = 1; r <= R; ++r) {
        const int32_t bI = bd[r].y, Bp = bd[r - 1].x;
        int32_t I = bI;
        for (int c = 0; c < W; ++c) {
            const int32_t pen = q[c] == d[r - 1] ? 0 : P;
            const int32_t M = (c ? H[c - 1] : Bp) - pen;
            Hn[c] = std::max(M, std::max(I, D[c]));
            D[c] = std::max(M + O, D[c]) + Ds;
            I = std::max(I, M + O);
        }
        H = Hn;
        (*pub)[r] = make_int2(H[W - 1], I);
    }
    *last = H;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <int K, int NC>
static int run(int stripes, int R, int reps) {
    constexpr int W = 64 * K;
    srand(7);
    const char al[4] = {'A', 'C', 'G', 'T'};
    std::vector<uint8_t> q((size_t)stripes * W), d(R);
    for (auto &c : q) c = al[rand() & 3];
    for (auto &c : d) c = al[rand() & 3];
    const size_t bs = (size_t)R + 1 + 2 * kG;
    std::vector<int2> bd(stripes * bs);
    std::vector<int32_t> h0((size_t)stripes * W), d1((size_t)stripes * W);
    for (int w = 0; w < stripes; ++w) {
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
    CK(hipMalloc(&dpub, (size_t)stripes * (R + 72) * sizeof(int2)));
    CK(hipMalloc(&dlast, (size_t)stripes * W * 4));
    CK(hipMemcpy(dq, q.data(), q.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dd, d.data(), d.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dbd, bd.data(), bd.size() * sizeof(int2), hipMemcpyHostToDevice));
    CK(hipMemcpy(dh0, h0.data(), h0.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dd1, d1.data(), d1.size() * 4, hipMemcpyHostToDevice));
    Args a{dq, dd, dbd, dh0, dd1, dpub, dlast, R, stripes};
    const int chk[2] = {0, stripes - 1};
    std::vector<std::vector<int32_t>> want_last(2);
    std::vector<std::vector<int2>> want_pub(2, std::vector<int2>(R + 1));
    for (int i = 0; i < 2; ++i)
        host_ref(W, &q[chk[i] * W], d.data(), &bd[chk[i] * bs], &h0[chk[i] * W], &d1[chk[i] * W], R,
                 &want_last[i], &want_pub[i]);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int waves = (stripes + NC - 1) / NC;
    float best = 1e30f;
    for (int it = 0; it < reps + 1; ++it) {
        CK(hipMemset(dlast, 0, (size_t)stripes * W * 4));
        CK(hipEventRecord(e0));
        rows_x<K, NC><<<waves, 64>>>(a);  // one wave per workgroup: dealt one per SIMD
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
        for (int r = 1; r <= R; ++r) bad += gp[r].x != want_pub[i][r].x || gp[r].y != want_pub[i][r].y;
    }
    // columns covered per wave-row, and the time per stripe-row
    printf("{\"K\": %d, \"chains\": %d, \"stripes\": %d, \"waves\": %d, \"rows\": %d, \"ms\": %.4f, "
           "\"us_per_row\": %.5f, \"cycles_per_row_2p4ghz\": %.1f, \"mismatches\": %d}\n",
           K, NC, stripes, waves, R, best, best * 1e3 / R, best * 1e3 / R * 2400.0, bad);
    fflush(stdout);
    hipFree(dq); hipFree(dd); hipFree(dbd); hipFree(dh0); hipFree(dd1); hipFree(dpub); hipFree(dlast);
    return bad ? 3 : 0;
}

int main(int argc, char **argv) {
    const int cols = argc > 1 ? atoi(argv[1]) : 100096;  // C4: 782 x 128 columns
    const int R = argc > 2 ? atoi(argv[2]) : 100000;
    const int reps = argc > 3 ? atoi(argv[3]) : 3;
    if (R < 8 || R % 8) { fprintf(stderr, "rows >= 8, rows %% 8 == 0\n"); return 2; }
    int rc = 0;
    rc |= run<2, 1>(cols / 128, R, reps);  // the shipped geometry: 782 lone waves
    rc |= run<1, 1>(cols / 64, R, reps);   // K = 1: 1,564 waves (two per SIMD on 64 % of them)
    rc |= run<1, 2>(cols / 64, R, reps);   // K = 1, two chains per wave: 782 waves
    rc |= run<2, 2>(cols / 128, R, reps);  // K = 2, two chains: 391 waves
    rc |= run<1, 1>(cols / 128, R, reps);  // a K = 1 chain alone, 782 waves (its step, no SIMD shared)
    return rc;
}

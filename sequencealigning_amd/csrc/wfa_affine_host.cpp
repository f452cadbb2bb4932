// C ABI of the corrected gap-affine WFA engine (include/saln.h,
// saln_wfa_affine_*): SURVEY.md §8(f) row 4.  Not a reference-parity path —
// the reference's wfa_align (src/wfa.rs:23-42, engine wfa_host.cpp) has no
// defined output for realistic inputs; this engine returns the minimum
// gap-affine penalty with the reference's penalties (wfa.rs:14-21) by
// default, checked against the Gotoh DP (oracle/refaffine.c).
//
// Two passes: every pair first runs with a W-diagonal wavefront ring; pairs
// whose wavefront outgrows it (score -2) are compacted on the device and run
// again with a 2x wider ring.  Score -1: the penalty exceeds max_score.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <numeric>
#include <string>
#include <vector>

#include "nw_host.hpp"
#include "saln.h"
#include "wfa_affine.hpp"
#include "saln_options.hpp"

using namespace saln;

struct saln_wfa_affine_plan {
    saln_context *ctx = nullptr;
    WfaAffParams prm{};
    bool wide = false;  // i32 offsets (a sequence longer than 32,000 bases)
    uint64_t n = 0;
    WfaAffPair *d_pairs = nullptr, *d_rerun = nullptr;
    uint32_t *d_count = nullptr;  // [rerun pairs, pass-1 next pair, pass-2 next pair]
    WfaAffParams p1{}, p2{};  // the two passes (ring width, LDS sequence staging)
    uint32_t grid1 = 0, grid2 = 0;
};

namespace {

// ring widths (diagonals) of the two passes, i16 / i32 offsets: the second
// pass's ring is the 64 KB LDS limit of a workgroup; a wavefront wider than it
// (|k| > W/2 diagonals: penalties above ~e * W / 2) leaves score -2
constexpr int32_t kW1 = 1024, kW2 = 2048, kW1Wide = 512, kW2Wide = 1024;

#define TRY(expr)                                                                          \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) {                                                            \
            set_error(std::string(#expr) + ": " + hipGetErrorString(e_));                  \
            return SALN_E_HIP;                                                             \
        }                                                                                  \
    } while (0)

int make_params(const saln_wfa_penalties *pen, int32_t max_score, WfaAffParams *out) {
    const int32_t x = pen ? pen->mismatch : 4, o = pen ? pen->gap_open : 2,
                  e = pen ? pen->gap_extend : 6;
    if (x <= 0 || e <= 0 || o < 0 || x > 4096 || o > 4096 || e > 4096) return SALN_E_INVALID;
    const int32_t g = std::gcd(std::gcd(x, o + e), e);
    WfaAffParams p{};
    p.x = x, p.o = o, p.e = e, p.g = g;
    p.RM = std::max(x, o + e) / g + 1;
    p.RI = e / g + 1;
    if (p.RM > 16 || p.RI > 16) {
        set_error("wfa_affine: penalties need more than 16 wavefront ring slots");
        return SALN_E_INVALID;
    }
    p.max_score = max_score > 0 ? max_score : INT32_MAX / 2;
    *out = p;
    return SALN_OK;
}

uint32_t grid_for(const WfaAffParams &prm, bool wide, uint64_t n, int device) {
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    const size_t lds = wfa_affine_lds_bytes(prm, wide);
    const uint64_t per_cu = std::max<uint64_t>(1, std::min<uint64_t>(16, (160u << 10) / lds));
    (void)wide;
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(n, per_cu * (uint64_t)cus));
}

int build_pairs(const uint64_t *q_off, uint64_t n_q, const uint64_t *db_off, uint64_t n_db,
                const uint32_t *pair_q, const uint32_t *pair_db, uint64_t n_pairs,
                std::vector<WfaAffPair> *out, bool *wide, uint64_t *seq_need,
                uint64_t *code_need) {
    out->resize(n_pairs);
    uint64_t maxlen = 0;
    for (uint64_t k = 0; k < n_pairs; ++k) {
        const uint64_t qi = pair_q ? pair_q[k] : k % n_q, di = pair_db ? pair_db[k] : k / n_q;
        if (qi >= n_q || di >= n_db) return SALN_E_INVALID;
        WfaAffPair p{};
        p.q_off = q_off[qi];
        p.d_off = db_off[di];
        const uint64_t lq = q_off[qi + 1] - q_off[qi], ld = db_off[di + 1] - db_off[di];
        if (lq > 0x3FFFFFFFull || ld > 0x3FFFFFFFull) return SALN_E_INVALID;
        p.lq = (uint32_t)lq;
        p.ld = (uint32_t)ld;
        p.out = (uint32_t)k;
        maxlen = std::max({maxlen, lq, ld});
        // LDS bytes to stage both sequences (wfa_affine_kernel's layout)
        *seq_need = std::max<uint64_t>(*seq_need, ((lq + 47) & ~15ull) + ld + 48);
        // ... or as 2-bit codes (16 per word, the 16-byte-aligned base's
        // words plus two pad words per sequence)
        // (at any alignment of the caller's buffers)
        *code_need = std::max<uint64_t>(*code_need, 4 * ((15 + lq + 15) / 16 + 2 + (15 + ld + 15) / 16 + 2));
        (*out)[k] = p;
    }
    *wide = maxlen > 32000;
    return SALN_OK;
}

}  // namespace

extern "C" {

int saln_wfa_affine_plan_create(saln_context *ctx, const uint64_t *q_off, uint64_t n_q,
                                const uint64_t *db_off, uint64_t n_db, const uint32_t *pair_q,
                                const uint32_t *pair_db, uint64_t n_pairs,
                                const saln_wfa_penalties *pen, int32_t max_score,
                                saln_wfa_affine_plan **out) {
    if (!ctx || !q_off || !db_off || !out || n_pairs > 0xFFFFFFFFull) return SALN_E_INVALID;
    if (!pair_q != !pair_db) return SALN_E_INVALID;
    if (!pair_q && n_pairs != n_q * n_db) return SALN_E_INVALID;
    auto *p = new saln_wfa_affine_plan();
    p->ctx = ctx;
    int rc = make_params(pen, max_score, &p->prm);
    std::vector<WfaAffPair> hp;
    uint64_t seq_need = 0, code_need = 0;
    if (rc == SALN_OK)
        rc = build_pairs(q_off, n_q, db_off, n_db, pair_q, pair_db, n_pairs, &hp, &p->wide,
                         &seq_need, &code_need);
    if (rc != SALN_OK) {
        delete p;
        return rc;
    }
    p->n = n_pairs;
    auto fail = [&](hipError_t e) {
        set_error(std::string("wfa_affine plan: ") + hipGetErrorString(e));
        saln_wfa_affine_plan_destroy(p);
        return SALN_E_HIP;
    };
    hipError_t e;
    if ((e = hipSetDevice(ctx->device)) != hipSuccess) return fail(e);
    if (n_pairs) {
        if ((e = hipMalloc(&p->d_pairs, n_pairs * sizeof(WfaAffPair))) != hipSuccess) return fail(e);
        if ((e = hipMalloc(&p->d_rerun, n_pairs * sizeof(WfaAffPair))) != hipSuccess) return fail(e);
        if ((e = hipMalloc(&p->d_count, 3 * sizeof(uint32_t))) != hipSuccess) return fail(e);
        if ((e = hipMemcpy(p->d_pairs, hp.data(), n_pairs * sizeof(WfaAffPair),
                           hipMemcpyHostToDevice)) != hipSuccess)
            return fail(e);
    }
    // Each pass stages the pair's sequences in LDS when they fit next to its
    // rings within kSeqLds / the 64 KB workgroup limit (else reads HBM).
    // tuning options (saln_option_set): staged-sequence LDS, ring widths (0 auto)
    const Options opts = ctx->opts.effective();
    const uint64_t seq_lds = (uint64_t)opts[Opt::Wfa2SeqLds];
    const int32_t w1 = (int32_t)opts[Opt::Wfa2W1];
    const int32_t w2 = (int32_t)opts[Opt::Wfa2W2];
    auto pass = [&](int32_t W) {
        WfaAffParams q = p->prm;
        q.W = W;
        q.seqcap = 0;
        const size_t rings = wfa_affine_lds_bytes(q, p->wide);
        const uint64_t cap = std::min<uint64_t>(seq_lds, (64u << 10) - rings);
        // 2-bit codes when they fit (a pair holding other bytes then reads
        // HBM), bytes too when they take little more: the kernel tries codes
        // first, then bytes, within seqcap
        uint64_t want = code_need <= cap ? code_need : 0;
        if (seq_need <= cap && seq_need <= std::max<uint64_t>(want, 8u << 10)) want = std::max(want, seq_need);
        q.seqcap = (int32_t)((want + 15) & ~15ull);
        return q;
    };
    p->p1 = pass(w1 ? w1 : p->wide ? kW1Wide : kW1);
    p->p2 = pass(w2 ? w2 : p->wide ? kW2Wide : kW2);
    p->grid1 = grid_for(p->p1, p->wide, n_pairs, ctx->device);
    p->grid2 = grid_for(p->p2, p->wide, n_pairs, ctx->device);
    *out = p;
    return SALN_OK;
}

int saln_wfa_affine_execute(saln_wfa_affine_plan *p, const uint8_t *d_q_seq,
                            const uint8_t *d_db_seq, int32_t *d_scores, void *stream) {
    if (!p || !d_scores || !d_q_seq || !d_db_seq) return SALN_E_INVALID;
    if (!p->n) return SALN_OK;
    hipStream_t s = resolve_stream(stream, p->ctx);
    TRY(hipSetDevice(p->ctx->device));
    TRY(hipMemsetAsync(p->d_count, 0, 3 * sizeof(uint32_t), s));
    TRY(launch_wfa_affine(p->d_pairs, (uint32_t)p->n, d_q_seq, d_db_seq, p->p1, p->wide, p->grid1,
                          nullptr, p->d_count + 1, d_scores, s));
    TRY(launch_wfa_affine_compact(p->d_pairs, (uint32_t)p->n, d_scores, p->d_rerun, p->d_count, s));
    // pass 2 reads its pair count from the device (no host round trip)
    TRY(launch_wfa_affine(p->d_rerun, (uint32_t)p->n, d_q_seq, d_db_seq, p->p2, p->wide, p->grid2,
                          p->d_count, p->d_count + 2, d_scores, s));
    return SALN_OK;
}

int saln_wfa_affine_plan_destroy(saln_wfa_affine_plan *p) {
    if (!p) return SALN_OK;
    if (p->d_pairs) (void)hipFree(p->d_pairs);
    if (p->d_rerun) (void)hipFree(p->d_rerun);
    if (p->d_count) (void)hipFree(p->d_count);
    delete p;
    return SALN_OK;
}

int saln_wfa_affine_batch(saln_context *ctx, const uint8_t *q_seq, const uint64_t *q_off,
                          uint64_t n_q, const uint8_t *db_seq, const uint64_t *db_off,
                          uint64_t n_db, const uint32_t *pair_q, const uint32_t *pair_db,
                          uint64_t n_pairs, const saln_wfa_penalties *pen, int32_t max_score,
                          int32_t *scores) {
    if (!ctx || !q_off || !db_off || !scores) return SALN_E_INVALID;
    if (n_pairs == 0) return SALN_OK;
    saln_wfa_affine_plan *plan = nullptr;
    int rc = saln_wfa_affine_plan_create(ctx, q_off, n_q, db_off, n_db, pair_q, pair_db, n_pairs,
                                         pen, max_score, &plan);
    if (rc != SALN_OK) return rc;
    struct Guard {
        saln_wfa_affine_plan *p;
        std::vector<void *> bufs;
        ~Guard() {
            for (void *b : bufs) (void)hipFree(b);
            saln_wfa_affine_plan_destroy(p);
        }
    } g{plan, {}};
    const uint64_t qb = q_off[n_q], db = db_off[n_db];
    void *dq = nullptr, *dd = nullptr, *dsc = nullptr;
    TRY(hipMalloc(&dq, qb + 16));
    g.bufs.push_back(dq);
    TRY(hipMalloc(&dd, db + 16));
    g.bufs.push_back(dd);
    TRY(hipMalloc(&dsc, n_pairs * sizeof(int32_t)));
    g.bufs.push_back(dsc);
    if (qb) TRY(hipMemcpy(dq, q_seq, qb, hipMemcpyHostToDevice));
    if (db) TRY(hipMemcpy(dd, db_seq, db, hipMemcpyHostToDevice));
    rc = saln_wfa_affine_execute(plan, (const uint8_t *)dq, (const uint8_t *)dd, (int32_t *)dsc,
                                 nullptr);
    if (rc != SALN_OK) return rc;
    TRY(hipStreamSynchronize(ctx->stream));
    TRY(hipMemcpy(scores, dsc, n_pairs * sizeof(int32_t), hipMemcpyDeviceToHost));
    return SALN_OK;
}

}  // extern "C"

// Score-only all-vs-all (include/saln.h saln_nw_avsa_*).
//
// The reference's pair loop (src/main.rs:61-67) over every (db, query) pair,
// keeping score + panic status.  At C5 scale (10^4 x 10^5 = 10^9 pairs) a
// per-pair descriptor table would be 80 GB of host planning, so short
// queries are grouped by fill variant into classes and each class runs as
// one index space (class query, non-empty db record) that the packed fill
// decodes itself (AvsaSrc, nw_kernels.hip).  Queries outside the packed-i16
// region go through an ordinary score-only plan; pairs with an empty side are
// written from the boundary formulas.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <memory>
#include <numeric>
#include <vector>

#include "nw_host.hpp"

using namespace saln;

struct saln_nw_avsa {
    struct Class {
        int variant = 0;
        uint32_t nq = 0;
        uint32_t *d_qids = nullptr;
    };
    saln_context *ctx = nullptr;
    Options opts{};  // the context's effective options at creation
    Scoring sc{};
    uint64_t n_q = 0, n_db = 0, cells = 0;
    uint64_t *d_qoff = nullptr, *d_doff = nullptr;
    std::vector<Class> classes;
    uint32_t ld_max = 0;
    uint32_t *d_dids = nullptr;  // non-empty db records, longest first
    uint32_t n_dn = 0;
    uint32_t *d_zero_q = nullptr, *d_zero_d = nullptr;
    uint32_t n_zq = 0, n_zd = 0;
    saln_nw_plan *fb = nullptr;  // fallback queries x non-empty db
    uint32_t *d_fb_qids = nullptr;
    uint32_t n_fb = 0;
    saln_nw_result *d_fb_res = nullptr;
    uint64_t q_bytes = 0, d_bytes = 0;  // sequence bytes (the ACGT check)
    uint32_t *d_generic = nullptr;      // 1: a byte outside A, C, G, T (no profiles)

    ~saln_nw_avsa() {
        if (fb) saln_nw_plan_destroy(fb);
        for (auto &c : classes) (void)hipFree(c.d_qids);
        for (void *ptr : {(void *)d_qoff, (void *)d_doff, (void *)d_dids, (void *)d_zero_q,
                          (void *)d_zero_d, (void *)d_fb_qids, (void *)d_fb_res,
                          (void *)d_generic})
            if (ptr) (void)hipFree(ptr);
    }
};

template <typename T>
static hipError_t upload(T **dst, const std::vector<T> &v) {
    *dst = nullptr;
    if (v.empty()) return hipSuccess;
    hipError_t e = hipMalloc(dst, v.size() * sizeof(T));
    if (e != hipSuccess) return e;
    return hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
}

extern "C" {

int saln_nw_avsa_create(saln_context *ctx, const uint64_t *q_off, uint64_t n_q,
                        const uint64_t *db_off, uint64_t n_db, int32_t mode,
                        const saln_nw_scoring *scoring, saln_nw_avsa **out) {
    if (!ctx || !q_off || !db_off || !out) return SALN_E_INVALID;
    *out = nullptr;
    if (mode != SALN_MODE_GLOBAL) {
        set_error("not implemented");  // needleman_wunsch_affine.rs:433-434
        return SALN_NOT_IMPLEMENTED;
    }
    if (n_q > 0xFFFFFFFFull || n_db > 0xFFFFFFFFull) {
        set_error("too many records");
        return SALN_E_INVALID;
    }
    HIP_TRY(hipSetDevice(ctx->device));
    auto a = std::make_unique<saln_nw_avsa>();
    a->ctx = ctx;
    a->opts = ctx->opts.effective();
    a->sc = scoring_or_default(scoring);
    a->n_q = n_q;
    a->n_db = n_db;
    uint64_t sum_q = 0, sum_d = 0;
    std::vector<uint32_t> dn, zd, zq;
    for (uint64_t d = 0; d < n_db; ++d) {
        const uint64_t ld = db_off[d + 1] - db_off[d];
        if (ld > 0x7FFFFFFFull) {
            set_error("sequence too long");
            return SALN_E_INVALID;
        }
        sum_d += ld;
        (ld ? dn : zd).push_back((uint32_t)d);
        a->ld_max = std::max<uint32_t>(a->ld_max, (uint32_t)ld);
    }
    std::stable_sort(dn.begin(), dn.end(), [&](uint32_t x, uint32_t y) {
        return db_off[x + 1] - db_off[x] > db_off[y + 1] - db_off[y];
    });
    std::vector<std::vector<uint32_t>> cls(kNumVariants);
    std::vector<uint32_t> fbq;
    // 8 x 19 groups for queries of <= 152 columns: the per-step overhead over
    // 19 columns and 7 steps of skew instead of 10 and 15 (C5 slice 6,738 ->
    // 7,858 GCUPS); option nw.avsa_narrow = 0 keeps the 16 x 10 geometry
    const bool avsa_narrow = a->opts[Opt::AvsaNarrow] != 0;
    for (uint64_t q = 0; q < n_q; ++q) {
        const uint64_t lq = q_off[q + 1] - q_off[q];
        if (lq > 0x7FFFFFFFull) {
            set_error("sequence too long");
            return SALN_E_INVALID;
        }
        sum_q += lq;
        if (!lq) {
            zq.push_back((uint32_t)q);
            continue;
        }
        int v = choose_variant((uint32_t)lq, a->ld_max, a->sc);
        // score-only queries of <= 152 columns: 8-lane groups of 19 columns
        // (variant 4's geometry; no mask, so no walker segment limit)
        // (32 groups per block stage their db rows in LDS: 4 B per row while
        // the db stays inside one int16 frame, <= 80 KB per block)
        if (v == 7 && lq <= 152 && avsa_narrow && a->ld_max <= 600) v = 4;
        (variant_packed(v) ? cls[v] : fbq).push_back((uint32_t)q);
    }
    a->cells = sum_q * sum_d;
    a->q_bytes = q_off[n_q];
    a->d_bytes = db_off[n_db];
    HIP_TRY(hipMalloc(&a->d_generic, sizeof(uint32_t)));
    std::vector<uint64_t> qo(q_off, q_off + n_q + 1), dof(db_off, db_off + n_db + 1);
    HIP_TRY(upload(&a->d_qoff, qo));
    HIP_TRY(upload(&a->d_doff, dof));
    a->n_dn = (uint32_t)dn.size();
    HIP_TRY(upload(&a->d_dids, dn));
    a->n_zq = (uint32_t)zq.size();
    a->n_zd = (uint32_t)zd.size();
    HIP_TRY(upload(&a->d_zero_q, zq));
    HIP_TRY(upload(&a->d_zero_d, zd));
    for (int v = 0; v < kNumVariants; ++v) {
        if (cls[v].empty() || dn.empty()) continue;
        auto &c = cls[v];
        std::stable_sort(c.begin(), c.end(), [&](uint32_t x, uint32_t y) {
            return q_off[x + 1] - q_off[x] > q_off[y + 1] - q_off[y];
        });
        saln_nw_avsa::Class k;
        k.variant = v;
        k.nq = (uint32_t)c.size();
        HIP_TRY(upload(&k.d_qids, c));
        a->classes.push_back(k);
    }
    if (!fbq.empty() && !dn.empty()) {
        const uint64_t n = (uint64_t)fbq.size() * dn.size();
        if (n > 0x7FFFFFFFull) {
            set_error("too many pairs outside the packed region for one plan");
            return SALN_E_INVALID;
        }
        std::vector<uint32_t> pq(n), pd(n);
        for (uint64_t k = 0; k < n; ++k) {
            pq[k] = fbq[k % fbq.size()];
            pd[k] = dn[k / fbq.size()];
        }
        const int rc = saln_nw_plan_create(ctx, q_off, n_q, db_off, n_db, pq.data(), pd.data(),
                                           n, mode, scoring, &a->fb);
        if (rc != SALN_OK) return rc;
        saln_nw_plan_set_score_only(a->fb, 1);
        a->n_fb = (uint32_t)fbq.size();
        HIP_TRY(upload(&a->d_fb_qids, fbq));
        HIP_TRY(hipMalloc(&a->d_fb_res, n * sizeof(saln_nw_result)));
    }
    *out = a.release();
    return SALN_OK;
}

int saln_nw_avsa_execute(saln_nw_avsa *a, const uint8_t *d_q_seq, const uint8_t *d_db_seq,
                         int32_t *d_out, void *stream) {
    if (!a || !d_out) return SALN_E_INVALID;
    if (a->n_q * a->n_db == 0) return SALN_OK;
    HIP_TRY(hipSetDevice(a->ctx->device));
    hipStream_t s = resolve_stream(stream, a->ctx);
    int2 *out = reinterpret_cast<int2 *>(d_out);
    const uint32_t nqt = (uint32_t)a->n_q;
    // the 8 x 19 class runs with query profiles when every byte is A, C, G
    // or T: checked here on the device, read by the kernel (no host sync)
    const bool prof = a->opts[Opt::AvsaProfile] != 0 && a->n_dn >= 2 &&
                      std::any_of(a->classes.begin(), a->classes.end(),
                                  [](const saln_nw_avsa::Class &c) { return c.variant == 4; });
    // the other classes take table penalties under the same check (nw.pk_tab)
    const bool checked = prof || a->opts[Opt::PkTab] != 0;
    const uint32_t *generic = checked ? a->d_generic : nullptr;
    if (checked) {
        HIP_TRY(hipMemsetAsync(a->d_generic, 0, sizeof(uint32_t), s));
        HIP_TRY(launch_acgt_check(d_q_seq, a->q_bytes, a->d_generic, s));
        HIP_TRY(launch_acgt_check(d_db_seq, a->d_bytes, a->d_generic, s));
    }
    for (const auto &c : a->classes) {
        // pairs per launch: the dispatch packet's grid size is a 32-bit count
        // of work-items, so the chunk depends on the class's pairs per block
        const uint64_t kChunk = avsa_chunk_pairs(c.variant);
        uint64_t total = (uint64_t)c.nq * a->n_dn;
        if (prof && c.variant == 4) {
            // whole db pairs through the profile kernel, an odd last db record
            // through the plain one
            const uint64_t tp = (uint64_t)c.nq * (a->n_dn & ~1u);
            hipError_t e = hipSuccess;
            for (uint64_t base = 0; base < tp && e == hipSuccess; base += kChunk) {
                const uint32_t n = (uint32_t)std::min<uint64_t>(kChunk, tp - base);
                e = launch_avsa_prof(a->d_qoff, a->d_doff, c.d_qids, c.nq, a->d_dids, nqt, base, n,
                                     d_q_seq, d_db_seq, out, a->sc, a->ld_max, a->d_generic, s,
                                     a->opts);
            }
            if (e == hipSuccess) {
                if (a->n_dn & 1u)
                    HIP_TRY(launch_avsa(c.variant, a->d_qoff, a->d_doff, c.d_qids, c.nq,
                                        a->d_dids + (a->n_dn - 1), nqt, 0, c.nq, d_q_seq, d_db_seq,
                                        out, a->sc, a->ld_max, s, a->opts, generic));
                continue;
            }
            if (e != hipErrorInvalidValue) HIP_TRY(e);  // not applicable: the plain path
            (void)hipGetLastError();
        }
        for (uint64_t base = 0; base < total; base += kChunk) {
            const uint32_t n = (uint32_t)std::min<uint64_t>(kChunk, total - base);
            HIP_TRY(launch_avsa(c.variant, a->d_qoff, a->d_doff, c.d_qids, c.nq, a->d_dids, nqt,
                                base, n, d_q_seq, d_db_seq, out, a->sc, a->ld_max, s, a->opts,
                                generic));
        }
    }
    // empty db records x every query; empty queries x non-empty db records
    HIP_TRY(launch_avsa_boundary(a->d_qoff, a->d_doff, nullptr, nqt, a->d_zero_d,
                                 (uint64_t)nqt * a->n_zd, nqt, out, a->sc, s));
    HIP_TRY(launch_avsa_boundary(a->d_qoff, a->d_doff, a->d_zero_q, a->n_zq, a->d_dids,
                                 (uint64_t)a->n_zq * a->n_dn, nqt, out, a->sc, s));
    if (a->fb) {
        // the caller's stream argument as given: `s` is the resolved handle,
        // and a resolved legacy null stream (0) would read as "the context's
        // own stream" there, unordered with the scatter below
        const int rc = saln_nw_execute(a->fb, d_q_seq, d_db_seq, a->d_fb_res, nullptr, stream);
        if (rc != SALN_OK) return rc;
        HIP_TRY(launch_avsa_scatter(a->d_fb_res, a->d_fb_qids, a->n_fb, a->d_dids,
                                    (uint64_t)a->n_fb * a->n_dn, nqt, out, s));
    }
    return SALN_OK;
}

int saln_nw_avsa_info(const saln_nw_avsa *a, uint64_t *cells, uint64_t *fallback_pairs) {
    if (!a) return SALN_E_INVALID;
    if (cells) *cells = a->cells;
    if (fallback_pairs) *fallback_pairs = (uint64_t)a->n_fb * a->n_dn;
    return SALN_OK;
}

int saln_nw_avsa_launch_geometry(int variant, uint64_t *chunk_pairs, uint64_t *grid_blocks) {
    const uint64_t c = avsa_chunk_pairs(variant);
    if (!c) return SALN_E_INVALID;
    if (chunk_pairs) *chunk_pairs = c;
    if (grid_blocks) *grid_blocks = avsa_launch_blocks(variant, c);
    return SALN_OK;
}

int saln_nw_avsa_status(saln_nw_avsa *a, uint32_t *flags) {
    if (flags) *flags = 0;
    if (!a) return SALN_E_INVALID;
    return a->fb ? saln_nw_plan_status(a->fb, flags) : SALN_OK;
}

int saln_nw_avsa_destroy(saln_nw_avsa *a) {
    if (!a) return SALN_OK;
    (void)hipSetDevice(a->ctx->device);
    delete a;
    return SALN_OK;
}

}  // extern "C"

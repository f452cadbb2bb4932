// Host-buffer entry points of the C ABI: per-pair n_w_align replacement,
// host batch, reference-text rendering and dense-mask export.  Each one is a
// thin wrapper: upload -> plan -> saln_nw_execute (GPU) -> download.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "nw_host.hpp"

using namespace saln;

namespace {

// a context-cached device block (saln::dev_alloc), released on scope exit
struct DevBuf {
    saln_context *ctx;
    void *p = nullptr;
    explicit DevBuf(saln_context *c) : ctx(c) {}
    ~DevBuf() {
        if (p) {
            (void)hipDeviceSynchronize();
            dev_free(ctx, p);
        }
    }
    hipError_t alloc(size_t n) { return dev_alloc(ctx, &p, n); }
};

#define TRY_HIP(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) {                                                            \
            set_error(std::string(#expr) + ": " + hipGetErrorString(e_));                  \
            return SALN_E_HIP;                                                             \
        }                                                                                  \
    } while (0)

struct PlanGuard {
    saln_nw_plan *p = nullptr;
    ~PlanGuard() { saln_nw_plan_destroy(p); }
};

}  // namespace

static int run_batch(saln_context *ctx, const uint8_t *q_seq, const uint64_t *q_off, uint64_t n_q,
                     const uint8_t *db_seq, const uint64_t *db_off, uint64_t n_db,
                     const uint32_t *pair_q, const uint32_t *pair_db, uint64_t n_pairs,
                     int32_t mode, const saln_nw_scoring *scoring, saln_nw_result *results,
                     uint32_t *cigar, const uint64_t *cigar_off,
                     std::vector<PairMask> *masks_out) {
    StageClock clk;
    PlanGuard g;
    int rc = saln_nw_plan_create(ctx, q_off, n_q, db_off, n_db, pair_q, pair_db, n_pairs, mode,
                                 scoring, &g.p);
    if (rc == SALN_NOT_IMPLEMENTED) {
        for (uint64_t k = 0; k < n_pairs; ++k) {
            std::memset(&results[k], 0, sizeof(saln_nw_result));
            results[k].status = SALN_NOT_IMPLEMENTED;
        }
        return rc;
    }
    if (rc != SALN_OK) return rc;
    if (masks_out) plan_set_full_codes(g.p, true);
    clk.mark("plan");
    std::vector<uint64_t> coff(n_pairs + 1);
    saln_nw_cigar_offsets(g.p, coff.data());
    uint64_t cig_words = coff[n_pairs];
    DevBuf dq(ctx), dd(ctx), dr(ctx), dc(ctx);
    const uint64_t qbytes = q_off[n_q], dbytes = db_off[n_db];
    TRY_HIP(dq.alloc(qbytes));
    TRY_HIP(dd.alloc(dbytes));
    TRY_HIP(dr.alloc(n_pairs * sizeof(saln_nw_result)));
    TRY_HIP(dc.alloc(cig_words * 4));
    if (qbytes) TRY_HIP(hipMemcpy(dq.p, q_seq, qbytes, hipMemcpyHostToDevice));
    if (dbytes) TRY_HIP(hipMemcpy(dd.p, db_seq, dbytes, hipMemcpyHostToDevice));
    clk.mark("alloc+h2d");
    rc = saln_nw_execute(g.p, (const uint8_t *)dq.p, (const uint8_t *)dd.p,
                         (saln_nw_result *)dr.p, (uint32_t *)dc.p, nullptr);
    if (rc != SALN_OK) return rc;
    TRY_HIP(hipDeviceSynchronize());
    if ((rc = plan_check_error(g.p)) != SALN_OK) return rc;
    clk.mark("execute");
    TRY_HIP(hipMemcpy(results, dr.p, n_pairs * sizeof(saln_nw_result), hipMemcpyDeviceToHost));
    // CIGARs: packed densely on the device, one download of the used words
    // into pinned staging, scattered to the caller's offsets
    std::vector<uint64_t> doff(n_pairs + 1, 0);
    for (uint64_t k = 0; k < n_pairs; ++k) doff[k + 1] = doff[k] + results[k].cigar_len;
    const uint32_t *hc = nullptr;
    DevBuf dso(ctx), ddo(ctx), dcd(ctx);
    if (cigar && doff[n_pairs]) {
        TRY_HIP(dso.alloc((n_pairs + 1) * 8));
        TRY_HIP(ddo.alloc((n_pairs + 1) * 8));
        TRY_HIP(dcd.alloc(doff[n_pairs] * 4));
        TRY_HIP(hipMemcpy(dso.p, coff.data(), (n_pairs + 1) * 8, hipMemcpyHostToDevice));
        TRY_HIP(hipMemcpy(ddo.p, doff.data(), (n_pairs + 1) * 8, hipMemcpyHostToDevice));
        TRY_HIP(launch_cigar_compact((const saln_nw_result *)dr.p, (const uint64_t *)dso.p,
                                     (const uint64_t *)ddo.p, (const uint32_t *)dc.p,
                                     (uint32_t *)dcd.p, n_pairs, ctx->stream));
        void *st = nullptr;
        TRY_HIP(pinned_staging(ctx, doff[n_pairs] * 4, &st));
        TRY_HIP(hipMemcpyAsync(st, dcd.p, doff[n_pairs] * 4, hipMemcpyDeviceToHost, ctx->stream));
        TRY_HIP(hipStreamSynchronize(ctx->stream));
        hc = (const uint32_t *)st;
    }
    clk.mark("d2h");
    if (cigar && hc) {
        // ~10^5 small copies (a few hundred bytes each): split over host threads
        auto scatter = [&](uint64_t a, uint64_t b) {
            for (uint64_t k = a; k < b; ++k) {
                const uint64_t dst = cigar_off ? cigar_off[k] : coff[k];
                std::memcpy(cigar + dst, hc + doff[k], results[k].cigar_len * 4);
            }
        };
        const uint64_t nt = std::min<uint64_t>(
            std::max(1u, std::min(16u, std::thread::hardware_concurrency())), n_pairs / 4096 + 1);
        if (nt <= 1) {
            scatter(0, n_pairs);
        } else {
            std::vector<std::thread> th;
            for (uint64_t t = 1; t < nt; ++t)
                th.emplace_back(scatter, n_pairs * t / nt, n_pairs * (t + 1) / nt);
            scatter(0, n_pairs / nt);
            for (auto &x : th) x.join();
        }
    }
    clk.mark("scatter");
    // callers that render reference text get every pair's full parent codes
    if (masks_out) {
        masks_out->resize(n_pairs);
        for (uint64_t k = 0; k < n_pairs; ++k) {
            rc = plan_pair_mask(g.p, k, &(*masks_out)[k]);
            if (rc != SALN_OK) return rc;
        }
    }
    clk.mark("fixups");
    return SALN_OK;
}

extern "C" {

int saln_nw_align_batch(saln_context *ctx, const uint8_t *q_seq, const uint64_t *q_off,
                        uint64_t n_q, const uint8_t *db_seq, const uint64_t *db_off,
                        uint64_t n_db, const uint32_t *pair_q, const uint32_t *pair_db,
                        uint64_t n_pairs, int32_t mode, const saln_nw_scoring *scoring,
                        saln_nw_result *results, uint32_t *cigar, const uint64_t *cigar_off) {
    if (!ctx || !q_off || !db_off || !results) return SALN_E_INVALID;
    return run_batch(ctx, q_seq, q_off, n_q, db_seq, db_off, n_db, pair_q, pair_db, n_pairs, mode,
                     scoring, results, cigar, cigar_off, nullptr);
}

int saln_nw_align(saln_context *ctx, const uint8_t *q, uint64_t len_q, const uint8_t *d,
                  uint64_t len_db, int verbose, int32_t mode, const saln_nw_scoring *scoring,
                  saln_nw_result *out, uint32_t *cigar, uint64_t cigar_cap) {
    (void)verbose;  // `_verbose` is unused by the reference (:424)
    if (!ctx || !out || (len_q && !q) || (len_db && !d)) return SALN_E_INVALID;
    const uint64_t qo[2] = {0, len_q}, dof[2] = {0, len_db};
    const uint32_t z = 0;
    std::vector<uint32_t> c(len_q + len_db + 1);
    const uint64_t co[1] = {0};
    int rc = run_batch(ctx, q, qo, 1, d, dof, 1, &z, &z, 1, mode, scoring, out, c.data(), co,
                       nullptr);
    if (rc != SALN_OK) return rc;
    if (cigar) {
        if (out->cigar_len > cigar_cap) return SALN_E_CAPACITY;
        std::memcpy(cigar, c.data(), out->cigar_len * 4);
    }
    return SALN_OK;
}

int saln_nw_render(saln_context *ctx, const uint8_t *q, uint64_t len_q, const uint8_t *d,
                   uint64_t len_db, int32_t mode, uint64_t max_blocks, char *out, uint64_t cap,
                   uint64_t *out_len, uint64_t *n_blocks, int32_t *status) {
    if (!ctx || (len_q && !q) || (len_db && !d)) return SALN_E_INVALID;
    const uint64_t qo[2] = {0, len_q}, dof[2] = {0, len_db};
    const uint32_t z = 0;
    saln_nw_result r;
    std::vector<PairMask> masks;
    int rc = run_batch(ctx, q, qo, 1, d, dof, 1, &z, &z, 1, mode, nullptr, &r, nullptr, nullptr,
                       &masks);
    if (rc == SALN_NOT_IMPLEMENTED) {
        if (status) *status = SALN_NOT_IMPLEMENTED;
        if (out_len) *out_len = 0;
        if (n_blocks) *n_blocks = 0;
        return rc;
    }
    if (rc != SALN_OK) return rc;
    const HostMask hm(masks[0], (uint32_t)len_q, (uint32_t)len_db, scoring_or_default(nullptr));
    std::string text;
    const DfsOutcome o = render_blocks(hm, q, d, max_blocks, &text);
    if (out_len) *out_len = text.size();
    if (n_blocks) *n_blocks = o.blocks;
    if (status) *status = o.status;
    if (out) {
        std::memcpy(out, text.data(), text.size() < cap ? text.size() : cap);
        if (text.size() > cap) return SALN_E_CAPACITY;
    }
    return SALN_OK;
}

int saln_nw_dense_mask(saln_context *ctx, const uint8_t *q, uint64_t len_q, const uint8_t *d,
                       uint64_t len_db, const saln_nw_scoring *scoring, uint8_t *out) {
    if (!ctx || !out || (len_q && !q) || (len_db && !d)) return SALN_E_INVALID;
    const uint64_t qo[2] = {0, len_q}, dof[2] = {0, len_db};
    const uint32_t z = 0;
    saln_nw_result r;
    std::vector<PairMask> masks;
    int rc = run_batch(ctx, q, qo, 1, d, dof, 1, &z, &z, 1, SALN_MODE_GLOBAL, scoring, &r,
                       nullptr, nullptr, &masks);
    if (rc != SALN_OK) return rc;
    const HostMask hm(masks[0], (uint32_t)len_q, (uint32_t)len_db, scoring_or_default(scoring));
    hm.to_dense(out);
    return SALN_OK;
}

}  // extern "C"

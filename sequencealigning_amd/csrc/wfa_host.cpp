// C ABI of the WFA engine (include/saln.h): replaces wfa_align
// (src/wfa.rs:23-42) and, batched, the pair loop of src/main.rs:61-67 for
// `-a wfa`.  The score loop, trim and traceback run in wfa_kernels.hip; the
// host uploads, launches in chunks that bound the tensor-history arena, and
// formats the reference's stdout from the per-step and traceback logs the
// kernel writes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "nw_host.hpp"
#include "wfa_host.hpp"

using namespace saln;

namespace {

#define TRY_HIP(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) {                                                            \
            set_error(std::string(#expr) + ": " + hipGetErrorString(e_));                  \
            return SALN_E_HIP;                                                             \
        }                                                                                  \
    } while (0)

struct DevBuf {
    void *p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    hipError_t alloc(size_t n) { return hipMalloc(&p, n ? n : 1); }
};

constexpr uint32_t kDefaultSteps = 64, kDefaultWidth = 64;
// bytes of tensor history per launch: sized for 288 GB of HBM, capped by the
// free memory at plan time (WfaScratch::arena)
constexpr uint64_t kArenaBudget = 32ull << 30;
// Batch runs start every pair with this step cap (a small arena, many lanes
// per launch); the pairs that reach it are re-run with the caller's cap.
// Essentially every realistic pair ends far earlier (REF_PANIC_TRIM at s = 20,
// SURVEY.md §8.5), so the big arena is only paid for the few that need it.
constexpr uint32_t kFirstPassSteps = 32;

uint32_t ev_cap_for(uint32_t max_steps) { return 7 * (max_steps / 4 + 2) + 8; }

struct Logs {
    std::vector<int32_t> lohi;  // 2 per pair-step
    std::vector<uint8_t> ev;    // ev_cap per pair
    uint32_t ev_cap = 0;
};

// Device scratch reused across launches / executes.
struct WfaScratch {
    DevBuf hdr, off, meta, tsome;
    uint64_t S = 0, W = 0, nl = 0;
    DevBuf rerun, cnt;
    uint64_t rerun_n = 0;

    hipError_t arena(uint64_t S_, uint64_t W_, uint64_t n_pairs, WfaArena *out) {
        const uint64_t per_lane = S_ * 3 * 4 * 4 + S_ * 3 * W_ * 8 + S_;
        // at most kArenaBudget, and at most half of the device memory free
        // now (the arena held so far counts as free: it is replaced)
        uint64_t budget = kArenaBudget;
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess) {
            const uint64_t held = S * 3 * 4 * 4 * nl + S * 3 * W * 8 * nl + S * nl;
            budget = std::min<uint64_t>(budget, (fr + held) / 2);
        } else {
            (void)hipGetLastError();
        }
        uint64_t nl_ = std::max<uint64_t>(256, std::min<uint64_t>(n_pairs, budget / per_lane));
        nl_ = std::min<uint64_t>(nl_, n_pairs);
        if (S_ * nl_ > S * nl || S_ * W_ * nl_ > S * W * nl) {
            for (;;) {  // out of memory: halve the lanes per launch (down to 256)
                for (DevBuf *b : {&hdr, &off, &meta, &tsome}) {
                    if (b->p) (void)hipFree(b->p);
                    b->p = nullptr;
                }
                S = W = nl = 0;
                hipError_t e;
                if ((e = hdr.alloc(S_ * 3 * 4 * nl_ * sizeof(int32_t))) == hipSuccess &&
                    (e = off.alloc(S_ * 3 * W_ * nl_ * sizeof(int32_t))) == hipSuccess &&
                    (e = meta.alloc(S_ * 3 * W_ * nl_ * sizeof(uint32_t))) == hipSuccess &&
                    (e = tsome.alloc(S_ * nl_)) == hipSuccess)
                    break;
                if (e != hipErrorOutOfMemory || nl_ <= 256) return e;
                (void)hipGetLastError();
                nl_ = std::max<uint64_t>(256, nl_ / 2);
            }
            S = S_;
            W = W_;
            nl = nl_;
        }
        // the kernel indexes with the launch's own (S, W, nl) inside the buffers
        *out = WfaArena{(int32_t *)hdr.p, (int32_t *)off.p, (uint32_t *)meta.p,
                        (uint8_t *)tsome.p, (uint32_t)nl_, (uint32_t)S_, (uint32_t)W_};
        return hipSuccess;
    }
};

// One pass over n pairs with step cap `steps`, chunked by the arena budget.
int wfa_pass(WfaScratch &ws, const WfaPairDesc *d_pairs, uint32_t n, const uint8_t *dq,
             const uint8_t *dd, uint32_t steps, uint32_t width, saln_wfa_result *d_res,
             uint8_t *d_aln, int32_t *d_lohi, uint8_t *d_ev, uint32_t ev_cap, WfaPairDesc *rerun,
             uint32_t *rerun_cnt, hipStream_t s) {
    WfaArena arena;
    TRY_HIP(ws.arena(steps / 2 + 1, width, n, &arena));
    for (uint64_t first = 0; first < n; first += arena.nl) {
        const uint32_t cnt = (uint32_t)std::min<uint64_t>(arena.nl, n - first);
        TRY_HIP(launch_wfa(d_pairs, (uint32_t)first, cnt, dq, dd, arena, steps, d_res, d_aln,
                           d_lohi, d_ev, ev_cap, rerun, rerun_cnt, s));
    }
    return SALN_OK;
}

// All pairs of d_pairs[0, n): with per-step logs (render) one pass at the
// caller's cap; otherwise a short first pass and a full-cap pass over the
// pairs that reached the short cap.  Results are identical either way: a
// pair's run does not depend on the cap until it reaches it.
int wfa_device(WfaScratch &ws, const WfaPairDesc *d_pairs, uint32_t n, const uint8_t *dq,
               const uint8_t *dd, uint32_t max_steps, uint32_t width, saln_wfa_result *d_res,
               uint8_t *d_aln, int32_t *d_lohi, uint8_t *d_ev, uint32_t ev_cap, hipStream_t s) {
    if (!n) return SALN_OK;
    if (d_lohi || max_steps <= kFirstPassSteps)
        return wfa_pass(ws, d_pairs, n, dq, dd, max_steps, width, d_res, d_aln, d_lohi, d_ev,
                        ev_cap, nullptr, nullptr, s);
    if (ws.rerun_n < n) {
        if (ws.rerun.p) (void)hipFree(ws.rerun.p);
        ws.rerun.p = nullptr;
        TRY_HIP(ws.rerun.alloc((uint64_t)n * sizeof(WfaPairDesc)));
        ws.rerun_n = n;
    }
    if (!ws.cnt.p) TRY_HIP(ws.cnt.alloc(sizeof(uint32_t)));
    TRY_HIP(hipMemsetAsync(ws.cnt.p, 0, sizeof(uint32_t), s));
    int rc = wfa_pass(ws, d_pairs, n, dq, dd, kFirstPassSteps, width, d_res, d_aln, nullptr,
                      nullptr, 0, (WfaPairDesc *)ws.rerun.p, (uint32_t *)ws.cnt.p, s);
    if (rc != SALN_OK) return rc;
    uint32_t again = 0;
    TRY_HIP(hipMemcpyAsync(&again, ws.cnt.p, sizeof again, hipMemcpyDeviceToHost, s));
    TRY_HIP(hipStreamSynchronize(s));
    if (!again) return SALN_OK;
    return wfa_pass(ws, (const WfaPairDesc *)ws.rerun.p, again, dq, dd, max_steps, width, d_res,
                    d_aln, nullptr, nullptr, 0, nullptr, nullptr, s);
}

int build_descs(const uint64_t *q_off, uint64_t n_q, const uint64_t *db_off, uint64_t n_db,
                const uint32_t *pair_q, const uint32_t *pair_db, uint64_t n_pairs, int32_t mode,
                const uint64_t *aln_off, uint32_t aln_cap, std::vector<WfaPairDesc> *out,
                uint64_t *aln_bytes) {
    out->resize(n_pairs);
    *aln_bytes = 0;
    for (uint64_t k = 0; k < n_pairs; ++k) {
        const uint64_t qi = pair_q ? pair_q[k] : k % n_q;
        const uint64_t di = pair_db ? pair_db[k] : k / n_q;
        if (qi >= n_q || di >= n_db) {
            set_error("pair index out of range");
            return SALN_E_INVALID;
        }
        WfaPairDesc &d = (*out)[k];
        std::memset(&d, 0, sizeof d);
        d.q_off = q_off[qi];
        d.db_off = db_off[di];
        const uint64_t lq = q_off[qi + 1] - q_off[qi], ld = db_off[di + 1] - db_off[di];
        if (lq > 0x7FFFFFFFull || ld > 0x7FFFFFFFull) {
            set_error("sequence too long");
            return SALN_E_INVALID;
        }
        d.len_q = (uint32_t)lq;
        d.len_db = (uint32_t)ld;
        d.pair_id = (uint32_t)k;
        d.mode = mode;
        d.aln_cap = aln_cap;
        d.aln_off = aln_cap && aln_off ? aln_off[k] : 0;
        if (aln_cap) *aln_bytes = std::max<uint64_t>(*aln_bytes, d.aln_off + 2ull * aln_cap);
    }
    return SALN_OK;
}

// Runs the pairs; logs (optional) receive the per-step lo/hi and the rec_tr
// events of every pair (used for rendering).
int run_wfa(saln_context *ctx, const uint8_t *q_seq, const uint64_t *q_off, uint64_t n_q,
            const uint8_t *db_seq, const uint64_t *db_off, uint64_t n_db, const uint32_t *pair_q,
            const uint32_t *pair_db, uint64_t n_pairs, int32_t mode, uint32_t max_steps,
            uint32_t max_width, saln_wfa_result *results, uint8_t *aln, const uint64_t *aln_off,
            uint32_t aln_cap, Logs *logs) {
    if (!ctx || !q_off || !db_off || !results) return SALN_E_INVALID;
    if (!max_steps) max_steps = kDefaultSteps;
    if (!max_width) max_width = kDefaultWidth;
    if (n_pairs == 0) return SALN_OK;
    if (n_pairs > 0xFFFFFFFFull) return SALN_E_INVALID;
    TRY_HIP(hipSetDevice(ctx->device));
    std::vector<WfaPairDesc> descs;
    uint64_t aln_bytes = 0;
    int rc = build_descs(q_off, n_q, db_off, n_db, pair_q, pair_db, n_pairs, mode, aln_off,
                         aln ? aln_cap : 0, &descs, &aln_bytes);
    if (rc != SALN_OK) return rc;
    const uint64_t qbytes = q_off[n_q], dbytes = db_off[n_db];
    DevBuf dq, dd, dp, dr, da, dl, de;
    TRY_HIP(dq.alloc(qbytes));
    TRY_HIP(dd.alloc(dbytes));
    TRY_HIP(dp.alloc(n_pairs * sizeof(WfaPairDesc)));
    TRY_HIP(dr.alloc(n_pairs * sizeof(saln_wfa_result)));
    if (qbytes) TRY_HIP(hipMemcpy(dq.p, q_seq, qbytes, hipMemcpyHostToDevice));
    if (dbytes) TRY_HIP(hipMemcpy(dd.p, db_seq, dbytes, hipMemcpyHostToDevice));
    TRY_HIP(hipMemcpy(dp.p, descs.data(), n_pairs * sizeof(WfaPairDesc), hipMemcpyHostToDevice));
    if (aln) TRY_HIP(da.alloc(aln_bytes));
    const uint32_t ev_cap = ev_cap_for(max_steps);
    if (logs) {
        TRY_HIP(dl.alloc(n_pairs * 2ull * max_steps * sizeof(int32_t)));
        TRY_HIP(de.alloc(n_pairs * (uint64_t)ev_cap));
    }
    WfaScratch ws;
    rc = wfa_device(ws, (const WfaPairDesc *)dp.p, (uint32_t)n_pairs, (const uint8_t *)dq.p,
                    (const uint8_t *)dd.p, max_steps, max_width, (saln_wfa_result *)dr.p,
                    (uint8_t *)da.p, (int32_t *)dl.p, (uint8_t *)de.p, ev_cap, ctx->stream);
    if (rc != SALN_OK) return rc;
    TRY_HIP(hipStreamSynchronize(ctx->stream));
    TRY_HIP(hipMemcpy(results, dr.p, n_pairs * sizeof(saln_wfa_result), hipMemcpyDeviceToHost));
    if (aln) TRY_HIP(hipMemcpy(aln, da.p, aln_bytes, hipMemcpyDeviceToHost));
    if (logs) {
        logs->lohi.resize(n_pairs * 2ull * max_steps);
        logs->ev.resize(n_pairs * (uint64_t)ev_cap);
        logs->ev_cap = ev_cap;
        TRY_HIP(hipMemcpy(logs->lohi.data(), dl.p, logs->lohi.size() * sizeof(int32_t),
                          hipMemcpyDeviceToHost));
        TRY_HIP(hipMemcpy(logs->ev.data(), de.p, logs->ev.size(), hipMemcpyDeviceToHost));
    }
    return SALN_OK;
}

const char *state_name(int s) { return s == 0 ? "M" : s == 1 ? "D" : "I"; }

void appendf(std::string *s, const char *fmt, long long v) {
    char b[64];
    std::snprintf(b, sizeof b, fmt, v);
    *s += b;
}

// The text wfa_align prints for one pair (wfa.rs; lines cited inline) from
// its result, its per-step lo/hi log, its rec_tr event log and its alignment
// rows (a1/a2, acap bytes each, reversed as the reference pushes them).
void render_pair(const saln_wfa_result &r, const int32_t *lohi, const uint8_t *ev, uint32_t nev,
                 const uint8_t *a1, const uint8_t *a2, uint32_t acap, long long diag,
                 std::string *out) {
    std::string &t = *out;
    if (r.status != SALN_NOT_IMPLEMENTED) {
        // `lo: {}, hi: {}` of every WaveFrontTensor::new that had sources (:251)
        for (uint32_t s = 0; s < r.steps; ++s) {
            const int32_t lo = lohi[2 * s], hi = lohi[2 * s + 1];
            if (lo == INT32_MIN) continue;
            appendf(&t, "lo: %lld, ", lo);
            appendf(&t, "hi: %lld\n", hi);
        }
    }
    if (r.status == SALN_OK || r.status == SALN_REF_PANIC_SLICE) {
        appendf(&t, "converged with score %lld: \n", r.score);       // :38
        appendf(&t, "huhu, diag: %lld\n", diag);  // :650
        t += "Element {\n";                                            // Debug :103-116
        t += std::string("\tstate: ") + state_name(r.conv_state) + "\n";
        appendf(&t, "\toffset: %lld\n", r.conv_offset);
        if (!r.conv_np) {
            t += "\tparents: []\n";
        } else {
            t += "\tparents: [\n";
            for (int k = 0; k < r.conv_np; ++k)
                t += std::string("    ") + state_name(r.conv_parents[k]) + ",\n";
            t += "]\n";
        }
        t += "}\n";
        appendf(&t, "\nscore: %lld\n", r.score);
        // rec_tr events (:654-853): every attempt prints `well shit` or
        // `yeah, score: N`; an attempt that moves prints its action and the
        // walk restarts at the lower score; `open` without a move is the
        // last attempt, so `huh` follows it.
        enum { WELL = 0, YEAH = 1, MISMATCH = 2, EXTEND = 3, OPEN = 4, RET = 5, HUH = 6 };
        static const uint64_t nds[3] = {4, 6, 8};
        uint64_t score = (uint64_t)r.score;
        int attempt = 0;
        for (uint32_t k = 0; k < nev;) {
            const uint8_t e = ev[k++];
            if (e == RET) { t += "ret\n"; break; }
            if (e == HUH) { t += "huh\n"; break; }
            if (e == WELL) { t += "well shit\n"; ++attempt; continue; }
            if (e != YEAH || attempt >= 3) break;
            const uint64_t ns = score - nds[attempt];
            appendf(&t, "yeah, score: %lld\n", (long long)ns);
            const uint8_t nx = k < nev ? ev[k] : (uint8_t)HUH;
            if (nx == MISMATCH || nx == EXTEND) {
                t += nx == MISMATCH ? "mismatch\n" : "extend\n";
                ++k;
                score = ns;
                attempt = 0;
            } else if (nx == OPEN) {
                t += "open\n";
                ++k;
                if (k < nev && ev[k] == HUH) {
                    ++attempt;
                } else {
                    score = ns;
                    attempt = 0;
                }
            } else {
                ++attempt;
            }
        }
        if (r.status == SALN_OK) {
            // Display (:950-980) + println, then Debug (`{:#?}`)
            const uint32_t n1 = std::min(r.aln_len1, acap), n2 = std::min(r.aln_len2, acap);
            for (uint32_t k = n1; k > 0; --k) t += (char)a1[k - 1];
            t += "\n";
            for (uint32_t k = std::min(n1, n2); k > 0; --k) t += a1[k - 1] != a2[k - 1] ? " " : "|";
            for (uint32_t k = n2; k > 0; --k) t += (char)a2[k - 1];
            t += "\n\n";
            t += "Alignment {\n";
            const uint8_t *rows[2] = {a1, a2};
            const uint32_t lens[2] = {n1, n2};
            const char *names[2] = {"seq1", "seq2"};
            for (int w = 0; w < 2; ++w) {
                if (!lens[w]) {
                    t += std::string("    ") + names[w] + ": [],\n";
                    continue;
                }
                t += std::string("    ") + names[w] + ": [\n";
                for (uint32_t k = 0; k < lens[w]; ++k) appendf(&t, "        %lld,\n", rows[w][k]);
                t += "    ],\n";
            }
            t += "}\n";
        }
    }
}

}  // namespace

struct saln_wfa_text {
    std::vector<std::string> text;
    std::vector<saln_wfa_result> res;
};

struct saln_wfa_plan {
    saln_context *ctx = nullptr;
    uint32_t n_pairs = 0, max_steps = 0, max_width = 0;
    DevBuf pairs;
    WfaScratch ws;
};

extern "C" {

int saln_wfa_align_batch(saln_context *ctx, const uint8_t *q_seq, const uint64_t *q_off,
                         uint64_t n_q, const uint8_t *db_seq, const uint64_t *db_off,
                         uint64_t n_db, const uint32_t *pair_q, const uint32_t *pair_db,
                         uint64_t n_pairs, int32_t mode, uint32_t max_steps, uint32_t max_width,
                         saln_wfa_result *results, uint8_t *aln, const uint64_t *aln_off,
                         uint32_t aln_cap) {
    return run_wfa(ctx, q_seq, q_off, n_q, db_seq, db_off, n_db, pair_q, pair_db, n_pairs, mode,
                   max_steps, max_width, results, aln, aln_off, aln_cap, nullptr);
}

int saln_wfa_render(saln_context *ctx, const uint8_t *q, uint64_t len_q, const uint8_t *d,
                    uint64_t len_db, int32_t mode, uint32_t max_steps, uint32_t max_width,
                    char *out, uint64_t cap, uint64_t *out_len, saln_wfa_result *result) {
    if (!ctx || (len_q && !q) || (len_db && !d)) return SALN_E_INVALID;
    if (!max_steps) max_steps = kDefaultSteps;
    const uint64_t qo[2] = {0, len_q}, dof[2] = {0, len_db};
    const uint32_t z = 0;
    const uint32_t acap = (uint32_t)std::min<uint64_t>(0x7FFFFFFF, 2 * (len_q + len_db) + 64);
    std::vector<uint8_t> aln(2ull * acap);
    const uint64_t aoff = 0;
    saln_wfa_result r;
    Logs logs;
    int rc = run_wfa(ctx, q, qo, 1, d, dof, 1, &z, &z, 1, mode, max_steps, max_width, &r,
                     aln.data(), &aoff, acap, &logs);
    if (rc != SALN_OK) return rc;
    if (result) *result = r;
    std::string t;
    render_pair(r, logs.lohi.data(), logs.ev.data(), logs.ev_cap, aln.data(), aln.data() + acap,
                acap, (long long)len_q - (long long)len_db, &t);
    if (out_len) *out_len = t.size();
    if (out) {
        std::memcpy(out, t.data(), std::min<uint64_t>(t.size(), cap));
        if (t.size() > cap) return SALN_E_CAPACITY;
    }
    return SALN_OK;
}

// wfa_align's text for every pair of a batch, each pair computed once: one
// run_wfa over the batch with logs and alignment rows, then the per-pair
// rendering on host threads.
int saln_wfa_render_batch(saln_context *ctx, const uint8_t *q_seq, const uint64_t *q_off,
                          uint64_t n_q, const uint8_t *db_seq, const uint64_t *db_off,
                          uint64_t n_db, const uint32_t *pair_q, const uint32_t *pair_db,
                          uint64_t n_pairs, int32_t mode, uint32_t max_steps, uint32_t max_width,
                          saln_wfa_text **out) {
    if (!ctx || !q_off || !db_off || !out) return SALN_E_INVALID;
    *out = nullptr;
    if (!max_steps) max_steps = kDefaultSteps;
    auto t = std::make_unique<saln_wfa_text>();
    t->text.resize(n_pairs);
    t->res.resize(n_pairs);
    if (!n_pairs) {
        *out = t.release();
        return SALN_OK;
    }
    std::vector<uint32_t> pq(n_pairs), pd(n_pairs);
    std::vector<uint64_t> acap_k(n_pairs);
    for (uint64_t k = 0; k < n_pairs; ++k) {
        const uint64_t qi = pair_q ? pair_q[k] : k % std::max<uint64_t>(n_q, 1);
        const uint64_t di = pair_db ? pair_db[k] : k / std::max<uint64_t>(n_q, 1);
        if (qi >= n_q || di >= n_db) {
            set_error("pair index out of range");
            return SALN_E_INVALID;
        }
        pq[k] = (uint32_t)qi;
        pd[k] = (uint32_t)di;
        acap_k[k] = 2 * ((q_off[qi + 1] - q_off[qi]) + (db_off[di + 1] - db_off[di])) + 64;
        if (acap_k[k] > 0x7FFFFFFF) {
            set_error("saln_wfa_render_batch: sequence too long");
            return SALN_E_INVALID;
        }
    }
    // chunks whose host/device buffers (alignment rows sized for the chunk's
    // longest pair, the per-step lo/hi log and the rec_tr events) stay under
    // kChunkBytes; each chunk is one GPU run
    constexpr uint64_t kChunkBytes = 1ull << 30;
    const uint64_t per_log = 2ull * max_steps * sizeof(int32_t) + ev_cap_for(max_steps);
    const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    for (uint64_t c0 = 0; c0 < n_pairs;) {
        uint64_t acap = 64, c1 = c0;
        while (c1 < n_pairs) {
            const uint64_t cap = std::max(acap, acap_k[c1]);
            if (c1 > c0 && (c1 + 1 - c0) * (2 * cap + per_log) > kChunkBytes) break;
            acap = cap;
            ++c1;
        }
        const uint64_t n = c1 - c0;
        std::vector<uint8_t> aln(n * 2 * acap);
        std::vector<uint64_t> aoff(n);
        for (uint64_t k = 0; k < n; ++k) aoff[k] = k * 2 * acap;
        Logs logs;
        int rc = run_wfa(ctx, q_seq, q_off, n_q, db_seq, db_off, n_db, pq.data() + c0,
                         pd.data() + c0, n, mode, max_steps, max_width, t->res.data() + c0,
                         aln.data(), aoff.data(), (uint32_t)acap, &logs);
        if (rc != SALN_OK) return rc;
        const unsigned nth = (unsigned)std::min<uint64_t>(hw, (n + 63) / 64);
        std::atomic<uint64_t> next{0};
        auto work = [&] {
            for (uint64_t k; (k = next.fetch_add(1)) < n;) {
                const uint64_t g = c0 + k;
                const uint8_t *al = aln.data() + aoff[k];
                const long long diag = (long long)(q_off[pq[g] + 1] - q_off[pq[g]]) -
                                       (long long)(db_off[pd[g] + 1] - db_off[pd[g]]);
                render_pair(t->res[g], logs.lohi.data() + k * 2 * max_steps,
                            logs.ev.data() + k * logs.ev_cap, logs.ev_cap, al, al + acap,
                            (uint32_t)acap, diag, &t->text[g]);
            }
        };
        std::vector<std::thread> th;
        for (unsigned i = 1; i < nth; ++i) th.emplace_back(work);
        work();
        for (auto &x : th) x.join();
        c0 = c1;
    }
    *out = t.release();
    return SALN_OK;
}

uint64_t saln_wfa_text_count(const saln_wfa_text *t) { return t ? t->text.size() : 0; }

int saln_wfa_text_get(const saln_wfa_text *t, uint64_t pair, const char **text, uint64_t *len,
                      saln_wfa_result *result) {
    if (!t || pair >= t->text.size()) return SALN_E_INVALID;
    if (text) *text = t->text[pair].data();
    if (len) *len = t->text[pair].size();
    if (result) *result = t->res[pair];
    return SALN_OK;
}

void saln_wfa_text_free(saln_wfa_text *t) { delete t; }

int saln_wfa_plan_create(saln_context *ctx, const uint64_t *q_off, uint64_t n_q,
                         const uint64_t *db_off, uint64_t n_db, const uint32_t *pair_q,
                         const uint32_t *pair_db, uint64_t n_pairs, int32_t mode,
                         uint32_t max_steps, uint32_t max_width, saln_wfa_plan **out) {
    if (!ctx || !q_off || !db_off || !out) return SALN_E_INVALID;
    *out = nullptr;
    if (n_pairs > 0xFFFFFFFFull) return SALN_E_INVALID;
    TRY_HIP(hipSetDevice(ctx->device));
    auto p = std::make_unique<saln_wfa_plan>();
    p->ctx = ctx;
    p->n_pairs = (uint32_t)n_pairs;
    p->max_steps = max_steps ? max_steps : kDefaultSteps;
    p->max_width = max_width ? max_width : kDefaultWidth;
    std::vector<WfaPairDesc> descs;
    uint64_t ab = 0;
    int rc = build_descs(q_off, n_q, db_off, n_db, pair_q, pair_db, n_pairs, mode, nullptr, 0,
                         &descs, &ab);
    if (rc != SALN_OK) return rc;
    if (n_pairs) {
        TRY_HIP(p->pairs.alloc(n_pairs * sizeof(WfaPairDesc)));
        TRY_HIP(hipMemcpy(p->pairs.p, descs.data(), n_pairs * sizeof(WfaPairDesc),
                          hipMemcpyHostToDevice));
    }
    *out = p.release();
    return SALN_OK;
}

int saln_wfa_execute(saln_wfa_plan *p, const uint8_t *d_q_seq, const uint8_t *d_db_seq,
                     saln_wfa_result *d_results, void *stream) {
    if (!p || (p->n_pairs && (!d_q_seq || !d_db_seq || !d_results))) return SALN_E_INVALID;
    TRY_HIP(hipSetDevice(p->ctx->device));
    hipStream_t s = resolve_stream(stream, p->ctx);
    return wfa_device(p->ws, (const WfaPairDesc *)p->pairs.p, p->n_pairs, d_q_seq, d_db_seq,
                      p->max_steps, p->max_width, d_results, nullptr, nullptr, nullptr, 0, s);
}

int saln_wfa_plan_destroy(saln_wfa_plan *p) {
    if (!p) return SALN_OK;
    (void)hipSetDevice(p->ctx->device);
    delete p;
    return SALN_OK;
}

}  // extern "C"

// Host-buffer entry points of the C ABI: per-pair n_w_align replacement,
// host batch, reference-text rendering and dense-mask export.  Each one is a
// thin wrapper: upload -> plan -> saln_nw_execute (GPU) -> download.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <new>
#include <numeric>
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
    if (!ctx) return SALN_E_INVALID;
    StageClock clk(ctx->opts.effective());
    if (!q_off || !db_off || (n_q && !q_seq && q_off[n_q]) || (n_db && !db_seq && db_off[n_db]))
        return SALN_E_INVALID;
    // the sequences' upload runs on a helper thread while this one plans (the
    // plan is host work: descriptors, order, layout), joined before execute
    DevBuf dq(ctx), dd(ctx), dr(ctx), dc(ctx);
    const uint64_t qbytes = q_off[n_q], dbytes = db_off[n_db];
    TRY_HIP(dq.alloc(qbytes));
    TRY_HIP(dd.alloc(dbytes));
    hipError_t up_err = hipSuccess;
    const bool upload = mode == SALN_MODE_GLOBAL;  // other modes: every pair "not implemented"
    std::thread up([&] {
        if (!upload) return;
        up_err = hipSetDevice(ctx->device);
        if (up_err == hipSuccess && qbytes) up_err = hipMemcpy(dq.p, q_seq, qbytes, hipMemcpyHostToDevice);
        if (up_err == hipSuccess && dbytes) up_err = hipMemcpy(dd.p, db_seq, dbytes, hipMemcpyHostToDevice);
    });
    struct Joiner {
        std::thread &t;
        ~Joiner() { if (t.joinable()) t.join(); }
    } joiner{up};
    PlanGuard g;
    int rc = plan_create(ctx, q_off, n_q, db_off, n_db, pair_q, pair_db, n_pairs, mode, scoring,
                         masks_out != nullptr, &g.p);
    if (rc == SALN_NOT_IMPLEMENTED) {
        for (uint64_t k = 0; k < n_pairs; ++k) {
            std::memset(&results[k], 0, sizeof(saln_nw_result));
            results[k].status = SALN_NOT_IMPLEMENTED;
        }
        return rc;
    }
    if (rc != SALN_OK) return rc;
    clk.mark("plan (upload beside it)");
    std::vector<uint64_t> coff(n_pairs + 1);
    saln_nw_cigar_offsets(g.p, coff.data());
    uint64_t cig_words = coff[n_pairs];
    TRY_HIP(dr.alloc(n_pairs * sizeof(saln_nw_result)));
    TRY_HIP(dc.alloc(cig_words * 4));
    up.join();
    TRY_HIP(up_err);
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
    // the context's pinned staging: held until the scatter below has read it
    std::unique_lock<std::mutex> stage_lk(ctx->staging_mu, std::defer_lock);
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
        stage_lk.lock();
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

// Rendered reference text of a batch (saln_nw_render_batch).
struct saln_nw_text {
    std::vector<std::string> text;  // the host-DFS pairs' text
    // the GPU-decided pairs' text, back to back in pair order: pair k's at
    // arena + aoff[k] (aoff[k] == kNoArena: in text[k])
    static constexpr uint64_t kNoArena = ~0ull;
    char *arena = nullptr;
    std::vector<uint64_t> aoff, alen;
    ~saln_nw_text() { std::free(arena); }
    std::vector<uint64_t> blocks, ns;
    std::vector<int32_t> status;
    std::vector<saln_nw_result> res;
    uint64_t count = 0;  // pairs rendered
    uint64_t gpu_decided = 0;  // of them rendered from the GPU's walk alone (no host DFS)
};

extern "C" {

// The pair loop main.rs:61-74 with the text n_w_align prints
// (needleman_wunsch_affine.rs:281-286, :390-411) for every pair, computed
// once: one full-code plan for the batch (fill + first walk on the GPU).  The
// GPU also decides what the reference DFS meets after each pair's first
// printed alignment (plan_next_event).  A pair whose text that decides - no
// block (the first event is the panic, or nothing), exactly one block, or
// under max_blocks = 1 the first block followed by a second block (the cap)
// or a panic - is rendered from its CIGAR: no parent codes cross PCIe for it
// and no host DFS runs.  The other pairs (more co-optimal alignments than the
// cap allows to skip, sentinel-rooted subtrees) run the reference DFS on host
// threads over their parent codes, downloaded for those pairs only.
namespace {

// One block of reference text from a first printed alignment (CIGAR words,
// forward): TraceBackInfo Display, needleman_wunsch_affine.rs:390-411.
constexpr char kBlockHead[] = "alignment found\n\nseq1: ", kBlockMid[] = "\n      ",
               kBlockTail[] = "\nseq2: ";
constexpr uint64_t kBlockFixed = sizeof(kBlockHead) + sizeof(kBlockMid) + sizeof(kBlockTail) - 2;

// the alignment's length (columns) from its CIGAR words
uint64_t cigar_columns(const uint32_t *w, uint32_t n) {
    uint64_t L = 0;
    for (uint32_t k = 0; k < n; ++k) L += w[k] >> 4;
    return L;
}

// One block of reference text from a first printed alignment of L columns
// (CIGAR words, forward) into out[0, kBlockFixed + 3 L): TraceBackInfo
// Display, needleman_wunsch_affine.rs:390-411.
void block_from_cigar(const uint8_t *q, const uint8_t *d, const uint32_t *w, uint32_t n,
                      uint64_t L, char *out) {
    constexpr size_t nh = sizeof(kBlockHead) - 1, nm = sizeof(kBlockMid) - 1,
                     nt = sizeof(kBlockTail) - 1;
    char *a = out;
    std::memcpy(a, kBlockHead, nh);
    a += nh;
    char *bars = a + L + nm, *c = bars + L + nt;
    std::memcpy(a + L, kBlockMid, nm);
    std::memcpy(bars + L, kBlockTail, nt);
    c[L] = '\n';
    uint64_t i = 0, j = 0, x = 0;  // db, query, column positions
    for (uint32_t k = 0; k < n; ++k) {
        const uint32_t len = w[k] >> 4, op = w[k] & 15u;
        // (a bar wherever the two printed chars are equal, a '-' byte in a
        // sequence against a gap included, as the reference's Display does)
        if (op == SALN_CIGAR_I) {  // query chars against gaps
            std::memcpy(a + x, q + j, len);
            std::memset(c + x, '-', len);
            for (uint32_t y = 0; y < len; ++y) bars[x + y] = q[j + y] == '-' ? '|' : ' ';
            j += len;
        } else if (op == SALN_CIGAR_D) {
            std::memset(a + x, '-', len);
            std::memcpy(c + x, d + i, len);
            for (uint32_t y = 0; y < len; ++y) bars[x + y] = d[i + y] == '-' ? '|' : ' ';
            i += len;
        } else {
            std::memcpy(a + x, q + j, len);
            std::memcpy(c + x, d + i, len);
            for (uint32_t y = 0; y < len; ++y) bars[x + y] = q[j + y] == d[i + y] ? '|' : ' ';
            i += len;
            j += len;
        }
        x += len;
    }
}

// work items [0, n) on up to 16 host threads, handed out in blocks of `grain`
void host_parallel(uint64_t n, uint64_t grain, const std::function<void(uint64_t)> &f) {
    const uint64_t nt = std::min<uint64_t>(std::max(1u, std::min(16u, std::thread::hardware_concurrency())),
                                           n / grain + 1);
    std::atomic<uint64_t> next{0};
    auto work = [&]() {
        for (;;) {
            const uint64_t b = next.fetch_add(grain);
            if (b >= n) return;
            for (uint64_t k = b; k < std::min(n, b + grain); ++k) f(k);
        }
    };
    std::vector<std::thread> th;
    for (uint64_t i = 1; i < nt; ++i) th.emplace_back(work);
    work();
    for (auto &x : th) x.join();
}

}  // namespace

int saln_nw_render_batch(saln_context *ctx, const uint8_t *q_seq, const uint64_t *q_off,
                         uint64_t n_q, const uint8_t *db_seq, const uint64_t *db_off,
                         uint64_t n_db, const uint32_t *pair_q, const uint32_t *pair_db,
                         uint64_t n_pairs, int32_t mode, uint64_t max_blocks, int stop_at_panic,
                         saln_nw_text **out) {
    if (!ctx || !q_off || !db_off || !out) return SALN_E_INVALID;
    *out = nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    auto *t = new saln_nw_text;
    t->text.resize(n_pairs);
    t->blocks.assign(n_pairs, 0);
    t->ns.assign(n_pairs, 0);
    t->status.assign(n_pairs, SALN_OK);
    t->res.resize(n_pairs);
    if (mode != SALN_MODE_GLOBAL) {  // needleman_wunsch_affine.rs:433-434: every pair errs
        for (uint64_t k = 0; k < n_pairs; ++k) {
            std::memset(&t->res[k], 0, sizeof(saln_nw_result));
            t->res[k].status = t->status[k] = SALN_NOT_IMPLEMENTED;
        }
        t->count = n_pairs;
        *out = t;
        return SALN_OK;
    }
    PlanGuard g;
    int rc = plan_create(ctx, q_off, n_q, db_off, n_db, pair_q, pair_db, n_pairs, mode, nullptr,
                         true, &g.p);
    if (rc != SALN_OK) {
        delete t;
        return rc;
    }
    StageClock clock(ctx->opts.effective());
    auto fail = [&](hipError_t e, const char *what) {
        set_error(std::string(what) + ": " + hipGetErrorString(e));
        delete t;
        return SALN_E_HIP;
    };
    std::vector<uint64_t> coff(n_pairs + 1), doff(n_pairs + 1, 0);
    std::vector<uint32_t> hcig;    // every pair's first alignment, packed (doff)
    std::vector<uint8_t> next(n_pairs, kNextHost);
    {
        DevBuf dq(ctx), dd(ctx), dr(ctx), dc(ctx), dnx(ctx), dso(ctx), ddo(ctx), dcd(ctx);
        const uint64_t qbytes = q_off[n_q], dbytes = db_off[n_db];
        saln_nw_cigar_offsets(g.p, coff.data());
        hipError_t e;
        if ((e = dq.alloc(qbytes)) != hipSuccess || (e = dd.alloc(dbytes)) != hipSuccess ||
            (e = dr.alloc(n_pairs * sizeof(saln_nw_result))) != hipSuccess ||
            (e = dc.alloc(std::max<uint64_t>(1, coff[n_pairs]) * 4)) != hipSuccess ||
            (e = dnx.alloc(std::max<uint64_t>(1, n_pairs))) != hipSuccess)
            return fail(e, "render batch: device buffers");
        if ((qbytes && (e = hipMemcpy(dq.p, q_seq, qbytes, hipMemcpyHostToDevice)) != hipSuccess) ||
            (dbytes && (e = hipMemcpy(dd.p, db_seq, dbytes, hipMemcpyHostToDevice)) != hipSuccess))
            return fail(e, "render batch: upload");
        clock.mark("render: plan + upload");
        rc = saln_nw_execute(g.p, (const uint8_t *)dq.p, (const uint8_t *)dd.p,
                             (saln_nw_result *)dr.p, (uint32_t *)dc.p, ctx->stream);
        if (rc == SALN_OK)
            rc = plan_next_event(g.p, (const saln_nw_result *)dr.p, (uint8_t *)dnx.p, ctx->stream);
        if (rc == SALN_OK && (e = hipStreamSynchronize(ctx->stream)) != hipSuccess)
            return fail(e, "execute");
        clock.mark("render: execute");
        if (rc == SALN_OK) rc = plan_check_error(g.p);
        if (rc != SALN_OK) {
            delete t;
            return rc;
        }
        if (n_pairs && ((e = hipMemcpy(t->res.data(), dr.p, n_pairs * sizeof(saln_nw_result),
                                       hipMemcpyDeviceToHost)) != hipSuccess ||
                        (e = hipMemcpy(next.data(), dnx.p, n_pairs, hipMemcpyDeviceToHost)) != hipSuccess))
            return fail(e, "render batch: results");
        // first alignments: packed densely on the device, one download
        for (uint64_t k = 0; k < n_pairs; ++k) doff[k + 1] = doff[k] + t->res[k].cigar_len;
        hcig.resize(doff[n_pairs]);
        if (doff[n_pairs]) {
            if ((e = dso.alloc((n_pairs + 1) * 8)) != hipSuccess ||
                (e = ddo.alloc((n_pairs + 1) * 8)) != hipSuccess ||
                (e = dcd.alloc(doff[n_pairs] * 4)) != hipSuccess ||
                (e = hipMemcpy(dso.p, coff.data(), (n_pairs + 1) * 8, hipMemcpyHostToDevice)) != hipSuccess ||
                (e = hipMemcpy(ddo.p, doff.data(), (n_pairs + 1) * 8, hipMemcpyHostToDevice)) != hipSuccess ||
                (e = launch_cigar_compact((const saln_nw_result *)dr.p, (const uint64_t *)dso.p,
                                          (const uint64_t *)ddo.p, (const uint32_t *)dc.p,
                                          (uint32_t *)dcd.p, n_pairs, ctx->stream)) != hipSuccess ||
                (e = hipStreamSynchronize(ctx->stream)) != hipSuccess ||
                (e = hipMemcpy(hcig.data(), dcd.p, doff[n_pairs] * 4, hipMemcpyDeviceToHost)) != hipSuccess)
                return fail(e, "render batch: alignments");
        }
    }
    clock.mark("render: results");
    // with stop_at_panic, pairs after the first panicking one are never
    // rendered: the reference aborts there (exit 101)
    uint64_t n = n_pairs;
    if (stop_at_panic)
        for (uint64_t k = 0; k < n_pairs; ++k)
            if (t->res[k].status == SALN_REF_PANIC_BOUNDARY) {
                n = k + 1;
                break;
            }
    const double dev_ns =
        (double)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0)
            .count();
    // the GPU-decided pairs (rendered from their CIGARs on host threads); the
    // rest go to the host DFS
    std::vector<uint64_t> host, dec;
    for (uint64_t k = 0; k < n; ++k) {
        const saln_nw_result &r = t->res[k];
        if (!r.printed) {  // the first DFS event is the panic, or every end state is dead
            t->status[k] = r.status == SALN_REF_PANIC_BOUNDARY ? SALN_REF_PANIC_BOUNDARY : SALN_OK;
            continue;
        }
        const uint8_t nx = next[k];
        const bool one = nx == kNextNone;
        const bool capped = max_blocks == 1 && (nx == kNextBlock || nx == kNextPanic);
        if (!one && !capped) {
            host.push_back(k);
            continue;
        }
        t->blocks[k] = 1;
        t->status[k] = one ? SALN_OK : nx == kNextBlock ? SALN_ENUM_CAP : SALN_REF_PANIC_BOUNDARY;
        dec.push_back(k);
    }
    // their text sizes, offsets in the arena, then the text, on host threads
    // (one arena: ~0.5 KB per configs[1] pair without an allocation each)
    const uint64_t nd = dec.size();
    t->aoff.assign(n_pairs, saln_nw_text::kNoArena);
    t->alen.assign(n_pairs, 0);
    std::vector<uint64_t> cols(nd);
    host_parallel(nd, 1024, [&](uint64_t x) {
        const uint64_t k = dec[x];
        cols[x] = cigar_columns(hcig.data() + doff[k], t->res[k].cigar_len);
    });
    uint64_t asz = 0;
    for (uint64_t x = 0; x < nd; ++x) {
        const uint64_t k = dec[x];
        t->aoff[k] = asz;
        t->alen[k] = kBlockFixed + 3 * cols[x];
        asz += t->alen[k];
    }
    if (asz) {
        constexpr size_t kHuge = size_t(2) << 20;
        const size_t want = (asz + kHuge - 1) / kHuge * kHuge;
        void *hp = nullptr;
        if (posix_memalign(&hp, kHuge, want) != 0 || !hp) {
            set_error("render batch: text buffer allocation failed");
            delete t;
            return SALN_E_HIP;
        }
        (void)madvise(hp, want, MADV_HUGEPAGE);  // advisory: fewer first-touch faults
        t->arena = (char *)hp;
    }
    host_parallel(nd, 256, [&](uint64_t x) {
        const uint64_t k = dec[x];
        const auto a = std::chrono::steady_clock::now();
        const uint64_t qi = pair_q ? pair_q[k] : k % n_q, di = pair_db ? pair_db[k] : k / n_q;
        block_from_cigar(q_seq + q_off[qi], db_seq + db_off[di], hcig.data() + doff[k],
                         t->res[k].cigar_len, cols[x], t->arena + t->aoff[k]);
        t->ns[k] = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                       std::chrono::steady_clock::now() - a).count();
    });
    clock.mark("render: gpu-decided");
    if (!host.empty()) {
        // their parent codes: the workspace prefix the last of them needs,
        // streamed in slices while the DFS threads render the pairs in the
        // order their bytes arrive (the download and the host work overlap)
        const uint8_t *d_mask = nullptr;
        if ((rc = plan_mask_source(g.p, &d_mask)) != SALN_OK) {
            delete t;
            return rc;
        }
        const uint64_t nh = host.size();
        std::vector<uint64_t> endb(nh);
        uint64_t total = 0;
        for (uint64_t x = 0; x < nh; ++x) {
            endb[x] = plan_mask_end(g.p, host[x]);
            total = std::max(total, endb[x]);
        }
        std::vector<uint64_t> order(nh);
        std::iota(order.begin(), order.end(), 0);
        std::sort(order.begin(), order.end(), [&](uint64_t x, uint64_t y) { return endb[x] < endb[y]; });
        // the context's host buffer is taken out under staging_mu and handed
        // back after the DFS, so the lock is not held while the pairs render
        saln_context::HostBuf hb;
        {
            std::lock_guard<std::mutex> lk(ctx->staging_mu);
            std::swap(hb.p, ctx->host_mask.p);
            std::swap(hb.n, ctx->host_mask.n);
        }
        auto give_back = [&]() {
            std::lock_guard<std::mutex> lk(ctx->staging_mu);
            if (hb.n > ctx->host_mask.n) {
                std::swap(hb.p, ctx->host_mask.p);
                std::swap(hb.n, ctx->host_mask.n);
            }
        };  // (hb frees whichever buffer it holds last)
        if (total > hb.n) {
            std::free(hb.p);
            hb.p = nullptr;
            hb.n = 0;
            constexpr size_t kHuge = size_t(2) << 20;
            const size_t want = (total + kHuge - 1) / kHuge * kHuge;
            void *hp = nullptr;
            if (posix_memalign(&hp, kHuge, want) != 0 || !hp) {
                set_error("render batch: host mask buffer allocation failed");
                delete t;
                return SALN_E_HIP;
            }
            (void)madvise(hp, want, MADV_HUGEPAGE);  // advisory: 4 KB pages if THP is off
            hb.p = (uint8_t *)hp;
            hb.n = want;
        }
        uint8_t *hbuf = hb.p;
        constexpr uint64_t kSlice = 32ull << 20;
        std::atomic<uint64_t> have{0};
        std::atomic<int> dl_err{0};
        std::thread dl([&] {
            hipError_t e = hipSetDevice(ctx->device);
            for (uint64_t off = 0; e == hipSuccess && off < total; off += kSlice) {
                const uint64_t len = std::min(kSlice, total - off);
                e = hipMemcpy(hbuf + off, d_mask + off, len, hipMemcpyDeviceToHost);
                if (e == hipSuccess) have.store(off + len, std::memory_order_release);
            }
            if (e != hipSuccess) dl_err.store((int)e, std::memory_order_release);  // (errors are per thread)
        });
        // per-pair DFS on host threads (its cost varies by orders of magnitude
        // with the number of co-optimal paths: pairs are handed out one by one)
        std::atomic<uint64_t> nxt{0};
        auto work = [&]() {
            for (;;) {
                const uint64_t x = nxt.fetch_add(1);
                if (x >= nh) return;
                const uint64_t k = host[order[x]];
                while (have.load(std::memory_order_acquire) < endb[order[x]]) {
                    if (dl_err.load(std::memory_order_acquire)) return;
                    std::this_thread::yield();
                }
                const auto a = std::chrono::steady_clock::now();
                const uint64_t qi = pair_q ? pair_q[k] : k % n_q, di = pair_db ? pair_db[k] : k / n_q;
                const HostMask hm = plan_host_mask(g.p, hbuf, k);
                const DfsOutcome o = render_blocks(hm, q_seq + q_off[qi], db_seq + db_off[di],
                                                   max_blocks, &t->text[k]);
                t->blocks[k] = o.blocks;
                t->status[k] = o.status;
                t->ns[k] = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                               std::chrono::steady_clock::now() - a).count();
            }
        };
        const uint64_t nt = std::min<uint64_t>(std::max(1u, std::min(16u, std::thread::hardware_concurrency())),
                                               nh / 64 + 1);
        std::vector<std::thread> th;
        for (uint64_t i = 1; i < nt; ++i) th.emplace_back(work);
        work();
        for (auto &x : th) x.join();
        dl.join();
        give_back();
        if (const int e = dl_err.load()) {
            set_error(std::string("render batch: mask download: ") + hipGetErrorString((hipError_t)e));
            delete t;
            return SALN_E_HIP;
        }
    }
    clock.mark("render: masks + dfs");
    // each pair's share of the batch's device work, added to its own host time
    for (uint64_t k = 0; k < n; ++k) t->ns[k] += (uint64_t)(dev_ns / (double)std::max<uint64_t>(1, n_pairs));
    t->gpu_decided = n - host.size();
    t->count = n;
    *out = t;
    return SALN_OK;
}

int saln_nw_render_text(saln_context *ctx, const uint8_t *q, uint64_t len_q, const uint8_t *d,
                        uint64_t len_db, int32_t mode, uint64_t max_blocks, saln_nw_text **out) {
    if (!ctx || (len_q && !q) || (len_db && !d) || !out) return SALN_E_INVALID;
    const uint64_t qo[2] = {0, len_q}, dof[2] = {0, len_db};
    const uint32_t z = 0;
    return saln_nw_render_batch(ctx, q, qo, 1, d, dof, 1, &z, &z, 1, mode, max_blocks, 0, out);
}

uint64_t saln_nw_text_count(const saln_nw_text *t) { return t ? t->count : 0; }
uint64_t saln_nw_text_gpu_decided(const saln_nw_text *t) { return t ? t->gpu_decided : 0; }

int saln_nw_text_get(const saln_nw_text *t, uint64_t pair, const char **text, uint64_t *len,
                     uint64_t *n_blocks, int32_t *status, saln_nw_result *result,
                     uint64_t *elapsed_ns) {
    if (!t || pair >= t->count) return SALN_E_INVALID;
    const bool ar = !t->aoff.empty() && t->aoff[pair] != saln_nw_text::kNoArena;
    if (text) *text = ar ? t->arena + t->aoff[pair] : t->text[pair].data();
    if (len) *len = ar ? t->alen[pair] : t->text[pair].size();
    if (n_blocks) *n_blocks = t->blocks[pair];
    if (status) *status = t->status[pair];
    if (result) *result = t->res[pair];
    if (elapsed_ns) *elapsed_ns = t->ns[pair];
    return SALN_OK;
}

void saln_nw_text_free(saln_nw_text *t) { delete t; }

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

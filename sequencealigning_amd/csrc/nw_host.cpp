// C ABI implementation for the NW-affine engine (include/saln.h).
//
// Replaces n_w_align (src/needleman_wunsch_affine.rs:424-437) and the
// db x query pair loop that calls it (src/main.rs:61-67).  All arithmetic
// runs in the HIP kernels of nw_kernels.hip; the host only plans batches,
// moves buffers and, for the reference's text output, walks the parent codes
// the GPU produced (the reference's exhaustive DFS, :281-329).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <array>
#include <cstring>
#include <map>
#include <numeric>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

#include <sys/mman.h>

#include "nw_host.hpp"

namespace saln {

static thread_local std::string g_err;
void set_error(const std::string &msg) { g_err = msg; }

Scoring scoring_or_default(const saln_nw_scoring *s) {
    if (!s) return Scoring{5, -4, -8, -6};  // SCHEME, needleman_wunsch_affine.rs:15-20
    return Scoring{s->match, s->mismatch, s->gap_open, s->gap_extend};
}

// The i32 fills carry V'' = 4V + 2a + p plus the position offsets alpha*r +
// beta*c (nw_common.hpp).  |V| is at most the sentinel plus one step's
// largest change per row and column of the path; a pair passes while that
// bound, scaled and offset, stays inside int32 (the reference's own i32
// arithmetic is exact far beyond it: the pairs rejected here are ~10^8 long
// or carry penalties of ~10^4).
bool scores_fit_i32(const Scoring &s, uint64_t lq, uint64_t ld) {
    auto a = [](int64_t v) { return v < 0 ? -v : v; };
    const int64_t step = std::max({a(s.match), a(s.mismatch), a(s.gap_open) + a(s.gap_extend)});
    const long double v = 32768.0L + (long double)(lq + ld) * (long double)step;
    const long double off = 4.0L * (a(s.match) + 2 * a(s.gap_extend)) * (long double)ld +
                            4.0L * a(s.gap_extend) * (long double)lq;
    return 4.0L * v + 3.0L + off < 2147483647.0L;
}

}  // namespace saln

using namespace saln;

// a plan's table-fill bail words per mask workspace: one per fill variant
constexpr size_t kBailBytes = kNumVariants * sizeof(uint32_t);

struct saln_nw_plan {
    saln_context *ctx = nullptr;
    Options opts{};  // the context's effective options at creation
    Scoring sc{};
    uint64_t n_pairs = 0;
    std::vector<NwPairDesc> h_pairs;  // plan order
    std::vector<uint32_t> plan_index;  // results index -> plan order
    NwPairDesc *d_pairs = nullptr;
    uint32_t var_first[kNumVariants] = {}, var_count[kNumVariants] = {};
    uint32_t var_maxld[kNumVariants] = {};  // longest db of each variant's pairs
    uint32_t n_fill = 0;  // plan order: [0, n_fill) filled pairs, then empty-side pairs
    uint8_t *d_mask = nullptr;
    uint8_t *d_mask2 = nullptr;  // second workspace for the async (2-deep) pipeline
    int32_t *d_endh2 = nullptr;
    bool async_tb = false;
    bool stripe_pk = false;  // column stripes use the packed fill and layout
    int stripe_rows = 0;     // else: row fill with this many columns per lane (0 = skewed fill)
    uint32_t stripe_sub = kStripeSubMax;  // boundary columns per 256-column chunk
    int stripe_layout() const { return stripe_pk ? 1 : stripe_rows ? 2 : 0; }
    bool full_codes = false;  // walk codes (default) or every parent set (decided at creation)
    bool nib[kNumVariants] = {};  // variant stores 4-bit walk codes (Geom::LBn segments)
    bool score_only = false;  // no parent codes / traceback (saln_nw_plan_set_score_only)
    int buf = 0;                           // workspace of the next execute (async mode)
    hipStream_t tb_stream = nullptr;       // traceback stream of async executes (NULL: ctx's)
    bool tb_pending[2] = {false, false};
    int last_buf = 0;
    uint64_t mask_bytes = 0;
    int2 *d_scratch = nullptr;
    // column-stripe pairs (kStripeVariant): work items (plan index, chunk),
    // per-pair first work item (plan order, n_pairs+1), progress counters
    uint2 *d_work = nullptr;
    std::vector<uint32_t> work_first;
    // d_err[0]: device error flags since the last saln_nw_plan_status (bit 0
    // a dependency wait timed out, bit 1 an unlinked speculative walk under
    // SALN_SPEC_STRICT); d_err[1]: the wait limit the fills read
    uint32_t *d_prog = nullptr, *d_err = nullptr;  // d_err: kErrWords (the row fill's XCD slots after the two)
    uint32_t fill_epoch = 0;  // stripe fills launched (the XCD slots' epochs)
    uint32_t wait_limit = kWaitLimitDefault;
    bool unchecked[2] = {false, false};  // executes on workspace b since the last status
    uint64_t n_prog = 0;
    uint32_t *d_ops = nullptr;  // traceback op-stream scratch of workspace 0
    uint32_t *d_ops2 = nullptr;  // ... of workspace 1 (async: its walks may overlap workspace 0's)
    uint64_t ops_words = 0;
    // per workspace: the table fills' bail word (zeroed once; a table launch
    // whose waves left pairs to its fallback launch stores its epoch there)
    uint32_t *d_bail[2] = {nullptr, nullptr};
    uint32_t epoch = 0;  // table launches of this plan (the bail word's values)
    // speculative stripe walks (a few long column-stripe pairs): block map,
    // pairs, stripe records, run words, per-pair done flags (plan order)
    uint32_t spec_pairs = 0, spec_blocks = 0;
    int spec_passes = 0;
    bool spec_strict = false;  // SALN_SPEC_STRICT=1: a pair left to the cooperative walker is an error
    uint2 *d_spec_blocks = nullptr;
    SpecPair *d_spec_pairs = nullptr;
    SpecStripe *d_spec_stripes = nullptr;
    uint32_t *d_spec_ops = nullptr, *d_spec_done = nullptr;
    uint64_t scratch_elems = 0;
    int32_t *d_endh = nullptr;
    std::vector<uint64_t> cigar_off;  // results order, n_pairs + 1
    uint64_t cells = 0;
    bool timing = false;
    // hipEvents around the fill and traceback launches of each execute;
    // resolved lazily (no host sync inside execute).
    std::vector<std::array<hipEvent_t, 4>> ev_pool;
    size_t ev_used = 0;
    std::map<std::string, std::pair<double, uint64_t>> ktime;
    int resolve_events();
    // the two events after the sub-batch events mark "traceback of workspace b done"
    hipEvent_t tb_done(int b) const { return sync_ev[1 + b]; }
    // fill -> traceback stream hand-off (async) and "traceback of workspace b
    // done" (two events)
    std::vector<hipEvent_t> sync_ev;
};

extern "C" {

const char *saln_last_error(void) { return g_err.c_str(); }
int saln_abi_version(void) { return SALN_ABI_VERSION; }

int saln_context_create(int device, saln_context **out) {
    if (!out) return SALN_E_INVALID;
    *out = nullptr;
    // host.prefault_mb: the host buffer of render batches' parent codes,
    // allocated and faulted in on a helper thread while the HIP runtime
    // starts (~0.2 s; the CLI's first full chunk otherwise faults ~0.4 GB in
    // during its mask download: 56 ms, round 6)
    saln_context::HostBuf pre;
    std::thread pre_th;
    if (const int64_t mb = opt(Opt::HostPrefaultMb); mb > 0) {
        pre_th = std::thread([&pre, mb] {
            constexpr size_t kHuge = size_t(2) << 20;
            const size_t want = (((size_t)mb << 20) + kHuge - 1) / kHuge * kHuge;
            void *hp = nullptr;
            if (posix_memalign(&hp, kHuge, want) != 0 || !hp) return;
            (void)madvise(hp, want, MADV_HUGEPAGE);
            std::memset(hp, 0, want);
            pre.p = (uint8_t *)hp;
            pre.n = want;
        });
    }
    struct Join {
        std::thread &t;
        ~Join() { if (t.joinable()) t.join(); }
    } join_pre{pre_th};
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) {
        set_error("no HIP device " + std::to_string(device) + " (saln has no CPU path)");
        return SALN_E_NO_DEVICE;
    }
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_error(std::string("device is ") + prop.gcnArchName + ", saln is built for gfx950");
        return SALN_E_NO_DEVICE;
    }
    HIP_TRY(hipSetDevice(device));
    auto *c = new saln_context;
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->tb_stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        set_error("hipStreamCreate failed");
        return SALN_E_HIP;
    }
    if (pre_th.joinable()) {
        pre_th.join();
        std::swap(c->host_mask.p, pre.p);
        std::swap(c->host_mask.n, pre.n);
    }
    *out = c;
    return SALN_OK;
}

int saln_context_destroy(saln_context *ctx) {
    if (!ctx) return SALN_OK;
    (void)hipSetDevice(ctx->device);
    (void)hipDeviceSynchronize();
    dev_cache_clear(ctx);
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->tb_stream) (void)hipStreamDestroy(ctx->tb_stream);
    delete ctx;
    return SALN_OK;
}

int saln_nw_plan_destroy(saln_nw_plan *p) {
    if (!p) return SALN_OK;
    (void)hipSetDevice(p->ctx->device);
    (void)hipDeviceSynchronize();  // the blocks go back to the context cache
    for (void *b : {(void *)p->d_pairs, (void *)p->d_mask, (void *)p->d_mask2, (void *)p->d_endh2,
                    (void *)p->d_scratch, (void *)p->d_work, (void *)p->d_prog, (void *)p->d_err,
                    (void *)p->d_ops, (void *)p->d_ops2, (void *)p->d_bail[0], (void *)p->d_bail[1],
                    (void *)p->d_endh, (void *)p->d_spec_blocks,
                    (void *)p->d_spec_pairs, (void *)p->d_spec_stripes, (void *)p->d_spec_ops,
                    (void *)p->d_spec_done})
        dev_free(p->ctx, b);
    for (auto &e : p->sync_ev) (void)hipEventDestroy(e);
    for (auto &t : p->ev_pool)
        for (auto &e : t) (void)hipEventDestroy(e);
    delete p;
    return SALN_OK;
}

int saln_nw_plan_create(saln_context *ctx, const uint64_t *q_off, uint64_t n_q,
                        const uint64_t *db_off, uint64_t n_db, const uint32_t *pair_q,
                        const uint32_t *pair_db, uint64_t n_pairs, int32_t mode,
                        const saln_nw_scoring *scoring, saln_nw_plan **out) {
    return saln::plan_create(ctx, q_off, n_q, db_off, n_db, pair_q, pair_db, n_pairs, mode,
                             scoring, false, out);
}

int saln_nw_plan_create_full(saln_context *ctx, const uint64_t *q_off, uint64_t n_q,
                             const uint64_t *db_off, uint64_t n_db, const uint32_t *pair_q,
                             const uint32_t *pair_db, uint64_t n_pairs, int32_t mode,
                             const saln_nw_scoring *scoring, saln_nw_plan **out) {
    return saln::plan_create(ctx, q_off, n_q, db_off, n_db, pair_q, pair_db, n_pairs, mode,
                             scoring, true, out);
}

int saln_nw_plan_dense_mask(saln_nw_plan *p, uint64_t pair, uint8_t *out) {
    if (!p || !out || pair >= p->n_pairs) return SALN_E_INVALID;
    if (p->async_tb) {  // the mask of the last execute may sit in either workspace
        set_error("saln_nw_plan_dense_mask: synchronous plans only");
        return SALN_E_INVALID;
    }
    HIP_TRY(hipSetDevice(p->ctx->device));
    for (int b = 0; b < 2; ++b)
        if (p->tb_pending[b]) HIP_TRY(hipEventSynchronize(p->tb_done(b)));
    saln::PairMask pm;
    const int rc = saln::plan_pair_mask(p, pair, &pm);
    if (rc != SALN_OK) return rc;
    const NwPairDesc &d = p->h_pairs[p->plan_index[pair]];
    const saln::HostMask hm(pm, d.len_q, d.len_db, p->sc);
    hm.to_dense(out);
    return SALN_OK;
}

int saln_nw_plan_walk_codes(saln_nw_plan *p, uint64_t pair, uint8_t *out) {
    if (!p || !out || pair >= p->n_pairs) return SALN_E_INVALID;
    if (p->async_tb) {
        set_error("saln_nw_plan_walk_codes: synchronous plans only");
        return SALN_E_INVALID;
    }
    const NwPairDesc &d = p->h_pairs[p->plan_index[pair]];
    if (d.variant >= (uint32_t)kNumVariants || !p->nib[d.variant] || !d.len_q || !d.len_db) {
        set_error("saln_nw_plan_walk_codes: the pair's fill stores no 4-bit walk codes");
        return SALN_E_INVALID;
    }
    HIP_TRY(hipSetDevice(p->ctx->device));
    for (int b = 0; b < 2; ++b)
        if (p->tb_pending[b]) HIP_TRY(hipEventSynchronize(p->tb_done(b)));
    // segments of block b at row i: mask_off + (i-1) rs + b bs (Geom::LBn
    // bytes; column c's nibble at bit nib_bit(c) of dword c / 8)
    const Geom g = variant_geom((int)d.variant);
    // every block of each row (rs / bs of them: the pack's width) as one
    // bs-pitched 2-D region of LBn-byte rows
    const uint64_t per_row = d.mask_rs / d.mask_bs;
    std::vector<uint8_t> all((uint64_t)d.len_db * per_row * g.LBn());
    HIP_TRY(hipMemcpy2D(all.data(), g.LBn(), p->d_mask + d.mask_off, d.mask_bs, g.LBn(),
                        (uint64_t)d.len_db * per_row, hipMemcpyDeviceToHost));
    for (uint32_t i = 1; i <= d.len_db; ++i)
        for (uint32_t j = 1; j <= d.len_q; ++j) {
            const uint32_t b = (j - 1) / g.K, c = (j - 1) % g.K;
            const uint8_t *sp = all.data() + ((uint64_t)(i - 1) * per_row + b) * g.LBn();
            uint32_t w;
            std::memcpy(&w, sp + 4 * (c >> 3), 4);
            const uint32_t bit = ((c & 4u) << 2) | ((c & 1u) << 3) | ((c & 2u) << 1);
            out[(uint64_t)(i - 1) * d.len_q + (j - 1)] = (uint8_t)((w >> bit) & 15u);
        }
    return SALN_OK;
}

}  // extern "C"

// Plan creation.  full_codes: the fills store every parent set (host DFS,
// dense mask) instead of walk codes; it fixes the mask layout (4-bit walk
// codes for the short-query packed variants, bytes otherwise).
int saln::plan_create(saln_context *ctx, const uint64_t *q_off, uint64_t n_q,
                      const uint64_t *db_off, uint64_t n_db, const uint32_t *pair_q,
                      const uint32_t *pair_db, uint64_t n_pairs, int32_t mode,
                      const saln_nw_scoring *scoring, bool full_codes, saln_nw_plan **out) {
    if (!ctx || !q_off || !db_off || !out) return SALN_E_INVALID;
    *out = nullptr;
    if (mode != SALN_MODE_GLOBAL) {
        set_error("not implemented");  // needleman_wunsch_affine.rs:433-434
        return SALN_NOT_IMPLEMENTED;
    }
    if ((pair_q == nullptr) != (pair_db == nullptr)) return SALN_E_INVALID;
    if (!pair_q && n_pairs != n_q * n_db) {
        set_error("all-vs-all needs n_pairs == n_q * n_db");
        return SALN_E_INVALID;
    }
    if (n_pairs > 0xFFFFFFFFull) return SALN_E_INVALID;
    HIP_TRY(hipSetDevice(ctx->device));
    const Options opts = ctx->opts.effective();
    StageClock clk(opts);
    auto *p = new saln_nw_plan;
    p->ctx = ctx;
    p->opts = opts;
    p->sc = scoring_or_default(scoring);
    p->full_codes = full_codes;
    // 4-bit walk codes for the short-query packed variants: 8 x 19 groups for
    // queries of <= 152 columns, 16 x 10 up to 160; full-code plans keep byte
    // codes and the 16 x 10 groups
    const bool nib_on = !full_codes;
    const bool narrow = nib_on;
    for (int v = 0; v < kNumVariants; ++v) p->nib[v] = nib_on && variant_nib(v);
    p->n_pairs = n_pairs;
    p->cigar_off.resize(n_pairs + 1);
    std::vector<NwPairDesc> descs(n_pairs);
    uint64_t cig = 0;
    // the range check and the variant depend on the shape only: batches of
    // alike pairs (the usual case) decide once per shape, not per pair
    uint64_t memo_lq = ~0ull, memo_ld = ~0ull;
    bool memo_fit = false;
    int memo_var = 0;
    for (uint64_t k = 0; k < n_pairs; ++k) {
        const uint64_t qi = pair_q ? pair_q[k] : k % n_q;
        const uint64_t di = pair_db ? pair_db[k] : k / n_q;
        if (qi >= n_q || di >= n_db) {
            delete p;
            set_error("pair index out of range");
            return SALN_E_INVALID;
        }
        NwPairDesc &d = descs[k];
        std::memset(&d, 0, sizeof(d));
        d.q_off = q_off[qi];
        d.db_off = db_off[di];
        const uint64_t lq = q_off[qi + 1] - q_off[qi], ld = db_off[di + 1] - db_off[di];
        if (lq > 0x7FFFFFFFull || ld > 0x7FFFFFFFull) {
            delete p;
            set_error("sequence too long");
            return SALN_E_INVALID;
        }
        if (lq != memo_lq || ld != memo_ld) {
            memo_lq = lq;
            memo_ld = ld;
            memo_fit = scores_fit_i32(p->sc, lq, ld);
            memo_var = memo_fit ? choose_variant((uint32_t)lq, (uint32_t)ld, p->sc, narrow) : 0;
        }
        if (!memo_fit) {
            delete p;
            set_error("pair too long for these penalties: its scores could leave the engine's "
                      "int32 range");
            return SALN_E_INVALID;
        }
        d.len_q = (uint32_t)lq;
        d.len_db = (uint32_t)ld;
        d.pair_id = (uint32_t)k;
        d.variant = (uint32_t)memo_var;
        d.cigar_off = cig;
        p->cigar_off[k] = cig;
        cig += lq + ld;
        p->cells += lq * ld;
    }
    p->cigar_off[n_pairs] = cig;
    clk.mark("plan: descs");
    {
        // Queries of 513-1,024 columns: the 64-lane packed variant is the
        // throughput choice (two pairs per wave), the column stripes the
        // latency choice (four waves per pair, pipelined): a plan with few
        // such pairs keeps them on stripes.
        const uint64_t v8_min = (uint64_t)opts[Opt::WideMinPairs];
        uint64_t wide = 0;
        for (const NwPairDesc &d : descs)
            wide += d.variant == (uint32_t)kWidePackedVariant && d.len_q > 512;
        if (wide && wide < v8_min)
            for (NwPairDesc &d : descs)
                if (d.variant == (uint32_t)kWidePackedVariant && d.len_q > 512)
                    d.variant = (uint32_t)kStripeVariant;
    }
    // plan order: fill pairs grouped by variant, then by query chunk count,
    // longest db first (balances the groups of a block and keeps the pairs of
    // a mask pack alike); pairs with an empty side last (traceback only).
    // (variant, ~chunks, ~len_db) packed in one word, ties by results index;
    // a batch of alike pairs is usually in order already
    std::vector<uint64_t> skey(n_pairs);
    for (uint64_t k = 0; k < n_pairs; ++k) {
        const NwPairDesc &d = descs[k];
        const bool empty = d.len_q == 0 || d.len_db == 0;
        const uint64_t nch = empty ? 0 : variant_geom((int)d.variant).n_chunks(d.len_q);
        skey[k] = (uint64_t)(empty ? (uint32_t)kNumVariants : d.variant) << 56 |
                  ((~nch) & 0xFFFFFFull) << 32 | (uint32_t)~d.len_db;
    }
    std::vector<uint32_t> order;
    const bool in_order = std::is_sorted(skey.begin(), skey.end());
    if (in_order) {
        p->h_pairs = std::move(descs);  // plan order = results order: no copy
    } else {
        order.resize(n_pairs);
        std::iota(order.begin(), order.end(), 0u);
        std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
            return skey[a] != skey[b] ? skey[a] < skey[b] : a < b;
        });
        p->h_pairs.resize(n_pairs);
    }
    clk.mark("plan: sort");
    uint64_t soff = 0, ooff = 0;
    for (uint64_t r = 0; r < n_pairs; ++r) {
        NwPairDesc d = in_order ? p->h_pairs[r] : descs[order[r]];
        const bool empty = d.len_q == 0 || d.len_db == 0;
        if (!empty) {
            const Geom g = variant_geom((int)d.variant);
            d.ops_off = ooff;
            ooff += (d.len_q + d.len_db + 9) / 10 + 1;  // 3-bit ops, ten per word
            if (g.n_chunks(d.len_q) > 1 || d.variant == kStripeVariant) {
                soff = (soff + 3) & ~3ull;  // 32-byte aligned columns (nw_fill_rows_kernel)
                d.scratch_off = soff;
                // stripes run concurrently: one boundary column per chunk boundary
                soff += (uint64_t)(d.variant == kStripeVariant ? kStripeSubMax * g.n_chunks(d.len_q)
                                                                : 1) *
                        scratch_col(d.len_db);
            }
            if (p->var_count[d.variant] == 0) p->var_first[d.variant] = (uint32_t)r;
            p->var_count[d.variant]++;
            p->var_maxld[d.variant] = std::max(p->var_maxld[d.variant], d.len_db);
            p->n_fill++;
        }
        p->h_pairs[r] = d;
    }
    {
        uint64_t waves = 0, cols = 0, waves_k1 = 0;  // 256-column chunks, columns, 64-column stripes
        bool free_all = true;  // the packed stripes carry no alive flag (nw_common.hpp)
        for (uint32_t r = 0; r < p->var_count[kStripeVariant]; ++r) {
            const NwPairDesc &d = p->h_pairs[p->var_first[kStripeVariant] + r];
            waves += variant_geom(kStripeVariant).n_chunks(d.len_q);
            waves_k1 += (d.len_q + 63) / 64;
            cols += d.len_q;
            free_all = free_all && sentinel_free(p->sc, d.len_q, d.len_db);
        }
        // packed stripes (int16x2, throughput) for batches of wide pairs; the
        // row fill (i32, latency) otherwise: 400 x 2 kbp^2 828 vs 678 GCUPS,
        // 400 x 5 kbp^2 953 vs 1,204 (one box, round 2)
        const bool wide = p->var_count[kStripeVariant] &&
                          cols / p->var_count[kStripeVariant] >= 3000;
        p->stripe_pk = waves > 0 && free_all && stripe_packed(p->sc, waves, wide, opts);
        p->stripe_rows = p->stripe_pk ? 0 : stripe_rows_k(waves_k1, opts);
        // boundary columns per 256-column chunk: the row fill's 4 / K stripes,
        // else one; the scratch offsets above reserved kStripeSubMax
        p->stripe_sub = p->stripe_rows ? 4u / (uint32_t)p->stripe_rows : 1u;
        if (p->stripe_sub != kStripeSubMax) {
            uint64_t so = 0;
            for (uint64_t r = 0; r < p->n_fill; ++r) {
                NwPairDesc &d = p->h_pairs[r];
                const Geom g = variant_geom((int)d.variant);
                if (g.n_chunks(d.len_q) > 1 || d.variant == kStripeVariant) {
                    so = (so + 3) & ~3ull;
                    d.scratch_off = so;
                    so += (uint64_t)(d.variant == kStripeVariant ? p->stripe_sub * g.n_chunks(d.len_q) : 1) *
                          scratch_col(d.len_db);
                }
            }
            soff = so;
        }
    }
    // Mask packs: up to 64 consecutive pairs of a variant (one traceback
    // wave) with interleaved segments (nw_common.hpp Geom), unless padding
    // them to the pack's longest db / widest query would cost over 25 % more
    // than storing them apart.
    uint64_t moff = 0;
    for (int v = 0; v < kNumVariants; ++v) {
        const Geom g = variant_geom(v);
        const uint64_t lb = p->nib[v] ? g.LBn() : g.LB();
        for (uint32_t a = p->var_first[v], e = a + p->var_count[v]; a < e; a += 64) {
            const uint32_t np = std::min<uint32_t>(64, e - a);
            uint64_t rows = 0, nbm = 0, own = 0;
            for (uint32_t s = 0; s < np; ++s) {
                const NwPairDesc &d = p->h_pairs[a + s];
                rows = std::max<uint64_t>(rows, d.len_db);
                nbm = std::max<uint64_t>(nbm, g.n_blocks(d.len_q));
                own += (uint64_t)d.len_db * g.n_blocks(d.len_q) * lb;
            }
            const uint64_t packed = rows * nbm * np * lb;
            if (v == kStripeVariant) {
                // one region per 256-column chunk: the row fill's unskewed
                // 256-column tiles (bs = 4), or the packed stripes' skewed
                // lines (bs = 0: every fill step writes one whole line)
                const bool pk = p->stripe_pk;
                for (uint32_t s = 0; s < np; ++s) {
                    NwPairDesc &d = p->h_pairs[a + s];
                    d.mask_off = moff;
                    d.mask_rs = g.W();
                    d.mask_bs = pk ? 0u : (uint32_t)lb;
                    d.mask_cs = ((uint64_t)d.len_db + (pk ? 2 * g.G : g.G) - 1) * g.W();
                    moff += g.n_chunks(d.len_q) * d.mask_cs;
                }
            } else if (4 * packed <= 5 * own + 4096) {
                for (uint32_t s = 0; s < np; ++s) {
                    NwPairDesc &d = p->h_pairs[a + s];
                    d.mask_off = moff + s * lb;
                    d.mask_bs = (uint32_t)(np * lb);
                    d.mask_rs = nbm * np * lb;
                    d.mask_cs = (uint64_t)g.G * d.mask_bs;
                }
                moff += (packed + 255) & ~255ull;
            } else {
                for (uint32_t s = 0; s < np; ++s) {
                    NwPairDesc &d = p->h_pairs[a + s];
                    d.mask_off = moff;
                    d.mask_bs = (uint32_t)lb;
                    d.mask_rs = g.n_blocks(d.len_q) * lb;
                    d.mask_cs = (uint64_t)g.G * lb;
                    moff += ((uint64_t)d.len_db * d.mask_rs + 255) & ~255ull;
                }
            }
        }
    }
    {
        p->sync_ev.resize(3);
        for (auto &e : p->sync_ev) {
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
                e = nullptr;
                set_error("hipEventCreate");
                saln_nw_plan_destroy(p);
                return SALN_E_HIP;
            }
        }
    }
    clk.mark("plan: layout");
    p->plan_index.resize(n_pairs);
    for (uint64_t r = 0; r < n_pairs; ++r) p->plan_index[p->h_pairs[r].pair_id] = (uint32_t)r;
    p->mask_bytes = moff;
    p->scratch_elems = soff;
    auto fail = [&](hipError_t e, const char *what) {
        set_error(std::string(what) + ": " + hipGetErrorString(e));
        saln_nw_plan_destroy(p);
        return SALN_E_HIP;
    };
    hipError_t e;
    if (n_pairs) {
        if ((e = dev_alloc(p->ctx, (void **)&p->d_pairs, n_pairs * sizeof(NwPairDesc))) != hipSuccess)
            return fail(e, "hipMalloc(pairs)");
        clk.mark("plan: pairs alloc");
        // through the context's pinned staging: a pageable copy of a freshly
        // built array pins its pages first (measured 12-17 ms for the 2.7-5.2
        // MB of a render chunk's descriptors, against ~1 ms of memcpy here)
        {
            std::lock_guard<std::mutex> lk(p->ctx->staging_mu);
            void *st = nullptr;
            const size_t nb = n_pairs * sizeof(NwPairDesc);
            if ((e = pinned_staging(p->ctx, nb, &st)) != hipSuccess) return fail(e, "pinned staging");
            std::memcpy(st, p->h_pairs.data(), nb);
            if ((e = hipMemcpy(p->d_pairs, st, nb, hipMemcpyHostToDevice)) != hipSuccess)
                return fail(e, "hipMemcpy(pairs)");
        }
        if ((e = dev_alloc(p->ctx, (void **)&p->d_endh, n_pairs * sizeof(int32_t))) != hipSuccess)
            return fail(e, "hipMalloc(end)");
    }
    clk.mark("plan: pairs h2d");
    // +64 B: the traceback walker reads whole 5-dword segments
    if (moff && (e = dev_alloc(p->ctx, (void **)&p->d_mask, moff + 64)) != hipSuccess)
        return fail(e, "hipMalloc(mask workspace)");
    {
        // stripe work list (pair-major, chunk-ascending: a stripe's predecessor
        // always has a lower workgroup id) and progress counters
        std::vector<uint2> work;
        p->work_first.assign(n_pairs + 1, 0);
        for (uint64_t r = 0; r < n_pairs; ++r) {
            NwPairDesc &d = p->h_pairs[r];
            p->work_first[r] = (uint32_t)work.size();
            if (d.variant != (uint32_t)kStripeVariant || !d.len_q || !d.len_db) continue;
            const uint32_t nch = variant_geom(kStripeVariant).n_chunks(d.len_q);
            d.reserved = (uint32_t)p->n_prog;
            p->n_prog += nch;
            for (uint32_t ch = 0; ch < nch; ++ch) work.push_back(make_uint2((uint32_t)r, ch));
        }
        p->work_first[n_pairs] = (uint32_t)work.size();
        if (!work.empty()) {
            if ((e = dev_alloc(p->ctx, (void **)&p->d_work, work.size() * sizeof(uint2))) != hipSuccess ||
                (e = hipMemcpy(p->d_work, work.data(), work.size() * sizeof(uint2),
                               hipMemcpyHostToDevice)) != hipSuccess ||
                (e = dev_alloc(p->ctx, (void **)&p->d_prog, p->n_prog * sizeof(uint32_t))) != hipSuccess ||
                (e = dev_alloc(p->ctx, (void **)&p->d_err, kErrWords * sizeof(uint32_t))) != hipSuccess ||
                // every XCD slot cleared: a recycled block must not hold a live epoch
                (e = hipMemset(p->d_err, 0, kErrWords * sizeof(uint32_t))) != hipSuccess ||
                (e = hipMemcpy(p->d_err, std::array<uint32_t, 2>{0u, kWaitLimitDefault}.data(),
                               2 * sizeof(uint32_t), hipMemcpyHostToDevice)) != hipSuccess)
                return fail(e, "stripe work list");
            if ((e = hipMemcpy(p->d_pairs, p->h_pairs.data(), n_pairs * sizeof(NwPairDesc),
                               hipMemcpyHostToDevice)) != hipSuccess)
                return fail(e, "hipMemcpy(pairs)");
        }
    }
    clk.mark("plan: mask+work");
    if (soff && (e = dev_alloc(p->ctx, (void **)&p->d_scratch, soff * sizeof(int2))) != hipSuccess)
        return fail(e, "hipMalloc(scratch)");
    p->ops_words = ooff;
    if (ooff && (e = dev_alloc(p->ctx, (void **)&p->d_ops, ooff * sizeof(uint32_t))) != hipSuccess)
        return fail(e, "hipMalloc(op stream)");
    // table fills (4-bit codes; full codes in 16-lane groups): a bail word per variant
    if ((p->var_count[kNarrowVariant] && p->nib[kNarrowVariant]) || (p->var_count[7] && p->nib[7]) ||
        (p->full_codes && (p->var_count[5] || p->var_count[7]))) {
        if ((e = dev_alloc(p->ctx, (void **)&p->d_bail[0], kBailBytes)) != hipSuccess ||
            (e = hipMemset(p->d_bail[0], 0, kBailBytes)) != hipSuccess)
            return fail(e, "table fill bail words");
    }
    {
        // Speculative stripe walks: a few long column-stripe pairs walk all
        // their 256-column stripes at once (nw_traceback_coop_kernel kSpec)
        // instead of one stripe after another (C4: walk 3.8 ms).  Off with
        // option nw.spec = 0; nw.spec_passes walk passes (default 3).
        const int passes = (int)opts[Opt::SpecPasses];
        const uint32_t nv = p->var_count[kStripeVariant];
        std::vector<SpecPair> sp;
        std::vector<uint2> blocks;
        if (opts[Opt::Spec] != 0 && passes > 0 && nv && nv <= kSpecMaxPairs) {
            for (uint32_t r = p->var_first[kStripeVariant]; r < p->var_first[kStripeVariant] + nv; ++r) {
                const NwPairDesc &d = p->h_pairs[r];
                const uint32_t S = (d.len_q + 255) / 256;
                if (S < kSpecMinStripes || S > kSpecMaxStripes) continue;
                sp.push_back(SpecPair{r, S, (uint32_t)blocks.size(), 0});
                for (uint32_t s = 0; s < S; ++s) blocks.push_back(make_uint2((uint32_t)sp.size() - 1, s));
            }
        }
        if (!sp.empty()) {
            p->spec_pairs = (uint32_t)sp.size();
            p->spec_blocks = (uint32_t)blocks.size();
            p->spec_passes = passes;
            p->spec_strict = opts[Opt::SpecStrict] != 0;
            if ((e = dev_alloc(p->ctx, (void **)&p->d_spec_blocks, blocks.size() * sizeof(uint2))) != hipSuccess ||
                (e = hipMemcpy(p->d_spec_blocks, blocks.data(), blocks.size() * sizeof(uint2),
                               hipMemcpyHostToDevice)) != hipSuccess ||
                (e = dev_alloc(p->ctx, (void **)&p->d_spec_pairs, sp.size() * sizeof(SpecPair))) != hipSuccess ||
                (e = hipMemcpy(p->d_spec_pairs, sp.data(), sp.size() * sizeof(SpecPair),
                               hipMemcpyHostToDevice)) != hipSuccess ||
                (e = dev_alloc(p->ctx, (void **)&p->d_spec_stripes, blocks.size() * sizeof(SpecStripe))) != hipSuccess ||
                (e = dev_alloc(p->ctx, (void **)&p->d_spec_ops,
                               blocks.size() * kSpecOpsCap * sizeof(uint32_t))) != hipSuccess ||
                (e = dev_alloc(p->ctx, (void **)&p->d_spec_done, n_pairs * sizeof(uint32_t))) != hipSuccess ||
                (e = hipMemset(p->d_spec_done, 0, n_pairs * sizeof(uint32_t))) != hipSuccess)
                return fail(e, "speculative walk tables");
        }
    }
    *out = p;
    return SALN_OK;
}

extern "C" {

int saln_nw_plan_info(const saln_nw_plan *p, uint64_t *mask_bytes, uint64_t *cigar_words,
                      uint64_t *cells) {
    if (!p) return SALN_E_INVALID;
    if (mask_bytes) *mask_bytes = p->mask_bytes;
    if (cigar_words) *cigar_words = p->cigar_off.back();
    if (cells) *cells = p->cells;
    return SALN_OK;
}

int saln_nw_cigar_offsets(const saln_nw_plan *p, uint64_t *off) {
    if (!p || !off) return SALN_E_INVALID;
    std::memcpy(off, p->cigar_off.data(), p->cigar_off.size() * sizeof(uint64_t));
    return SALN_OK;
}

int saln_nw_plan_set_timing(saln_nw_plan *p, int enable) {
    if (!p) return SALN_E_INVALID;
    HIP_TRY(hipSetDevice(p->ctx->device));
    if (p->ev_used) {
        const int rc = p->resolve_events();
        if (rc != SALN_OK) return rc;
    }
    p->timing = enable != 0;
    p->ktime.clear();
    // the event sets of the next executes, created now rather than inside
    // them (a timed C2 step that created its four events ran 0.5 % slower,
    // round 6, profiles/r06_timing_events_ab.jsonl); more are made on demand
    constexpr size_t kEventSets = 64;
    while (p->timing && p->ev_pool.size() < kEventSets) {
        std::array<hipEvent_t, 4> e4{};
        for (auto &e : e4) HIP_TRY(hipEventCreate(&e));
        p->ev_pool.push_back(e4);
    }
    return SALN_OK;
}

int saln_nw_plan_kernel_time(const saln_nw_plan *p, const char *kernel, double *total_ms,
                             uint64_t *launches) {
    if (!p || !kernel) return SALN_E_INVALID;
    const int rc = const_cast<saln_nw_plan *>(p)->resolve_events();
    if (rc != SALN_OK) return rc;
    auto it = p->ktime.find(kernel);
    if (total_ms) *total_ms = it == p->ktime.end() ? 0.0 : it->second.first;
    if (launches) *launches = it == p->ktime.end() ? 0 : it->second.second;
    return SALN_OK;
}

// Waves of an LDS walk launch (nw.walk_waves; -1 auto).  Beside the next
// step's fill (async plans) every lane walks two pairs in turn: half the
// walker waves take SIMD slots from the fill, and the walk still ends inside
// it (round 5, profiles/r05_walk_waves_ab.jsonl: C2 step 0.853-0.861 ->
// 0.836-0.846 ms at 768 waves; 512 made the walk outlast the fill, 0.97 ms).
// Alone, a lane per pair (the shortest walk).
static uint32_t walk_waves(int64_t opt, uint32_t n, bool beside_fill) {
    if (opt >= 0) return (uint32_t)opt;
    return beside_fill ? (n + 127) / 128 : 0;
}

int saln_nw_execute(saln_nw_plan *p, const uint8_t *d_q, const uint8_t *d_db,
                    saln_nw_result *d_results, uint32_t *d_cigar, void *stream) {
    if (!p || !d_results || (!d_q && p->n_pairs) || (!d_db && p->n_pairs)) return SALN_E_INVALID;
    if (p->n_pairs == 0) return SALN_OK;
    HIP_TRY(hipSetDevice(p->ctx->device));
    hipStream_t s = resolve_stream(stream, p->ctx);
    // the traceback stream: the second one only in async plans (the walk of
    // execute n beside the fill of n+1); otherwise the same stream, so no
    // cross-stream hand-off sits between the fill and the walk
    hipStream_t t = p->async_tb ? (p->tb_stream ? p->tb_stream : p->ctx->tb_stream) : s;
    const int cur = p->async_tb ? p->buf : 0;
    uint8_t *mask = cur ? p->d_mask2 : p->d_mask;
    int32_t *endh = cur ? p->d_endh2 : p->d_endh;
    uint32_t *ops = cur ? p->d_ops2 : p->d_ops;
    // this workspace may still be read by the traceback of execute n-2
    if (p->tb_pending[cur]) HIP_TRY(hipStreamWaitEvent(s, p->tb_done(cur), 0));
    // boundary columns preset to kColEmpty: a row is published once its value
    // replaces the preset (nw_fill_rows_kernel).  Issued ahead of the timing
    // events, so "nw_fill" times the fill kernels alone.
    {
        const uint32_t a = p->var_first[kStripeVariant];
        const uint32_t b = a + p->var_count[kStripeVariant];
        if (a < b && p->work_first[b] > p->work_first[a]) {
            const NwPairDesc &la = p->h_pairs[b - 1];
            const uint64_t c0 = p->h_pairs[a].scratch_off;
            const uint64_t c1 = la.scratch_off + (uint64_t)p->stripe_sub *
                                                     variant_geom(kStripeVariant).n_chunks(la.len_q) *
                                                     scratch_col(la.len_db);
            HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)(p->d_scratch + c0), (int)0x80000000u,
                                      2 * (c1 - c0), s));
        }
    }
    hipEvent_t *ev = nullptr;
    if (p->timing) {
        if (p->ev_used == p->ev_pool.size()) {
            std::array<hipEvent_t, 4> e4{};
            for (auto &e : e4) HIP_TRY(hipEventCreate(&e));
            p->ev_pool.push_back(e4);
        }
        ev = p->ev_pool[p->ev_used++].data();
        HIP_TRY(hipEventRecord(ev[0], s));
    }
    // fills on `s`, then the walks on `t` (async: beside the next fill)
    FillExtras fx;
    fx.o = &p->opts;
    // async: the table fills' fallback launches go to the walk stream, behind
    // the hand-off, so nothing but the hand-off's packets sits between this
    // fill and the next one on `s` (each packet there left ~5 us idle, rocprof
    // kernel trace, round 5)
    std::vector<std::function<hipError_t(hipStream_t)>> fallbacks;
    if (t != s) fx.deferred = &fallbacks;
    for (int v = 0; v < kNumVariants; ++v) {
        const uint32_t a = p->var_first[v], b = a + p->var_count[v];
        if (a >= b) continue;
        if (v == kStripeVariant) {
            const uint32_t w0 = p->work_first[a], w1 = p->work_first[b];
            if (w1 > w0)
                HIP_TRY(launch_fill_stripes(p->d_pairs, p->d_work + w0, w1 - w0, d_q, d_db, mask,
                                            p->d_scratch, p->d_prog, p->d_err, endh, p->sc,
                                            p->score_only ? 2 : p->full_codes ? 1 : 0,
                                            p->stripe_layout(), p->stripe_rows, s, p->opts,
                                            ++p->fill_epoch));
            continue;
        }
        fx.epoch = ++p->epoch;
        // one bail word per variant: two table fills queued before either
        // deferred fallback runs must not overwrite each other's epoch
        fx.bail = p->d_bail[cur] ? p->d_bail[cur] + v : nullptr;
        HIP_TRY(launch_fill(v, p->d_pairs, a, b - a, d_q, d_db, mask, p->d_scratch, endh,
                            d_results, d_cigar, p->sc,
                            p->score_only ? 2 : p->full_codes ? 1 : p->nib[v] ? 3 : 0,
                            p->var_maxld[v], s, fx));
    }
    // the fill's end (timed: its timing event doubles as the hand-off)
    hipEvent_t filled = ev ? ev[1] : p->sync_ev[0];
    HIP_TRY(hipEventRecord(filled, s));
    if (t != s) HIP_TRY(hipStreamWaitEvent(t, filled, 0));
    for (auto &fb : fallbacks) HIP_TRY(fb(t));
    // (async plans: the deferred fallback launches sit between ev[1] and
    // ev[2], so neither "nw_fill" nor "nw_traceback" counts them; they run
    // only for waves whose pairs hold a byte other than A, C, G, T)
    if (ev) HIP_TRY(hipEventRecord(ev[2], t));
    for (int v = 0; v < kNumVariants; ++v) {
        const uint32_t a = p->var_first[v], b = a + p->var_count[v];
        if (a >= b) continue;
        const bool spec = v == kStripeVariant && p->spec_pairs && !p->score_only;
        if (spec)
            HIP_TRY(launch_traceback_spec(
                p->d_pairs,
                SpecArgs{p->d_spec_blocks, p->d_spec_pairs, p->d_spec_stripes, p->d_spec_ops,
                         p->d_spec_done, 0},
                p->spec_blocks, p->spec_pairs, p->d_spec_done, p->spec_passes, d_q, d_db, mask,
                endh, d_results, d_cigar, p->sc, p->stripe_layout(),
                p->spec_strict ? p->d_err : nullptr, t));
        if (p->score_only)
            HIP_TRY(launch_score_results(p->d_pairs, a, b - a, endh, d_results, p->sc, t));
        else
            HIP_TRY(launch_traceback(v, p->d_pairs, a, b - a, d_q, d_db, mask, endh, ops,
                                     d_results, d_cigar, p->sc, p->stripe_layout(), t,
                                     spec ? p->d_spec_done : nullptr, p->nib[v],
                                     walk_waves(p->opts[Opt::WalkWaves], b - a, t != s)));
    }
    // pairs with an empty side (boundary-only walk) ride on the traceback stream
    if (p->n_pairs > p->n_fill && p->score_only)
        HIP_TRY(launch_score_results(p->d_pairs, p->n_fill, (uint32_t)(p->n_pairs - p->n_fill),
                                     endh, d_results, p->sc, t));
    else if (p->n_pairs > p->n_fill)
        HIP_TRY(launch_traceback(-1, p->d_pairs, p->n_fill, (uint32_t)(p->n_pairs - p->n_fill),
                                 d_q, d_db, mask, endh, ops, d_results, d_cigar, p->sc,
                                 p->stripe_layout(), t));
    if (ev) HIP_TRY(hipEventRecord(ev[3], t));
    HIP_TRY(hipEventRecord(p->tb_done(cur), t));
    p->tb_pending[cur] = true;
    p->unchecked[cur] = true;
    p->last_buf = cur;
    if (p->async_tb) {
        p->buf ^= 1;  // results complete once saln_nw_plan_sync'ed
    } else {
        if (t != s) HIP_TRY(hipStreamWaitEvent(s, p->tb_done(cur), 0));
        p->tb_pending[cur] = false;
    }
    return SALN_OK;
}

int saln_nw_plan_set_score_only(saln_nw_plan *p, int enable) {
    if (!p) return SALN_E_INVALID;
    p->score_only = enable != 0;
    return SALN_OK;
}

int saln_nw_plan_set_async(saln_nw_plan *p, int enable) {
    if (!p) return SALN_E_INVALID;
    HIP_TRY(hipSetDevice(p->ctx->device));
    if (enable && !p->d_mask2 && p->mask_bytes) {
        HIP_TRY(dev_alloc(p->ctx, (void **)&p->d_mask2, p->mask_bytes + 64));
        HIP_TRY(dev_alloc(p->ctx, (void **)&p->d_endh2, p->n_pairs * sizeof(int32_t)));
        if (p->ops_words)
            HIP_TRY(dev_alloc(p->ctx, (void **)&p->d_ops2, p->ops_words * sizeof(uint32_t)));
        if (p->d_bail[0]) {
            HIP_TRY(dev_alloc(p->ctx, (void **)&p->d_bail[1], kBailBytes));
            HIP_TRY(hipMemset(p->d_bail[1], 0, kBailBytes));
        }
    }
    p->async_tb = enable != 0;
    p->buf = 0;
    return SALN_OK;
}

int saln_nw_plan_set_tb_stream(saln_nw_plan *p, void *stream) {
    if (!p) return SALN_E_INVALID;
    p->tb_stream = (hipStream_t)stream;
    return SALN_OK;
}

int saln_nw_plan_status(saln_nw_plan *p, uint32_t *flags) {
    if (flags) *flags = 0;
    if (!p) return SALN_E_INVALID;
    HIP_TRY(hipSetDevice(p->ctx->device));
    for (int b = 0; b < 2; ++b)
        if (p->unchecked[b]) HIP_TRY(hipEventSynchronize(p->tb_done(b)));
    p->unchecked[0] = p->unchecked[1] = false;
    uint32_t v = 0;
    if (p->d_err) {
        HIP_TRY(hipMemcpy(&v, p->d_err, sizeof v, hipMemcpyDeviceToHost));
        if (v) HIP_TRY(hipMemset(p->d_err, 0, sizeof v));  // read and clear
    }
    if (flags) *flags = v;
    if (v & SALN_FLAG_WAIT_TIMEOUT) {
        set_error("column-stripe dependency wait timed out (results of the executes since the "
                  "last status are invalid)");
        return SALN_E_DEVICE_WAIT;
    }
    if (v & SALN_FLAG_SPEC_UNLINKED) {
        set_error("speculative stripe walk did not link (SALN_SPEC_STRICT=1)");
        return SALN_E_DEVICE_WAIT;
    }
    return SALN_OK;
}

int saln_nw_plan_set_wait_limit(saln_nw_plan *p, uint32_t polls) {
    if (!p) return SALN_E_INVALID;
    HIP_TRY(hipSetDevice(p->ctx->device));
    p->wait_limit = polls;
    if (p->d_err) HIP_TRY(hipMemcpy(p->d_err + 1, &polls, sizeof polls, hipMemcpyHostToDevice));
    return SALN_OK;
}

int saln_nw_plan_sync(saln_nw_plan *p, void *stream, int keep_latest) {
    if (!p) return SALN_E_INVALID;
    HIP_TRY(hipSetDevice(p->ctx->device));
    hipStream_t s = resolve_stream(stream, p->ctx);
    for (int b = 0; b < 2; ++b) {
        if (!p->tb_pending[b] || (keep_latest && b == p->last_buf)) continue;
        HIP_TRY(hipStreamWaitEvent(s, p->tb_done(b), 0));
        p->tb_pending[b] = false;
    }
    return SALN_OK;
}

}  // extern "C"

int saln_nw_plan::resolve_events() {
    HIP_TRY(hipSetDevice(ctx->device));
    for (size_t k = 0; k < ev_used; ++k) {
        hipEvent_t *ev = ev_pool[k].data();
        HIP_TRY(hipEventSynchronize(ev[3]));
        float a = 0, b = 0, c = 0;
        HIP_TRY(hipEventElapsedTime(&a, ev[0], ev[1]));  // fill span on the caller's stream
        HIP_TRY(hipEventElapsedTime(&b, ev[2], ev[3]));  // traceback span on its stream
        HIP_TRY(hipEventElapsedTime(&c, ev[0], ev[3]));  // whole execute
        auto &f = ktime["nw_fill"];
        f.first += a;
        f.second += 1;
        auto &t = ktime["nw_traceback"];
        t.first += b;
        t.second += 1;
        auto &x = ktime["nw_execute"];
        x.first += c;
        x.second += 1;
    }
    ev_used = 0;
    return SALN_OK;
}

// ----------------------------------------------------------- host traceback
namespace saln {

int plan_pair_mask(const saln_nw_plan *p, uint64_t pair_id, PairMask *pm) {
    if (!p || pair_id >= p->n_pairs) return SALN_E_INVALID;
    const NwPairDesc &d = p->h_pairs[p->plan_index[pair_id]];
    if (!p->full_codes) {  // every fill stores walk codes unless the plan asks for all parents
        set_error("plan_pair_mask: plan stores walk codes only");
        return SALN_E_INVALID;
    }
    pm->g = variant_geom((int)d.variant);
    pm->m.clear();
    pm->rs = 0;
    pm->bs = pm->g.LB();
    if (d.len_q == 0 || d.len_db == 0) return SALN_OK;
    if (d.variant == (uint32_t)kStripeVariant) {  // skewed stripe regions: copied whole
        pm->rs = d.mask_rs;
        pm->bs = d.mask_bs;
        pm->cs = d.mask_cs;
        pm->m.resize(pm->g.n_chunks(d.len_q) * d.mask_cs);
        HIP_TRY(hipSetDevice(p->ctx->device));
        HIP_TRY(hipMemcpy(pm->m.data(), p->d_mask + d.mask_off, pm->m.size(), hipMemcpyDeviceToHost));
        return SALN_OK;
    }
    const uint64_t lb = pm->g.LB();
    // every row holds rs / bs blocks (the pack's width); copy them all as
    // LB-byte rows of one bs-pitched 2-D region
    const uint64_t nb = d.mask_rs / d.mask_bs;
    pm->rs = nb * lb;
    pm->cs = (uint64_t)pm->g.G * lb;
    pm->m.resize((uint64_t)d.len_db * nb * lb);
    HIP_TRY(hipSetDevice(p->ctx->device));
    HIP_TRY(hipMemcpy2D(pm->m.data(), lb, p->d_mask + d.mask_off, d.mask_bs, lb,
                        (uint64_t)d.len_db * nb, hipMemcpyDeviceToHost));
    return SALN_OK;
}

int plan_next_event(saln_nw_plan *p, const saln_nw_result *d_results, uint8_t *d_next,
                    hipStream_t stream) {
    if (!p || !d_results || !d_next) return SALN_E_INVALID;
    if (!p->full_codes) {
        set_error("plan_next_event: plan stores walk codes only");
        return SALN_E_INVALID;
    }
    if (!p->n_pairs) return SALN_OK;
    HIP_TRY(hipSetDevice(p->ctx->device));
    HIP_TRY(launch_next_event(p->d_pairs, (uint32_t)p->n_pairs, p->d_mask, d_results, p->sc,
                              d_next, stream));
    return SALN_OK;
}

int plan_mask_source(const saln_nw_plan *p, const uint8_t **d_mask) {
    if (!p || !d_mask) return SALN_E_INVALID;
    if (!p->full_codes) {
        set_error("plan_mask_source: plan stores walk codes only");
        return SALN_E_INVALID;
    }
    *d_mask = p->d_mask;
    return SALN_OK;
}

// one past the largest offset of the pair's cells in every layout
// (nw_common.hpp Geom::cell): its end cell
uint64_t plan_mask_end(const saln_nw_plan *p, uint64_t pair_id) {
    const NwPairDesc &d = p->h_pairs[p->plan_index[pair_id]];
    if (d.len_q == 0 || d.len_db == 0) return 0;
    const Geom g = variant_geom((int)d.variant);
    return d.mask_off + g.cell(d.len_db, d.len_q, d.mask_rs, d.mask_bs, d.mask_cs) + 1;
}

HostMask plan_host_mask(const saln_nw_plan *p, const uint8_t *host, uint64_t pair_id) {
    const NwPairDesc &d = p->h_pairs[p->plan_index[pair_id]];
    HostMask hm;
    hm.m = host + d.mask_off;
    hm.g = variant_geom((int)d.variant);
    hm.rs = d.mask_rs;
    hm.bs = d.mask_bs;
    hm.cs = d.mask_cs;
    hm.lq = d.len_q;
    hm.ld = d.len_db;
    hm.sc = p->sc;
    return hm;
}

void HostMask::to_dense(uint8_t *out) const {
    const uint64_t W = (uint64_t)lq + 1;
    for (uint32_t i = 0; i <= ld; ++i) {
        for (uint32_t j = 0; j <= lq; ++j) {
            uint8_t b = argmax(i, j);
            if (i >= 1 && j >= 1) b |= (uint8_t)(ibits(i, j) << 3 | dbits(i, j) << 5);
            if (i == 0 && j >= 1) b |= kDExt;  // D[0][j] <- D[0][j-1], :196
            if (j == 0 && i >= 1) b |= kIExt;  // I[i][0] <- I[i-1][0], :208
            out[(uint64_t)i * W + j] = b;
        }
    }
}

namespace {
enum { ST_M = 0, ST_I = 1, ST_D = 2 };

// Parents of a node in the reference's push order (DFS visits them reversed).
int parents(const HostMask &hm, int st, uint32_t i, uint32_t j, int *ps, uint32_t *pi,
            uint32_t *pj) {
    int n = 0;
    if (i == 0 || j == 0) {  // boundary nodes, :172-216
        if (st == ST_D && i == 0 && j >= 1) { ps[0] = ST_D; pi[0] = 0; pj[0] = j - 1; return 1; }
        if (st == ST_I && j == 0 && i >= 1) { ps[0] = ST_I; pi[0] = i - 1; pj[0] = 0; return 1; }
        return 0;
    }
    if (st == ST_M) {
        const uint8_t a = hm.argmax(i - 1, j - 1);
        if (a & kArgM) { ps[n] = ST_M; pi[n] = i - 1; pj[n] = j - 1; ++n; }
        if (a & kArgI) { ps[n] = ST_I; pi[n] = i - 1; pj[n] = j - 1; ++n; }
        if (a & kArgD) { ps[n] = ST_D; pi[n] = i - 1; pj[n] = j - 1; ++n; }
    } else if (st == ST_I) {
        const uint8_t b = hm.ibits(i, j);
        if (b & 1) { ps[n] = ST_I; pi[n] = i; pj[n] = j - 1; ++n; }
        if (b & 2) { ps[n] = ST_M; pi[n] = i; pj[n] = j - 1; ++n; }
    } else {
        const uint8_t b = hm.dbits(i, j);
        if (b & 1) { ps[n] = ST_D; pi[n] = i - 1; pj[n] = j; ++n; }
        if (b & 2) { ps[n] = ST_M; pi[n] = i - 1; pj[n] = j; ++n; }
    }
    return n;
}

// Panics when a node with parents is expanded at x == 0 (M, D) or y == 0 (M, I).
bool panics(int st, uint32_t i, uint32_t j, int np) {
    if (np == 0) return false;
    if (st == ST_M) return i == 0 || j == 0;
    if (st == ST_D) return i == 0;
    return j == 0;
}

struct Node {
    int st;
    uint32_t i, j;
};

// end states in DFS pop order: D, M, I (pushed I, M, D at :251-280)
int end_nodes(const HostMask &hm, Node *out) {
    const uint8_t a = hm.argmax(hm.ld, hm.lq);
    int n = 0;
    if (a & kArgD) out[n++] = {ST_D, hm.ld, hm.lq};
    if (a & kArgM) out[n++] = {ST_M, hm.ld, hm.lq};
    if (a & kArgI) out[n++] = {ST_I, hm.ld, hm.lq};
    return n;
}

char col_q(int st, const uint8_t *q, uint32_t j) { return st == ST_D ? '-' : (char)q[j - 1]; }
char col_d(int st, const uint8_t *d, uint32_t i) { return st == ST_I ? '-' : (char)d[i - 1]; }
}  // namespace

DfsOutcome render_blocks(const HostMask &hm, const uint8_t *q, const uint8_t *d,
                         uint64_t max_blocks, std::string *out) {
    DfsOutcome res;
    const uint32_t lq = hm.lq, ld = hm.ld;
    // Every mask layout is row-separable: cell(i, j) = (i-1) RS + co[j] (the
    // packed stripes' skew included, RS = 256), so a node's code byte is a
    // row pointer and a column offset from two tables instead of
    // Geom::cell's divisions.
    std::vector<uint64_t> co(lq + 1, 0);
    for (uint32_t j = 1; j <= lq && ld; ++j) co[j] = hm.g.cell(1, j, hm.rs, hm.bs, hm.cs);
    const uint64_t RS = hm.bs == 0 ? 256 : hm.rs;
    std::vector<const uint8_t *> rowp(ld + 1, nullptr);
    for (uint32_t i = 1; i <= ld && lq; ++i) rowp[i] = hm.m + (uint64_t)(i - 1) * RS;
    auto byte = [&](uint32_t i, uint32_t j) -> uint32_t { return rowp[i][co[j]] ^ 0x7Fu; };
    struct Item {
        uint32_t i, j, st, depth;
    };
    std::vector<Item> stack;
    stack.reserve(4 * ((size_t)lq + ld) + 8);
    // the path's columns stored back to front (depth k at cap - 1 - k), so a
    // block's three lines are three contiguous copies
    const uint32_t cap = lq + ld + 1;
    std::vector<char> p1(cap), p2(cap), pb(cap);
    {   // end states pushed I, M, D (:251-280): popped D, M, I
        const uint8_t a = hm.argmax(ld, lq);
        if (a & kArgI) stack.push_back({ld, lq, ST_I, 0});
        if (a & kArgM) stack.push_back({ld, lq, ST_M, 0});
        if (a & kArgD) stack.push_back({ld, lq, ST_D, 0});
    }
    while (!stack.empty()) {
        Item it = stack.back();
        stack.pop_back();
        // a node's last pushed parent is the next popped: it is followed at
        // once, without the stack, down the chain until a leaf
        for (;;) {
            const uint32_t i = it.i, j = it.j, st = it.st, dep = it.depth;
            if (i == 0 && j == 0) {  // :283-286
                if (max_blocks && res.blocks >= max_blocks) {
                    res.status = SALN_ENUM_CAP;
                    return res;
                }
                if (out) {
                    const uint32_t a = cap - dep;
                    out->append("alignment found\n\nseq1: ");
                    out->append(p1.data() + a, dep);
                    out->append("\n      ");
                    out->append(pb.data() + a, dep);
                    out->append("\nseq2: ");
                    out->append(p2.data() + a, dep);
                    out->push_back('\n');
                }
                ++res.blocks;
                break;
            }
            // parents in the reference's push order (parents() above)
            uint32_t ps[3], pi[3], pj[3];
            int np = 0;
            if (i == 0 || j == 0) {  // boundary nodes, :172-216
                if (st == ST_D && i == 0) { ps[0] = ST_D; pi[0] = 0; pj[0] = j - 1; np = 1; }
                else if (st == ST_I && j == 0) { ps[0] = ST_I; pi[0] = i - 1; pj[0] = 0; np = 1; }
            } else if (st == ST_M) {
                const uint32_t a = (i == 1 || j == 1) ? hm.argmax(i - 1, j - 1) : (byte(i - 1, j - 1) & 7u);
                if (a & kArgM) { ps[np] = ST_M; pi[np] = i - 1; pj[np] = j - 1; ++np; }
                if (a & kArgI) { ps[np] = ST_I; pi[np] = i - 1; pj[np] = j - 1; ++np; }
                if (a & kArgD) { ps[np] = ST_D; pi[np] = i - 1; pj[np] = j - 1; ++np; }
            } else if (st == ST_I) {
                const uint32_t b = j == 1 ? ibits_col1(hm.sc, i) : (byte(i, j - 1) >> 3) & 3u;
                if (b & 1) { ps[np] = ST_I; pi[np] = i; pj[np] = j - 1; ++np; }
                if (b & 2) { ps[np] = ST_M; pi[np] = i; pj[np] = j - 1; ++np; }
            } else {
                const uint32_t b = i == 1 ? dbits_row1(hm.sc, j) : (byte(i - 1, j) >> 5) & 3u;
                if (b & 1) { ps[np] = ST_D; pi[np] = i - 1; pj[np] = j; ++np; }
                if (b & 2) { ps[np] = ST_M; pi[np] = i - 1; pj[np] = j; ++np; }
            }
            if (np == 0) break;  // a sentinel-rooted dead end: dropped silently
            if (panics((int)st, i, j, np)) {
                res.status = SALN_REF_PANIC_BOUNDARY;
                return res;
            }
            const uint32_t x = cap - 1 - dep;
            const char c1 = col_q((int)st, q, j), c2 = col_d((int)st, d, i);
            p1[x] = c1;
            p2[x] = c2;
            pb[x] = c1 == c2 ? '|' : ' ';
            for (int k = 0; k < np - 1; ++k) stack.push_back({pi[k], pj[k], ps[k], dep + 1});
            it = {pi[np - 1], pj[np - 1], ps[np - 1], dep + 1};
        }
    }
    return res;
}

bool first_alignment(const HostMask &hm, const uint8_t *q, const uint8_t *d,
                     std::vector<uint32_t> *cigar) {
    // DFS in the reference order with "no event below" memoisation: the
    // first event is the origin (printed) or a panic node (nothing printed).
    auto key = [&](const Node &n) {
        return ((uint64_t)n.i * ((uint64_t)hm.lq + 1) + n.j) * 3 + (uint64_t)n.st;
    };
    std::unordered_set<uint64_t> dead;
    struct Frame {
        Node n;
        int np, next;  // next child index (counting down)
        int ps[3];
        uint32_t pi[3], pj[3];
    };
    std::vector<Frame> path;
    Node ends[3];
    const int ne = end_nodes(hm, ends);
    for (int e = 0; e < ne; ++e) {
        path.clear();
        auto enter = [&](const Node &n) -> int {  // 1 origin, 2 panic, 0 continue
            if (n.i == 0 && n.j == 0) return 1;
            Frame f;
            f.n = n;
            f.np = parents(hm, n.st, n.i, n.j, f.ps, f.pi, f.pj);
            if (panics(n.st, n.i, n.j, f.np)) return 2;
            f.next = f.np - 1;
            path.push_back(f);
            return 0;
        };
        int ev = enter(ends[e]);
        while (ev == 0 && !path.empty()) {
            Frame &f = path.back();
            bool descended = false;
            while (f.next >= 0) {
                const Node c{f.ps[f.next], f.pi[f.next], f.pj[f.next]};
                --f.next;
                if (dead.count(key(c))) continue;
                ev = enter(c);
                descended = true;
                break;
            }
            if (ev) break;
            if (!descended) {
                dead.insert(key(path.back().n));
                path.pop_back();
            }
        }
        if (ev == 2) return false;
        if (ev == 1) {
            if (cigar) {
                cigar->clear();
                // path holds the expanded nodes from the end to the origin's child
                for (size_t k = path.size(); k-- > 0;) {
                    const Node &n = path[k].n;
                    uint32_t op = n.st == ST_I ? SALN_CIGAR_I
                                  : n.st == ST_D ? SALN_CIGAR_D
                                  : (q[n.j - 1] == d[n.i - 1] ? SALN_CIGAR_EQ : SALN_CIGAR_X);
                    if (!cigar->empty() && (cigar->back() & 15u) == op)
                        cigar->back() += 16u;
                    else
                        cigar->push_back(16u | op);
                }
            }
            return true;
        }
    }
    return false;
}

}  // namespace saln

namespace saln {
int plan_check_error(saln_nw_plan *p) { return saln_nw_plan_status(p, nullptr); }
}  // namespace saln

namespace saln {

hipError_t dev_alloc(saln_context *ctx, void **p, size_t n) {
    n = n ? (n + 255) & ~size_t(255) : 256;
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        auto it = ctx->cache.lower_bound(n);
        if (it != ctx->cache.end() && it->first <= 2 * n) {
            *p = it->second;
            ctx->live[it->second] = it->first;
            ctx->cached -= it->first;
            ctx->cache.erase(it);
            return hipSuccess;
        }
    }
    hipError_t e = hipMalloc(p, n);
    if (e == hipErrorOutOfMemory) {  // give the cached blocks back and retry once
        (void)hipGetLastError();
        dev_cache_clear(ctx);
        e = hipMalloc(p, n);
    }
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->live[*p] = n;
    return hipSuccess;
}

void dev_free(saln_context *ctx, void *p) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(ctx->mu);
    auto it = ctx->live.find(p);
    if (it == ctx->live.end()) {
        (void)hipFree(p);
        return;
    }
    const size_t n = it->second;
    ctx->live.erase(it);
    if (ctx->cached + n > kDevCacheMax) {
        (void)hipFree(p);
        return;
    }
    ctx->cache.emplace(n, p);
    ctx->cached += n;
}

void dev_cache_clear(saln_context *ctx) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    for (auto &kv : ctx->cache) (void)hipFree(kv.second);
    ctx->cache.clear();
    ctx->cached = 0;
}

hipError_t pinned_staging(saln_context *ctx, size_t n, void **p) {
    if (n > ctx->pinned_bytes) {
        const size_t want = std::max(n, ctx->pinned_bytes * 2);
        if (ctx->pinned) (void)hipHostFree(ctx->pinned);
        ctx->pinned = nullptr;
        ctx->pinned_bytes = 0;
        hipError_t e = hipHostMalloc(&ctx->pinned, want, hipHostMallocDefault);
        if (e != hipSuccess) return e;
        ctx->pinned_bytes = want;
    }
    *p = ctx->pinned;
    return hipSuccess;
}

}  // namespace saln

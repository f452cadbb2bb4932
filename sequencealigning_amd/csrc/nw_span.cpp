// Column spans of one long pair (include/saln.h "one long pair split by
// columns").
//
// The reference fills one pair row by row, query inner
// (needleman_wunsch_affine.rs:217-236), and walks it back from the end cell
// (:242-334).  A span is the row fill (nw_fill_rows_kernel) restricted to the
// column stripes of query columns col_lo+1 .. col_hi: its work items are the
// pair's 256-column chunks of that range, and its kernel arguments are
// rebased so that
//   - the stripe left of its first one reads boundary column 0 (the inbox),
//     which a peer fills row by row while the fill runs (the same polled
//     8-byte elements as between two stripes of one GPU), and its last stripe
//     publishes into the last column (the outbox);
//   - its mask holds only its own 256-column tiles (a pair whose 1 B/cell
//     mask exceeds one GPU's HBM spreads over the spans' GPUs).
// The walk enters at a known cell (the exit of the span to the right): the
// speculative stripe walker's passes over the span's 256-column stripes,
// linked on the host (span_walk_spec), or, when they do not link, one walk
// through the span that stops only where it leaves it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "nw_host.hpp"

namespace saln {
bool scores_fit_i32(const Scoring &s, uint64_t lq, uint64_t ld);
}
using namespace saln;

struct saln_nw_span {
    saln_context *ctx = nullptr;
    Options opts{};  // the context's effective options at creation
    Scoring sc{};
    uint32_t lq = 0, ld = 0, col_lo = 0, col_hi = 0;
    int K = 2;                  // row-fill columns per lane (stripe width 64 K)
    uint32_t g0 = 0, nst = 0;   // first stripe (pair-wide index), stripes
    uint32_t t0 = 0, ntiles = 0;  // first 256-column mask tile, tiles
    uint64_t scol = 0, cs = 0, mask_bytes = 0, ops_cap = 0;
    bool own_bnd = false;
    int2 *d_bnd = nullptr;      // nst + 1 boundary columns
    uint8_t *d_mask = nullptr;
    NwPairDesc *d_pair = nullptr;
    uint2 *d_work = nullptr;
    uint32_t n_work = 0;
    uint32_t *d_err = nullptr;  // [flags, wait limit, XCD slots] (kErrWords; the fill's and the watch's waits)
    uint32_t fill_epoch = 0;    // fills launched (the XCD slots' epochs)
    int32_t *d_endh = nullptr;
    uint2 *d_blocks = nullptr;
    SpecPair *d_sp = nullptr;
    SpecStripe *d_rec = nullptr;  // [0] this span's walk, [1] its entry (pass-2 exit slot)
    uint32_t *d_ops = nullptr;
    // speculative passes over the span's walker stripes (one record per
    // stripe + the entry record after the rightmost), linked on the host
    int spec_passes = 0;
    uint2 *d_sblocks = nullptr;
    SpecPair *d_ssp = nullptr;
    SpecStripe *d_srec = nullptr;
    uint32_t *d_sops = nullptr;
    SpecStripe *h_srec = nullptr;  // pinned host copies (ntiles + 1 records, ntiles op slots)
    uint32_t *h_sops = nullptr;

    // kernel arguments rebased to the span: tile t of the pair at d_mask +
    // (t - t0) * cs; stripe g's output column g - g0 + 1 (its input g - g0)
    uint8_t *mask_arg() const { return (uint8_t *)((uintptr_t)d_mask - (uint64_t)t0 * cs); }
    int2 *scratch_arg() const {
        return (int2 *)((uintptr_t)d_bnd + (uint64_t)(1 - (int64_t)g0) * scol * sizeof(int2));
    }
    int2 *inbox() const { return d_bnd; }
    int2 *outbox() const { return d_bnd + (uint64_t)nst * scol; }
    void release() {
        for (void *b : {(void *)d_mask, (void *)d_pair, (void *)d_work, (void *)d_err,
                        (void *)d_endh, (void *)d_blocks, (void *)d_sp, (void *)d_rec,
                        (void *)d_ops, (void *)d_sblocks, (void *)d_ssp, (void *)d_srec,
                        (void *)d_sops})
            if (b) dev_free(ctx, b);
        if (own_bnd && d_bnd) dev_free(ctx, d_bnd);
        if (h_srec) (void)hipHostFree(h_srec);
        if (h_sops) (void)hipHostFree(h_sops);
    }
};

// The span's walk from the speculative passes: every walker stripe walks at
// once (the rightmost from the given entry, the others from a guess, then
// from their right neighbour's previous exit); the stored walks form the
// sequential walk when, from the rightmost stripe leftwards, each stripe's
// stored entry is where the walk left the stripe after it.  Returns SALN_OK,
// an error, or SALN_SPAN_UNLINKED when they do not link (the caller walks
// sequentially).
static int span_walk_spec(saln_nw_span *s, const uint8_t *d_q, const uint8_t *d_db,
                          const saln_nw_span_cursor *entry, saln_nw_span_cursor *exit,
                          uint32_t *ops, uint64_t ops_cap, uint64_t *n_ops, hipStream_t st) {
    const uint32_t n = s->ntiles;
    for (uint32_t t = 0; t < n; ++t) {
        s->h_srec[t] = SpecStripe{};
        s->h_srec[t].in_k = kSpecNone;  // no stored walk to keep
    }
    SpecStripe &d = s->h_srec[n];
    d = SpecStripe{};
    d.out_i[0] = d.out_i[1] = entry->i;
    d.out_j[0] = d.out_j[1] = entry->j;
    d.out_k[0] = d.out_k[1] = entry->kind;
    HIP_TRY(hipMemcpyAsync(s->d_srec, s->h_srec, (n + 1) * sizeof(SpecStripe),
                           hipMemcpyHostToDevice, st));
    // the kernel indexes records and op slots by the pair-wide stripe t:
    // tables rebased so that stripe t0 is element 0 (never read below it)
    SpecStripe *rec0 = (SpecStripe *)((uintptr_t)s->d_srec - (uint64_t)s->t0 * sizeof(SpecStripe));
    uint32_t *ops0 = (uint32_t *)((uintptr_t)s->d_sops -
                                  (uint64_t)s->t0 * kSpecOpsCap * sizeof(uint32_t));
    SpecArgs sa{s->d_sblocks, s->d_ssp, rec0, ops0, nullptr, 0, 0, 0, (int32_t)(s->t0 + n)};
    HIP_TRY(launch_span_spec(s->d_pair, sa, n, s->spec_passes, d_q, d_db, s->mask_arg(),
                             s->d_endh, s->sc, st));
    HIP_TRY(hipMemcpyAsync(s->h_srec, s->d_srec, n * sizeof(SpecStripe), hipMemcpyDeviceToHost,
                           st));
    HIP_TRY(hipMemcpyAsync(s->h_sops, s->d_sops, (size_t)n * kSpecOpsCap * sizeof(uint32_t),
                           hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const int cf = s->spec_passes & 1;  // exit slot of the last pass
    int32_t ci = entry->i, cj = entry->j, ck = entry->kind;
    uint64_t nw = 0;
    for (int t = (int)n - 1;; --t) {
        const SpecStripe &r = s->h_srec[t];
        if (r.in_i != ci || r.in_j != cj || r.in_k != ck || r.nops > kSpecOpsCap) return SALN_SPAN_UNLINKED;
        if (ops && nw + r.nops > ops_cap) {
            set_error("span walk: ops buffer too small (saln_nw_span_info ops_cap)");
            return SALN_E_CAPACITY;
        }
        if (ops) std::memcpy(ops + nw, s->h_sops + (size_t)t * kSpecOpsCap, r.nops * sizeof(uint32_t));
        nw += r.nops;
        ci = r.out_i[cf];
        cj = r.out_j[cf];
        ck = r.out_k[cf];
        if (ck >= kSpecEv || t == 0) break;  // ended, or left the span
    }
    if (ck == kSpecNone) return SALN_SPAN_UNLINKED;
    *n_ops = nw;
    exit->i = ci;
    exit->j = cj;
    exit->kind = ck;
    exit->end_states = entry->kind == SALN_SPAN_END ? s->h_srec[n - 1].am_end : 0u;
    return SALN_OK;
}

// Row-fill columns per lane of a span: K = 1 while every 64-column stripe of
// the span has a SIMD to itself (stripe_rows_k)
static int span_k(uint64_t col_lo, uint64_t col_hi, uint64_t device_cols, const Options &o) {
    return stripe_rows_k((std::max(col_hi - col_lo, device_cols) + 63) / 64, o);
}

extern "C" {

uint64_t saln_nw_span_boundary_elems(uint64_t len_db) {
    return len_db > 0xFFFFFFFFull ? 0 : scratch_col((uint32_t)len_db);
}

uint64_t saln_nw_span_boundary_cols(uint64_t col_lo, uint64_t col_hi, uint64_t device_cols) {
    if (col_hi <= col_lo) return 0;
    // (no context: the process registry's nw.rows_k)
    const uint64_t W = 64u * (uint64_t)span_k(col_lo, col_hi, device_cols, opt_registry());
    return (col_hi + W - 1) / W - col_lo / W + 1;
}

int saln_nw_span_create(saln_context *ctx, uint64_t len_q, uint64_t len_db, uint64_t col_lo,
                        uint64_t col_hi, uint64_t device_cols, const saln_nw_scoring *scoring,
                        void *d_boundary, saln_nw_span **out) {
    if (!ctx || !out) return SALN_E_INVALID;
    *out = nullptr;
    if (len_q <= 256 || len_db == 0 || len_q > 0x7FFFFFFFull || len_db > 0x7FFFFFFFull) {
        set_error("span: a pair of more than 256 query columns and at least one db row "
                  "(shorter pairs: saln_nw_plan_create)");
        return SALN_E_INVALID;
    }
    if (col_lo % 256 || col_lo >= col_hi || col_hi > len_q || (col_hi != len_q && col_hi % 256)) {
        set_error("span: columns col_lo+1 .. col_hi with col_lo and col_hi (unless len_q) "
                  "multiples of 256");
        return SALN_E_INVALID;
    }
    const Scoring sc = scoring_or_default(scoring);
    if (!scores_fit_i32(sc, len_q, len_db)) {
        set_error("pair too long for these penalties: its scores could leave the engine's int32 "
                  "range");
        return SALN_E_INVALID;
    }
    HIP_TRY(hipSetDevice(ctx->device));
    auto *s = new saln_nw_span;
    s->ctx = ctx;
    s->opts = ctx->opts.effective();
    s->sc = sc;
    s->lq = (uint32_t)len_q;
    s->ld = (uint32_t)len_db;
    s->col_lo = (uint32_t)col_lo;
    s->col_hi = (uint32_t)col_hi;
    s->K = span_k(col_lo, col_hi, device_cols, s->opts);
    const uint32_t W = 64u * (uint32_t)s->K;
    s->g0 = s->col_lo / W;
    s->nst = (s->col_hi + W - 1) / W - s->g0;
    s->t0 = s->col_lo / 256;
    s->ntiles = (s->col_hi + 255) / 256 - s->t0;
    s->scol = scratch_col(s->ld);
    s->cs = ((uint64_t)s->ld + 63) * 256;  // the plan's tile stride (nw_host.cpp)
    s->mask_bytes = (uint64_t)s->ntiles * s->cs;
    s->ops_cap = (uint64_t)(s->col_hi - s->col_lo) + s->ld + 16;
    auto fail = [&](hipError_t e, const char *what) {
        set_error(std::string("span: ") + what + ": " + hipGetErrorString(e));
        s->release();
        delete s;
        return SALN_E_HIP;
    };
    hipError_t e;
    if (d_boundary) {
        s->d_bnd = (int2 *)d_boundary;
    } else {
        s->own_bnd = true;
        if ((e = dev_alloc(ctx, (void **)&s->d_bnd, (s->nst + 1) * s->scol * sizeof(int2))) != hipSuccess)
            return fail(e, "boundary columns");
    }
    NwPairDesc d;
    std::memset(&d, 0, sizeof d);
    d.len_q = s->lq;
    d.len_db = s->ld;
    d.mask_rs = 256;
    d.mask_bs = 4;
    d.mask_cs = s->cs;
    d.variant = kStripeVariant;
    std::vector<uint2> work;
    for (uint32_t t = 0; t < s->ntiles; ++t) work.push_back(make_uint2(0u, s->t0 + t));
    s->n_work = (uint32_t)work.size();
    const uint32_t err0[2] = {0u, kWaitLimitDefault};
    const uint2 blk = make_uint2(0u, 0u);
    const SpecPair sp{0u, 1u, 0u, 0u};
    if ((e = dev_alloc(ctx, (void **)&s->d_mask, s->mask_bytes + 64)) != hipSuccess)
        return fail(e, "mask");
    if ((e = dev_alloc(ctx, (void **)&s->d_pair, sizeof d)) != hipSuccess ||
        (e = hipMemcpy(s->d_pair, &d, sizeof d, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = dev_alloc(ctx, (void **)&s->d_work, work.size() * sizeof(uint2))) != hipSuccess ||
        (e = hipMemcpy(s->d_work, work.data(), work.size() * sizeof(uint2), hipMemcpyHostToDevice)) != hipSuccess ||
        (e = dev_alloc(ctx, (void **)&s->d_err, kErrWords * sizeof(uint32_t))) != hipSuccess ||
        // every XCD slot cleared: a recycled block must not hold a live epoch
        (e = hipMemset(s->d_err, 0, kErrWords * sizeof(uint32_t))) != hipSuccess ||
        (e = hipMemcpy(s->d_err, err0, sizeof err0, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = dev_alloc(ctx, (void **)&s->d_endh, sizeof(int32_t))) != hipSuccess ||
        (e = dev_alloc(ctx, (void **)&s->d_blocks, sizeof blk)) != hipSuccess ||
        (e = hipMemcpy(s->d_blocks, &blk, sizeof blk, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = dev_alloc(ctx, (void **)&s->d_sp, sizeof sp)) != hipSuccess ||
        (e = hipMemcpy(s->d_sp, &sp, sizeof sp, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = dev_alloc(ctx, (void **)&s->d_rec, 2 * sizeof(SpecStripe))) != hipSuccess ||
        (e = dev_alloc(ctx, (void **)&s->d_ops, (s->ops_cap + 8) * sizeof(uint32_t))) != hipSuccess)
        return fail(e, "tables");
    // speculative walk passes (options nw.spec, nw.spec_passes, default 3)
    // for spans of at least two walker stripes
    {
        const int passes = (int)s->opts[Opt::SpecPasses];
        if (s->opts[Opt::Spec] != 0 && passes > 0 && s->ntiles >= 2) {
            s->spec_passes = passes;
            std::vector<uint2> blocks;
            for (uint32_t t = 0; t < s->ntiles; ++t) blocks.push_back(make_uint2(0u, s->t0 + t));
            // stripe t's record at index t - t0 (span_walk_spec rebases the
            // table pointers by t0), the entry record at ntiles
            const SpecPair ssp{0u, s->ntiles, 0u, 0u};
            if ((e = dev_alloc(ctx, (void **)&s->d_sblocks, blocks.size() * sizeof(uint2))) != hipSuccess ||
                (e = hipMemcpy(s->d_sblocks, blocks.data(), blocks.size() * sizeof(uint2),
                               hipMemcpyHostToDevice)) != hipSuccess ||
                (e = dev_alloc(ctx, (void **)&s->d_ssp, sizeof ssp)) != hipSuccess ||
                (e = hipMemcpy(s->d_ssp, &ssp, sizeof ssp, hipMemcpyHostToDevice)) != hipSuccess ||
                (e = dev_alloc(ctx, (void **)&s->d_srec, (s->ntiles + 1) * sizeof(SpecStripe))) != hipSuccess ||
                (e = dev_alloc(ctx, (void **)&s->d_sops, (size_t)s->ntiles * kSpecOpsCap * sizeof(uint32_t))) != hipSuccess ||
                (e = hipHostMalloc((void **)&s->h_srec, (s->ntiles + 1) * sizeof(SpecStripe), 0)) != hipSuccess ||
                (e = hipHostMalloc((void **)&s->h_sops, (size_t)s->ntiles * kSpecOpsCap * sizeof(uint32_t), 0)) != hipSuccess)
                return fail(e, "speculative walk tables");
        }
    }
    *out = s;
    return SALN_OK;
}

int saln_nw_span_info(const saln_nw_span *s, uint64_t *mask_bytes, uint64_t *boundary_cols,
                      uint64_t *ops_cap) {
    if (!s) return SALN_E_INVALID;
    if (mask_bytes) *mask_bytes = s->mask_bytes;
    if (boundary_cols) *boundary_cols = (uint64_t)s->nst + 1;
    if (ops_cap) *ops_cap = s->ops_cap;
    return SALN_OK;
}

int saln_nw_span_boundary(const saln_nw_span *s, void **inbox, void **outbox) {
    if (!s) return SALN_E_INVALID;
    if (inbox) *inbox = s->inbox();
    if (outbox) *outbox = s->outbox();
    return SALN_OK;
}

int saln_nw_span_reset(saln_nw_span *s, void *stream) {
    if (!s) return SALN_E_INVALID;
    HIP_TRY(hipSetDevice(s->ctx->device));
    // every column: the inbox, the columns between the span's stripes, the outbox
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)s->d_bnd, (int)0x80000000u,
                              2 * (s->nst + 1) * s->scol, resolve_stream(stream, s->ctx)));
    return SALN_OK;
}

int saln_nw_span_fill(saln_nw_span *s, const uint8_t *d_q, const uint8_t *d_db, void *stream) {
    if (!s || !d_q || !d_db) return SALN_E_INVALID;
    HIP_TRY(hipSetDevice(s->ctx->device));
    HIP_TRY(launch_fill_stripes(s->d_pair, s->d_work, s->n_work, d_q, d_db, s->mask_arg(),
                                s->scratch_arg(), nullptr, s->d_err, s->d_endh, s->sc,
                                0 /* walk codes */, 2 /* row-major tiles */, s->K,
                                resolve_stream(stream, s->ctx), s->opts, ++s->fill_epoch));
    return SALN_OK;
}

int saln_nw_span_watch(saln_nw_span *s, uint64_t row_lo, uint64_t row_hi, void *stream) {
    if (!s || row_lo < 1 || row_hi > s->ld || row_lo > row_hi) return SALN_E_INVALID;
    HIP_TRY(hipSetDevice(s->ctx->device));
    HIP_TRY(launch_span_watch(s->outbox(), (uint32_t)row_lo, (uint32_t)row_hi, s->d_err,
                              resolve_stream(stream, s->ctx)));
    return SALN_OK;
}

int saln_nw_span_walk(saln_nw_span *s, const uint8_t *d_q, const uint8_t *d_db,
                      const saln_nw_span_cursor *entry, saln_nw_span_cursor *exit, uint32_t *ops,
                      uint64_t ops_cap, uint64_t *n_ops, void *stream) {
    if (!s || !d_q || !d_db || !entry || !exit || !n_ops) return SALN_E_INVALID;
    *n_ops = 0;
    if (entry->kind >= SALN_SPAN_EXIT) {  // the walk ended in a span to the right
        *exit = *entry;
        return SALN_OK;
    }
    const bool end = entry->kind == SALN_SPAN_END;
    const bool at_end = entry->i == (int32_t)s->ld && entry->j == (int32_t)s->lq;
    if (entry->kind < 0 || entry->kind > SALN_SPAN_END || (end && !at_end) ||
        entry->i < 0 || entry->i > (int32_t)s->ld || entry->j <= (int32_t)s->col_lo ||
        entry->j > (int32_t)s->col_hi) {
        set_error("span walk: entry outside the span");
        return SALN_E_INVALID;
    }
    HIP_TRY(hipSetDevice(s->ctx->device));
    hipStream_t st = resolve_stream(stream, s->ctx);
    if (s->spec_passes) {
        const int rc = span_walk_spec(s, d_q, d_db, entry, exit, ops, ops_cap, n_ops, st);
        if (rc != SALN_SPAN_UNLINKED) return rc;  // not linked: walk sequentially
    }
    SpecStripe rec[2];
    std::memset(rec, 0, sizeof rec);
    rec[0].in_k = kSpecNone;  // no stored walk to keep
    rec[1].out_i[1] = entry->i;
    rec[1].out_j[1] = entry->j;
    rec[1].out_k[1] = entry->kind;
    HIP_TRY(hipMemcpyAsync(s->d_rec, rec, sizeof rec, hipMemcpyHostToDevice, st));
    SpecArgs sa{s->d_blocks, s->d_sp, s->d_rec, s->d_ops, nullptr, 2, 1, (int32_t)s->col_lo};
    HIP_TRY(launch_span_walk(s->d_pair, sa, d_q, d_db, s->mask_arg(), s->d_endh, s->sc, st));
    HIP_TRY(hipMemcpyAsync(rec, s->d_rec, sizeof(SpecStripe), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const uint64_t n = rec[0].nops;
    if (n > s->ops_cap) {
        set_error("span walk: op stream overflow");
        return SALN_E_HIP;
    }
    if (ops && n > ops_cap) {
        set_error("span walk: ops buffer too small (saln_nw_span_info ops_cap)");
        return SALN_E_CAPACITY;
    }
    if (ops && n)
        HIP_TRY(hipMemcpy(ops, s->d_ops, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    *n_ops = n;
    exit->i = rec[0].out_i[0];
    exit->j = rec[0].out_j[0];
    exit->kind = rec[0].out_k[0];
    exit->end_states = end ? rec[0].am_end : 0u;
    return SALN_OK;
}

int saln_nw_span_score(saln_nw_span *s, int32_t *score, int32_t *status, void *stream) {
    if (!s || s->col_hi != s->lq) {
        set_error("span score: only the span holding the end cell has it");
        return SALN_E_INVALID;
    }
    HIP_TRY(hipSetDevice(s->ctx->device));
    HIP_TRY(hipStreamSynchronize(resolve_stream(stream, s->ctx)));
    int32_t h = 0;
    HIP_TRY(hipMemcpy(&h, s->d_endh, sizeof h, hipMemcpyDeviceToHost));
    if (score) *score = h >> 1;  // V' = 2V + p (make_result, nw_kernels.hip)
    if (status) *status = (h & 1) ? SALN_REF_PANIC_BOUNDARY : SALN_OK;
    return SALN_OK;
}

int saln_nw_span_status(saln_nw_span *s, uint32_t *flags) {
    if (flags) *flags = 0;
    if (!s) return SALN_E_INVALID;
    HIP_TRY(hipSetDevice(s->ctx->device));
    HIP_TRY(hipDeviceSynchronize());
    uint32_t v = 0;
    HIP_TRY(hipMemcpy(&v, s->d_err, sizeof v, hipMemcpyDeviceToHost));
    if (v) HIP_TRY(hipMemset(s->d_err, 0, sizeof v));  // read and clear
    if (flags) *flags = v;
    if (v & SALN_FLAG_WAIT_TIMEOUT) {
        set_error("span: a boundary wait timed out (the fill's results are invalid)");
        return SALN_E_DEVICE_WAIT;
    }
    return SALN_OK;
}

int saln_nw_span_set_wait_limit(saln_nw_span *s, uint32_t polls) {
    if (!s) return SALN_E_INVALID;
    HIP_TRY(hipSetDevice(s->ctx->device));
    HIP_TRY(hipMemcpy(s->d_err + 1, &polls, sizeof polls, hipMemcpyHostToDevice));
    return SALN_OK;
}

int saln_nw_span_forward(saln_nw_span *src, saln_nw_span *dst, uint64_t row_lo, uint64_t row_hi,
                         void *stream) {
    if (!src || !dst || src->ctx != dst->ctx || src->ld != dst->ld || src->col_hi != dst->col_lo ||
        row_lo < 1 || row_hi > src->ld || row_lo > row_hi)
        return SALN_E_INVALID;
    HIP_TRY(hipSetDevice(src->ctx->device));
    hipStream_t st = resolve_stream(stream, src->ctx);
    HIP_TRY(launch_span_relay(src->outbox(), dst->inbox(), (uint32_t)row_lo, (uint32_t)row_hi,
                              src->d_err, st));
    return SALN_OK;
}

int saln_nw_spans_walk(saln_nw_span *const *spans, uint32_t n, const uint8_t *d_q,
                       const uint8_t *d_db, saln_nw_span_cursor *exit, uint32_t *ops,
                       uint64_t ops_cap, uint64_t *n_ops, void *stream) {
    if (!spans || !n || !d_q || !d_db || !exit || !n_ops) return SALN_E_INVALID;
    *n_ops = 0;
    const saln_nw_span *f = spans[0];
    if (f->col_lo != 0 || spans[n - 1]->col_hi != f->lq) return SALN_E_INVALID;
    for (uint32_t r = 0; r < n; ++r) {
        const saln_nw_span *s = spans[r];
        if (s->ctx != f->ctx || s->lq != f->lq || s->ld != f->ld ||
            (r + 1 < n && s->col_hi != spans[r + 1]->col_lo))
            return SALN_E_INVALID;
        if (!s->spec_passes) return SALN_SPAN_UNLINKED;  // no speculative tables: span by span
    }
    HIP_TRY(hipSetDevice(f->ctx->device));
    hipStream_t st = resolve_stream(stream, f->ctx);
    const uint32_t T = (f->lq + 255) / 256;  // the pair's walker stripes
    const int P = f->spec_passes;
    SpecStripe *d_rec = nullptr, *h_rec = nullptr;
    uint32_t *d_ops = nullptr, *h_ops = nullptr;
    // the context's pinned staging is shared with the host-buffer entry
    // points: held from the first copy to the end of the host-side link
    std::unique_lock<std::mutex> stage_lk(f->ctx->staging_mu);
    bool queued = false;  // async work on st may still use d_rec / d_ops
    auto done = [&](int r) {
        if (queued) (void)hipStreamSynchronize(st);  // no block goes back while in use
        if (d_rec) dev_free(f->ctx, d_rec);
        if (d_ops) dev_free(f->ctx, d_ops);
        return r;
    };
    const size_t ops_words = (size_t)T * kSpecOpsCap;
    // host copies in the context's pinned staging buffer (grow-only, reused)
    const size_t rec_bytes = ((T + 1) * sizeof(SpecStripe) + 255) & ~(size_t)255;
    void *stage = nullptr;
    if (dev_alloc(f->ctx, (void **)&d_rec, (T + 1) * sizeof(SpecStripe)) != hipSuccess ||
        dev_alloc(f->ctx, (void **)&d_ops, ops_words * sizeof(uint32_t)) != hipSuccess ||
        pinned_staging(f->ctx, rec_bytes + ops_words * sizeof(uint32_t), &stage) != hipSuccess) {
        set_error("spans walk: tables");
        return done(SALN_E_HIP);
    }
    h_rec = (SpecStripe *)stage;
    h_ops = (uint32_t *)((uint8_t *)stage + rec_bytes);
    for (uint32_t t = 0; t <= T; ++t) {
        h_rec[t] = SpecStripe{};
        h_rec[t].in_k = kSpecNone;
    }
    // one record array for the pair's stripes (pair-wide index) shared by
    // every span's launch: a span's rightmost stripe reads the exit of the
    // next span's leftmost stripe from the previous pass, the pair's last
    // stripe enters at the end cell (nw_traceback_coop_kernel kSpec)
    queued = true;
    if (hipMemcpyAsync(d_rec, h_rec, (T + 1) * sizeof(SpecStripe), hipMemcpyHostToDevice, st) !=
        hipSuccess)
        return done(SALN_E_HIP);
    for (int k = 1; k <= P; ++k)
        for (uint32_t r = 0; r < n; ++r) {
            const saln_nw_span *s = spans[r];
            SpecArgs sa{s->d_sblocks, s->d_ssp, d_rec, d_ops, nullptr, k, 0, 0, 0};
            if (launch_span_spec(s->d_pair, sa, s->ntiles, k, d_q, d_db, s->mask_arg(), s->d_endh,
                                 s->sc, st, k) != hipSuccess)
                return done(SALN_E_HIP);
        }
    if (hipMemcpyAsync(h_rec, d_rec, T * sizeof(SpecStripe), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(h_ops, d_ops, ops_words * sizeof(uint32_t), hipMemcpyDeviceToHost, st) !=
            hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return done(SALN_E_HIP);
    queued = false;
    // link from the end cell's stripe leftwards (as span_walk_spec): the
    // stripes' run words in walk order, runs of one op merged at the seams
    const int cf = P & 1;
    int32_t ci = (int32_t)f->ld, cj = (int32_t)f->lq, ck = kSpecEnd;
    std::vector<uint32_t> walk;
    walk.reserve(1024);
    for (int t = (int)T - 1;; --t) {
        const SpecStripe &r = h_rec[t];
        if (r.in_i != ci || r.in_j != cj || r.in_k != ck || r.nops > kSpecOpsCap) return done(SALN_SPAN_UNLINKED);
        const uint32_t *w = h_ops + (size_t)t * kSpecOpsCap;
        for (uint32_t k = 0; k < r.nops; ++k) {
            if ((w[k] >> 4) == 0) continue;  // empty run
            if (!walk.empty() && (walk.back() & 15u) == (w[k] & 15u))
                walk.back() += w[k] & ~15u;
            else
                walk.push_back(w[k]);
        }
        ci = r.out_i[cf];
        cj = r.out_j[cf];
        ck = r.out_k[cf];
        if (ck >= kSpecEv || t == 0) break;
    }
    const uint64_t nw = walk.size();
    const uint32_t es = h_rec[T - 1].am_end;
    // not ended at column 0, or a dead end with tied end states left (the
    // span-by-span walk restarts in the next state): walk span by span
    if (ck < kSpecEv || ck == kSpecNone ||
        (ck - kSpecEv == 2 /* dead */ && (es & ~(uint32_t)(es & 4u ? 4u : es & 1u ? 1u : 2u))))
        return done(SALN_SPAN_UNLINKED);
    if (ops && nw > ops_cap) {
        set_error("spans walk: CIGAR buffer too small");
        return done(SALN_E_CAPACITY);
    }
    if (ops)  // forward order: the CIGAR
        for (uint64_t k = 0; k < nw; ++k) ops[k] = walk[nw - 1 - k];
    *n_ops = nw;
    exit->i = ci;
    exit->j = cj;
    exit->kind = ck;
    exit->end_states = es;
    return done(SALN_OK);
}

int saln_device_cu_count(saln_context *ctx, uint32_t *n) {
    if (!ctx || !n) return SALN_E_INVALID;
    int v = 0;
    HIP_TRY(hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, ctx->device));
    *n = (uint32_t)v;
    return SALN_OK;
}

// CU mask bit c selects a CU of XCD c mod n_xcd (measured on MI355X with
// saln_device_cu_probe, tools/cu_map.py -> profiles/r04_cu_map.json: every
// contiguous range of 8k bits holds k CUs of each XCD, spread over its shader
// engines), so a contiguous range is XCD-balanced by construction.  An XCD
// whose bits are all clear is NOT idle: the mask is applied per XCD and an
// empty per-XCD mask runs that XCD unmasked (one bit gave 225 CUs).  Ranges
// that leave an XCD without a bit are refused for that reason.
int saln_stream_create_cu_range(saln_context *ctx, uint32_t cu_lo, uint32_t cu_hi, void **stream) {
    if (!ctx || !stream || cu_lo >= cu_hi) return SALN_E_INVALID;
    uint32_t n = 0;
    const int rc = saln_device_cu_count(ctx, &n);
    if (rc != SALN_OK) return rc;
    if (cu_hi > n) return SALN_E_INVALID;
    HIP_TRY(hipSetDevice(ctx->device));
    int n_xcd = 1;
    if (hipDeviceGetAttribute(&n_xcd, hipDeviceAttributeNumberOfXccs, ctx->device) != hipSuccess ||
        n_xcd < 1)
        n_xcd = 1;
    if (cu_hi - cu_lo < (uint32_t)n_xcd) {
        set_error("saln_stream_create_cu_range: a range of fewer than " + std::to_string(n_xcd) +
                  " CUs leaves an XCD without a mask bit, and that XCD would run unmasked");
        return SALN_E_INVALID;
    }
    std::vector<uint32_t> mask((n + 31) / 32, 0u);
    for (uint32_t c = cu_lo; c < cu_hi; ++c) mask[c / 32] |= 1u << (c % 32);
    hipStream_t s = nullptr;
    HIP_TRY(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    *stream = s;
    return SALN_OK;
}

int saln_device_cu_probe(saln_context *ctx, void *stream, uint32_t n_blocks, uint32_t *hw_id,
                         uint32_t *xcc_id) {
    if (!ctx || !hw_id || !xcc_id || !n_blocks) return SALN_E_INVALID;
    HIP_TRY(hipSetDevice(ctx->device));
    uint32_t *d = nullptr;
    HIP_TRY(dev_alloc(ctx, (void **)&d, 2ull * n_blocks * sizeof(uint32_t)));
    hipStream_t st = resolve_stream(stream, ctx);
    hipError_t e = launch_cu_probe(n_blocks, d, d + n_blocks, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess) e = hipMemcpy(hw_id, d, n_blocks * sizeof(uint32_t), hipMemcpyDeviceToHost);
    if (e == hipSuccess)
        e = hipMemcpy(xcc_id, d + n_blocks, n_blocks * sizeof(uint32_t), hipMemcpyDeviceToHost);
    (void)hipStreamSynchronize(st);
    dev_free(ctx, d);
    HIP_TRY(e);
    return SALN_OK;
}

int saln_stream_create_cu_mask(saln_context *ctx, const uint32_t *mask, uint32_t n_words,
                               void **stream) {
    if (!ctx || !mask || !n_words || !stream) return SALN_E_INVALID;
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = nullptr;
    HIP_TRY(hipExtStreamCreateWithCUMask(&s, n_words, mask));
    *stream = s;
    return SALN_OK;
}

int saln_stream_destroy(saln_context *ctx, void *stream) {
    if (!ctx || !stream) return SALN_E_INVALID;
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipStreamDestroy((hipStream_t)stream));
    return SALN_OK;
}

int saln_nw_span_destroy(saln_nw_span *s) {
    if (!s) return SALN_OK;
    (void)hipSetDevice(s->ctx->device);
    (void)hipDeviceSynchronize();
    s->release();
    delete s;
    return SALN_OK;
}

}  // extern "C"

// Host-side pieces shared by the C ABI and the CLI.
#pragma once
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "nw_common.hpp"
#include "saln_options.hpp"
#include "saln.h"

struct saln_context {
    int device = 0;
    saln::OptOverrides opts;  // saln_context_option_set (on top of the process registry)
    hipStream_t stream = nullptr;
    hipStream_t tb_stream = nullptr;  // traceback stream (pipelined NW plans)
    // Device blocks released by plans / host-path calls, kept for reuse
    // (hipMalloc + hipFree of a 3 GB mask workspace cost more than the C2
    // kernels): size -> block; `live` maps handed-out blocks to their size.
    std::mutex mu;
    std::multimap<size_t, void *> cache;
    std::unordered_map<void *, size_t> live;
    size_t cached = 0;
    // pinned host staging for the host-path downloads (grow-only); staging_mu
    // is held by a user of the buffer from its first copy to its last host
    // read (pinned_staging may free and reallocate it when it grows)
    std::mutex staging_mu;
    void *pinned = nullptr;
    size_t pinned_bytes = 0;
    // pageable host copy of render batches' mask workspaces (grow-only,
    // uninitialised, 2 MB-aligned with transparent huge pages requested: the
    // first copy into 1.1 GB of 4 KB pages spent ~0.17 s in page faults; under
    // staging_mu): pinning a GB-sized buffer costs more than the copy it
    // speeds up (measured: 333 ms to pin, 234 ms to unpin 1.1 GB)
    struct HostBuf {
        uint8_t *p = nullptr;
        size_t n = 0;
        ~HostBuf() { std::free(p); }
    } host_mask;
};

// A C-ABI stream argument: NULL = the context's own (non-blocking) stream;
// hipStreamLegacy = the legacy null stream (torch's default stream), used as
// the handle 0 that every HIP call accepts; anything else as given.
inline hipStream_t resolve_stream(void *stream, const saln_context *ctx) {
    if (!stream) return ctx->stream;
    if ((hipStream_t)stream == hipStreamLegacy) return (hipStream_t)0;
    return (hipStream_t)stream;
}


namespace saln {

// option host.timing = 1: stage times of the host-side paths on stderr
struct StageClock {
    bool on;
    explicit StageClock(const Options &o) : on(o[Opt::HostTiming] != 0) {}
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(const char *what) {
        if (!on) return;
        (void)hipDeviceSynchronize();
        const auto n = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[saln host] %-16s %8.3f ms\n", what,
                     std::chrono::duration<double, std::milli>(n - t).count());
        t = n;
    }
};

// Context-cached device memory: a released block is reused by a later request
// of at most twice its size; at most kDevCacheMax bytes stay cached.  A block
// must not be released while kernels may still use it (plan destroy syncs).
constexpr size_t kDevCacheMax = size_t(32) << 30;
hipError_t dev_alloc(saln_context *ctx, void **p, size_t n);
void dev_free(saln_context *ctx, void *p);
void dev_cache_clear(saln_context *ctx);
hipError_t pinned_staging(saln_context *ctx, size_t n, void **p);  // caller holds ctx->staging_mu

// kernels (nw_kernels.hip)
// What a packed fill launch needs besides the pairs: the plan's options, the
// workspace's bail word and the launch's epoch (4-bit-code table fills: the
// fallback launch runs only when a wave of its table launch left pairs to it).
// deferred: when set, the fallback launch is appended there instead of being
// queued behind the table launch, for the caller to queue on the stream that
// walks the workspace once the fills are done (pipelined plans: the fill
// stream then runs the next step's fill without it in between).
struct FillExtras {
    const Options *o = nullptr;
    uint32_t *bail = nullptr;
    uint32_t epoch = 0;
    std::vector<std::function<hipError_t(hipStream_t)>> *deferred = nullptr;
};
hipError_t launch_fill(int variant, const NwPairDesc *pairs, uint32_t first, uint32_t count,
                       const uint8_t *qs, const uint8_t *ds, uint8_t *mask, int2 *scratch,
                       int32_t *end_h, saln_nw_result *results, uint32_t *cigar, Scoring sc,
                       int codes /* 0 walk, 1 full, 2 none, 3 4-bit walk */, uint32_t ld_max,
                       hipStream_t stream, const FillExtras &fx);
hipError_t launch_fill_stripes(const NwPairDesc *pairs, const uint2 *work, uint32_t n_work,
                               const uint8_t *qs, const uint8_t *ds, uint8_t *mask,
                               int2 *scratch, uint32_t *prog, uint32_t *err, int32_t *end_h,
                               Scoring sc, int codes /* 0 walk, 1 full, 2 none */,
                               int layout /* 0 skewed, 1 packed, 2 row-major tiles */,
                               int rows_k /* layout 2: columns per lane */, hipStream_t stream,
                               const Options &o, uint32_t epoch);
// err buffer of a stripe fill: [device error flags, wait limit, kXcdSlots
// slots] - the row fill's XCD runs post {epoch, XCC_ID} per wave there, so a
// launch needs an epoch its buffer has not seen (1, 2, ...)
constexpr uint32_t kXcdSlots = 1024;
constexpr size_t kErrWords = 2 + kXcdSlots;
// render batches: the reference DFS's event after each pair's first printed
// alignment (full-code plans; next[pair_id]: 0 none, 1 block, 2 panic, 3 host)
hipError_t launch_next_event(const NwPairDesc *pairs, uint32_t n, const uint8_t *mask,
                             const saln_nw_result *results, Scoring sc, uint8_t *next,
                             hipStream_t stream);
hipError_t launch_cigar_compact(const saln_nw_result *res, const uint64_t *src_off,
                                const uint64_t *dst_off, const uint32_t *src, uint32_t *dst,
                                uint64_t n, hipStream_t stream);
constexpr int kStripeVariant = 3;
// column-stripe pairs: boundary columns allocated per pair (the row fill cuts
// each 256-column chunk into up to 4 stripes)
constexpr uint32_t kStripeSubMax = 4;
// row fill (nw_fill_rows_kernel) columns per lane, 0 = the skewed stripe fill;
// waves_k1: the plan's stripe waves at one column per lane
int stripe_rows_k(uint64_t waves_k1, const Options &o);
// column stripes run the packed (int16 halves) fill for this scoring and
// this many stripe waves in the plan (decided once per plan: it sets the layout)
bool stripe_packed(const Scoring &sc, uint64_t n_waves, bool wide, const Options &o);
constexpr int kWidePackedVariant = 8;        // packed, 64-lane groups, up to 1,024 columns
constexpr uint64_t kWidePackedMinPairs = 1536;  // fewer such pairs: column stripes (measured crossover 1,024-2,048)
hipError_t launch_score_results(const NwPairDesc *pairs, uint32_t first, uint32_t n,
                                const int32_t *end_h, saln_nw_result *results, Scoring sc,
                                hipStream_t stream);
hipError_t launch_traceback(int variant, const NwPairDesc *pairs, uint32_t first, uint32_t n,
                            const uint8_t *qs,
                            const uint8_t *ds, const uint8_t *mask, const int32_t *end_h,
                            uint32_t *ops, saln_nw_result *results, uint32_t *cigar, Scoring sc,
                            int stripe_layout, hipStream_t stream,
                            const uint32_t *spec_done = nullptr, bool nib = false,
                            uint32_t walk_waves = 0);
// variants whose walk codes may be 4-bit (kCodesNib): the short-query packed
// fills 7 (16 x 10) and 4 (8 x 19, 4-bit only)
inline bool variant_nib(int v) { return v == 7 || v == 4; }
constexpr int kNarrowVariant = 4;  // 8 x 19 groups, queries of <= 152 columns
// speculative stripe walks of the plan's long column-stripe pairs: `passes`
// walk passes, the link (accept or leave to the cooperative walker, `done`)
// and the CIGAR copy; strict_err (SALN_SPEC_STRICT=1, tests): bit 1 set when a
// pair did not link
hipError_t launch_traceback_spec(const NwPairDesc *pairs, SpecArgs sa, uint32_t n_blocks,
                                 uint32_t n_spec_pairs, uint32_t *done, int passes,
                                 const uint8_t *qs, const uint8_t *ds, const uint8_t *mask,
                                 const int32_t *end_h, saln_nw_result *results, uint32_t *cigar,
                                 Scoring sc, int stripe_layout, uint32_t *strict_err,
                                 hipStream_t stream);
// column spans of one long pair (nw_span.cpp): one walk from sa.stripes[1]'s
// pass-2 exit slot, and a wait for published rows of a boundary column
hipError_t launch_span_walk(const NwPairDesc *pairs, SpecArgs sa, const uint8_t *qs,
                            const uint8_t *ds, const uint8_t *mask, const int32_t *end_h,
                            Scoring sc, hipStream_t stream);
hipError_t launch_span_watch(const int2 *col, uint32_t r0, uint32_t r1, uint32_t *err,
                             hipStream_t stream);
hipError_t launch_cu_probe(uint32_t n_blocks, uint32_t *hw, uint32_t *xcc, hipStream_t stream);
hipError_t launch_span_relay(const int2 *src, int2 *dst, uint32_t r0, uint32_t r1, uint32_t *err,
                             hipStream_t stream);
hipError_t launch_span_spec(const NwPairDesc *pairs, SpecArgs sa, uint32_t n_blocks, int passes,
                            const uint8_t *qs, const uint8_t *ds, const uint8_t *mask,
                            const int32_t *end_h, Scoring sc, hipStream_t stream,
                            int pass_lo = 1);
// score-only all-vs-all (nw_avsa.cpp); avsa_chunk_pairs: the most pairs one
// launch of a packed class may take (0: not a packed variant)
uint64_t avsa_chunk_pairs(int variant);
uint64_t avsa_launch_blocks(int variant, uint64_t count);  // workgroups of one launch
hipError_t launch_avsa_prof(const uint64_t *q_off, const uint64_t *d_off, const uint32_t *q_ids,
                            uint32_t nq, const uint32_t *d_ids, uint32_t nq_total, uint64_t base,
                            uint32_t count, const uint8_t *qs, const uint8_t *ds, int2 *out,
                            Scoring sc, uint32_t ld_max, const uint32_t *generic,
                            hipStream_t stream, const Options &o);
hipError_t launch_acgt_check(const uint8_t *seq, uint64_t n, uint32_t *flag, hipStream_t stream);
hipError_t launch_avsa(int variant, const uint64_t *q_off, const uint64_t *d_off,
                       const uint32_t *q_ids, uint32_t nq, const uint32_t *d_ids,
                       uint32_t nq_total, uint64_t base, uint32_t count, const uint8_t *qs,
                       const uint8_t *ds, int2 *out, Scoring sc, uint32_t ld_max,
                       hipStream_t stream, const Options &o, const uint32_t *generic = nullptr);
hipError_t launch_avsa_boundary(const uint64_t *q_off, const uint64_t *d_off,
                                const uint32_t *q_ids, uint32_t nq, const uint32_t *d_ids,
                                uint64_t n, uint32_t nq_total, int2 *out, Scoring sc,
                                hipStream_t stream);
hipError_t launch_avsa_scatter(const saln_nw_result *res, const uint32_t *q_ids, uint32_t nq,
                               const uint32_t *d_ids, uint64_t n, uint32_t nq_total, int2 *out,
                               hipStream_t stream);
Geom variant_geom(int v);
bool variant_packed(int v);
int choose_variant(uint32_t len_q, uint32_t len_db, const Scoring &sc, bool narrow = false);

void set_error(const std::string &msg);
Scoring scoring_or_default(const saln_nw_scoring *s);

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) {                                                            \
            ::saln::set_error(std::string(#expr) + ": " + hipGetErrorString(e_));          \
            return SALN_E_HIP;                                                             \
        }                                                                                  \
    } while (0)

// Host copy of one pair's parent codes: LB-byte segments, row-major, with
// row stride rs and block stride bs (nw_common.hpp Geom).
struct PairMask {
    std::vector<uint8_t> m;
    Geom g{16, 10};
    uint64_t rs = 0;
    uint32_t bs = 0;
    uint64_t cs = 0;
};

// Random access to one pair's parent codes (kernel layout + boundary rules).
struct HostMask {
    const uint8_t *m = nullptr;  // pair's mask bytes (host copy)
    Geom g{16, 10};
    uint64_t rs = 0;
    uint32_t bs = 0;
    uint64_t cs = 0;
    uint32_t lq = 0, ld = 0;
    Scoring sc{5, -4, -8, -6};
    HostMask() = default;
    HostMask(const PairMask &pm, uint32_t lq_, uint32_t ld_, const Scoring &sc_)
        : m(pm.m.data()), g(pm.g), rs(pm.rs), bs(pm.bs), cs(pm.cs), lq(lq_), ld(ld_), sc(sc_) {}
    // codes are stored inverted (bit set = parent absent)
    uint8_t byte(uint32_t i, uint32_t j) const { return m[g.cell(i, j, rs, bs, cs)] ^ 0x7F; }
    uint8_t argmax(uint32_t i, uint32_t j) const {
        if (i == 0) return argmax_row0(sc, j);
        if (j == 0) return argmax_col0(sc, i);
        return byte(i, j) & 7;
    }
    uint8_t ibits(uint32_t i, uint32_t j) const {
        return j == 1 ? ibits_col1(sc, i) : (byte(i, j - 1) >> 3) & 3;
    }
    uint8_t dbits(uint32_t i, uint32_t j) const {
        return i == 1 ? dbits_row1(sc, j) : (byte(i - 1, j) >> 5) & 3;
    }
    // Dense export (include/saln.h saln_nw_dense_mask).
    void to_dense(uint8_t *out) const;
};

// saln_nw_plan_status without the flags: SALN_E_DEVICE_WAIT if a column-stripe
// fill hit its dependency-wait bound since the last check.
int plan_check_error(saln_nw_plan *plan);

// saln_nw_plan_create with the code format fixed at creation: full_codes =
// every parent set (needed by the host DFS and the dense export) instead of
// the walk codes a plan stores by default.
int plan_create(saln_context *ctx, const uint64_t *q_off, uint64_t n_q, const uint64_t *db_off,
                uint64_t n_db, const uint32_t *pair_q, const uint32_t *pair_db, uint64_t n_pairs,
                int32_t mode, const saln_nw_scoring *scoring, bool full_codes, saln_nw_plan **out);

// Render batches: the reference DFS's event after each pair's first printed
// alignment, for every pair of a full-code plan after its execute
// (nw_next_event_kernel; d_next[results index]: kNext* of nw_kernels.hip).
int plan_next_event(saln_nw_plan *plan, const saln_nw_result *d_results, uint8_t *d_next,
                    hipStream_t stream);
enum { kNextNone = 0, kNextBlock = 1, kNextPanic = 2, kNextHost = 3 };

// Copies one pair's parent codes from a plan's workspace after execute
// (compact: bs = LB); pair_id is the results index.
int plan_pair_mask(const saln_nw_plan *plan, uint64_t pair_id, PairMask *mask);

// A full-code plan's mask workspace for host reads (render batches: one
// streamed download instead of a copy per pair): the device base, the end of
// pair pair_id's bytes in it (results index; 0 for an empty pair), and a
// pair's view on a host copy of the workspace prefix that holds it.
int plan_mask_source(const saln_nw_plan *plan, const uint8_t **d_mask);
uint64_t plan_mask_end(const saln_nw_plan *plan, uint64_t pair_id);
HostMask plan_host_mask(const saln_nw_plan *plan, const uint8_t *host, uint64_t pair_id);

// Reference DFS (needleman_wunsch_affine.rs:246-329) over the parent codes.
struct DfsOutcome {
    uint64_t blocks = 0;
    int32_t status = SALN_OK;  // SALN_OK | SALN_REF_PANIC_BOUNDARY | SALN_ENUM_CAP
};
// Prints every block (reference text, no timing line) until panic / cap.
DfsOutcome render_blocks(const HostMask &hm, const uint8_t *q, const uint8_t *d,
                         uint64_t max_blocks, std::string *out);
// First printed alignment with backtracking over sentinel dead ends.
// Returns true if one is printed; cigar gets forward RLE words.
bool first_alignment(const HostMask &hm, const uint8_t *q, const uint8_t *d,
                     std::vector<uint32_t> *cigar);

}  // namespace saln

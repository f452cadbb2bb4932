/*
 * saln — MI355X-native drop-in engine for the NW-affine (and WFA) hot path of
 * Qw11111111111/SequenceAligning.
 *
 * C ABI only: plain pointers, sizes and POD structs; no C++ or torch types.
 * Every entry point names the reference interface it replaces.  The
 * reference is Rust (src/main.rs dispatches to free functions), so the
 * binding a maintainer adds is an `extern "C"` block in Rust — see
 * INTEGRATION.md.
 *
 * Orientation (reference convention, needleman_wunsch_affine.rs:424-430):
 *   seq1 = query  -> y, columns, inner loop
 *   seq2 = db     -> x, rows,    outer loop
 */
#ifndef SALN_H
#define SALN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SALN_ABI_VERSION 1

/* Mode — src/parse.rs:44-50 (declaration order Global, Local, SemiGlobal). */
typedef enum {
    SALN_MODE_GLOBAL = 0,
    SALN_MODE_LOCAL = 1,
    SALN_MODE_SEMI_GLOBAL = 2
} saln_mode;

/* Per-pair status and API return codes.  The reference returns
 * AlignerError values (src/errors.rs:7-15) or panics (aborting the whole
 * process, exit 101); this library never aborts and reports a status instead. */
typedef enum {
    SALN_OK = 0,
    SALN_NOT_IMPLEMENTED = 1,    /* AlignmentError("not implemented"): NW :433-434, WFA :26 */
    SALN_REF_PANIC_BOUNDARY = 2, /* NW traceback index panic, needleman_wunsch_affine.rs:299/:303 */
    SALN_REF_PANIC_TRIM = 3,     /* WFA Ocean::trim rotate_left panic, wfa.rs:577/:603 */
    SALN_REF_PANIC_SLICE = 4,    /* WFA rec_tr slice panic, wfa.rs:695-744 */
    SALN_NONCONVERGED = 5,       /* WFA score loop hit the caller's step cap (wfa.rs:28) */
    SALN_ENUM_CAP = 6,           /* NW co-optimal enumeration hit the caller's cap */
    SALN_SPAN_UNLINKED = 7,      /* saln_nw_spans_walk only: the speculative passes did not
                                    link; walk span by span (saln_nw_span_walk) */

    SALN_E_INVALID = -1,   /* bad argument */
    SALN_E_HIP = -2,       /* HIP runtime error (message: saln_last_error) */
    SALN_E_NO_DEVICE = -3, /* no gfx950 device / extension not usable */
    SALN_E_CAPACITY = -4,  /* caller buffer too small */
    SALN_E_IO = -5,        /* file could not be read */
    SALN_E_FASTA = -6,     /* AlignerError::FastaError (bad extension), parse.rs:55-60 */
    SALN_E_FASTA_CHARS = -7, /* AlignerError::CharError; records are still returned, parse.rs:92-97 */
    SALN_E_DEVICE_WAIT = -8  /* a kernel's inter-workgroup dependency wait gave up: the results
                                of the executes since the last status check are invalid
                                (saln_nw_plan_status; message: saln_last_error) */
} saln_status;

/* Device error flags (saln_nw_plan_status, saln_nw_avsa_status). */
#define SALN_FLAG_WAIT_TIMEOUT 1u  /* a column-stripe fill's wait for its left neighbour's
                                      boundary rows exceeded the plan's wait limit */
#define SALN_FLAG_SPEC_UNLINKED 2u /* tests only (option nw.spec_strict = 1): a speculative
                                      stripe walk fell back to the sequential walker */

/* ScoringScheme, needleman_wunsch_affine.rs:15-20 / :382-388.
 * NULL everywhere means the reference SCHEME {5, -4, -8, -6}. */
typedef struct {
    int32_t match;      /* +5 */
    int32_t mismatch;   /* -4 */
    int32_t gap_open;   /* -8 (added once when a gap opens from M) */
    int32_t gap_extend; /* -6 (added for every gap column) */
} saln_nw_scoring;

/* Result of one NW pair (16 bytes). */
typedef struct {
    int32_t score;      /* max(M,I,D)[len_db][len_q], :247-250 (never printed by the reference) */
    int32_t status;     /* SALN_OK | SALN_REF_PANIC_BOUNDARY | SALN_NOT_IMPLEMENTED */
    uint32_t cigar_len; /* RLE ops written for the first printed alignment (0 if none) */
    uint8_t end_states; /* bit0 M, bit1 I, bit2 D: end states equal to score (:251-280) */
    uint8_t printed;    /* 1 if the reference prints at least one alignment block; 0 when
                           its DFS panics first or every co-optimal path is
                           sentinel-rooted (dropped silently, :172-216) */
    uint8_t flags;      /* bit 3: score-only result; bit 1: internal inconsistency
                           (never set); all other bits 0 */
    uint8_t reserved;
} saln_nw_result;

/* CIGAR words: (run_length << 4) | op, BAM op codes, forward order, db as
 * the reference sequence:  '=' 7 (M column, bases equal), 'X' 8 (M column,
 * bases differ), 'I' 1 (query base vs '-', I state), 'D' 2 ('-' vs db base,
 * D state).  A run never exceeds 2^28-1. */
#define SALN_CIGAR_EQ 7u
#define SALN_CIGAR_X 8u
#define SALN_CIGAR_I 1u
#define SALN_CIGAR_D 2u

/* ---------------------------------------------------------------- context */
typedef struct saln_context saln_context;

/* Creates a context bound to HIP device `device` (one stream per context;
 * reentrant per context, not shared across threads).  Fails with
 * SALN_E_NO_DEVICE if no gfx950 device is present: there is no CPU path.
 * Device blocks released by plans and host-buffer calls stay cached in the
 * context (up to 32 GiB, reused by later requests of up to twice the size)
 * until saln_context_destroy; an allocation that fails drops the cache and
 * retries once. */
int saln_context_create(int device, saln_context **out);
int saln_context_destroy(saln_context *ctx);
const char *saln_last_error(void);     /* thread-local message for the last error */
int saln_abi_version(void);

/* ---------------------------------------------------------------- options
 * Tuning knobs (kernel geometry and A/B variants), all with the product's
 * defaults.  No reference counterpart: the reference has no tuning (its
 * constants are compile-time, needleman_wunsch_affine.rs:15-20).  The engine
 * reads nothing from the process environment; these calls are the only way
 * to change what it runs.  Every option gives the same results.  Names:
 * "nw.wide_min_pairs", "nw.rows_k", "nw.stripe_pk", "nw.spec",
 * "nw.spec_passes", "nw.spec_strict", "nw.avsa_narrow", "nw.rows_lone",
 * "nw.rows_xcd", "nw.avsa_profile", "nw.pk_tab", "nw.walk_waves",
 * "wfa2.seq_lds", "wfa2.w1", "wfa2.w2", "host.timing", "host.prefault_mb".
 * Two levels, no other shared state:
 *  - saln_option_*: the process registry, the default of every context;
 *  - saln_context_option_*: overrides of one context (its own thread's
 *    choices; another context is not affected).
 * A plan, all-vs-all handle, span or host-buffer call takes its context's
 * effective values when it is created (or called); a later change does not
 * reach it.  SALN_E_INVALID for an unknown name or a value out of range. */
int saln_option_set(const char *name, int64_t value);
int saln_option_get(const char *name, int64_t *value, int64_t *default_value);
/* Name of option `index` (0, 1, ...; SALN_E_INVALID past the last). */
int saln_option_name(uint32_t index, const char **name);
/* Every option of the registry back to its default. */
int saln_options_reset(void);
/* One context's override; _get returns the context's effective value; _clear
 * drops one override (name) or all of them (name NULL). */
int saln_context_option_set(saln_context *ctx, const char *name, int64_t value);
int saln_context_option_get(saln_context *ctx, const char *name, int64_t *value);
int saln_context_option_clear(saln_context *ctx, const char *name);

/* ------------------------------------------------------- NW: per pair (drop-in)
 * Replaces `pub fn n_w_align(seq1: &Record, seq2: &Record, _verbose: bool,
 * mode: Mode) -> Result<()>` (needleman_wunsch_affine.rs:424-437).
 * q = seq1.seq (query), d = seq2.seq (db).  `verbose` is ignored, as in the
 * reference.  cigar (capacity cigar_cap words) may be NULL.
 * Returns SALN_OK or SALN_NOT_IMPLEMENTED (mode != GLOBAL, like :433-434) or
 * an SALN_E_* error; the per-pair outcome (incl. reference panics) is in
 * out->status. */
int saln_nw_align(saln_context *ctx, const uint8_t *q, uint64_t len_q, const uint8_t *d,
                  uint64_t len_db, int verbose, int32_t mode, const saln_nw_scoring *scoring,
                  saln_nw_result *out, uint32_t *cigar, uint64_t cigar_cap);

/* Text the reference prints for this pair (needleman_wunsch_affine.rs:281-286
 * with TraceBackInfo Display :390-411): every co-optimal alignment block in
 * the reference's DFS order, up to the first panic.  The nondeterministic
 * `{:#?}` timing line (:431) is not produced.  max_blocks = 0: unlimited.
 * *status: SALN_OK, SALN_REF_PANIC_BOUNDARY (the reference would abort after
 * the returned text) or SALN_ENUM_CAP.  out may be NULL to query *out_len. */
int saln_nw_render(saln_context *ctx, const uint8_t *q, uint64_t len_q, const uint8_t *d,
                   uint64_t len_db, int32_t mode, uint64_t max_blocks, char *out, uint64_t cap,
                   uint64_t *out_len, uint64_t *n_blocks, int32_t *status);

/* The same text for a batch, each pair computed once (the drop-in CLI and
 * hosts that print per pair).  Replaces the pair loop main.rs:61-74 with the
 * text every n_w_align call prints: one plan for all pairs (same CSR / pair
 * conventions as saln_nw_align_batch; NULL pair lists = all-vs-all, db outer).
 * The GPU walks each pair's first printed alignment and decides what the
 * reference DFS meets after it; pairs whose text that settles (no block,
 * exactly one block, or with max_blocks = 1 the first block and then the cap
 * or the panic) are rendered from that walk, the others by the reference DFS
 * on host threads over their parent codes.  The text stays in the
 * returned handle until saln_nw_text_free.  stop_at_panic = 1: pairs after
 * the first one whose traceback panics (REF_PANIC_BOUNDARY) are not rendered
 * - the reference aborts there (exit 101) - so saln_nw_text_count is that
 * pair's index + 1.  mode != GLOBAL: every pair SALN_NOT_IMPLEMENTED with no
 * text (main.rs:68-74 prints the error and goes on). */
typedef struct saln_nw_text saln_nw_text;
int saln_nw_render_batch(saln_context *ctx, const uint8_t *q_seq, const uint64_t *q_off,
                         uint64_t n_q, const uint8_t *db_seq, const uint64_t *db_off,
                         uint64_t n_db, const uint32_t *pair_q, const uint32_t *pair_db,
                         uint64_t n_pairs, int32_t mode, uint64_t max_blocks, int stop_at_panic,
                         saln_nw_text **out);
/* One pair in one call: saln_nw_render_batch of (q, d). */
int saln_nw_render_text(saln_context *ctx, const uint8_t *q, uint64_t len_q, const uint8_t *d,
                        uint64_t len_db, int32_t mode, uint64_t max_blocks, saln_nw_text **out);
uint64_t saln_nw_text_count(const saln_nw_text *t);
/* Of those pairs, the ones rendered from the GPU's walk alone (no parent-code
 * download, no host DFS). */
uint64_t saln_nw_text_gpu_decided(const saln_nw_text *t);
/* Pair `pair` (< count): its text (valid until free; not NUL-terminated), the
 * blocks printed, the render status (SALN_OK, SALN_REF_PANIC_BOUNDARY after
 * the text, SALN_ENUM_CAP, SALN_NOT_IMPLEMENTED), its saln_nw_result, and
 * its wall time (its DFS plus its share of the batch's device work).  Any
 * output pointer may be NULL. */
int saln_nw_text_get(const saln_nw_text *t, uint64_t pair, const char **text, uint64_t *len,
                     uint64_t *n_blocks, int32_t *status, saln_nw_result *result,
                     uint64_t *elapsed_ns);
void saln_nw_text_free(saln_nw_text *t);

/* Dense parent mask for parity checks: (len_db+1) x (len_q+1) bytes,
 * row-major over db.  Byte bits: 0-2 = {M,I,D} equal to max(M,I,D) at the
 * cell (so the M parent set of (x,y) is the byte of (x-1,y-1)), 3-4 = I
 * parents {extend I[x][y-1], open M[x][y-1]}, 5-6 = D parents {extend
 * D[x-1][y], open M[x-1][y]} (needleman_wunsch_affine.rs:96-153, boundary
 * parents :196,:208). */
int saln_nw_dense_mask(saln_context *ctx, const uint8_t *q, uint64_t len_q, const uint8_t *d,
                       uint64_t len_db, const saln_nw_scoring *scoring, uint8_t *out);

/* --------------------------------------------------------- NW: batched (host)
 * Replaces the pair loop `for d in db { for q in query { n_w_align(q, d) } }`
 * (main.rs:61-67).  Sequences are CSR: q_seq bytes with q_off[n_q+1].  Pair p
 * aligns query pair_q[p] against db pair_db[p]; if pair_q == pair_db == NULL,
 * all-vs-all in the reference order (db outer, query inner:
 * p = d * n_q + q).  cigar/cigar_off may be NULL; cigar_off[p] (words) must
 * leave room for len_q + len_db words per pair (saln_nw_cigar_offsets). */
int saln_nw_align_batch(saln_context *ctx, const uint8_t *q_seq, const uint64_t *q_off,
                        uint64_t n_q, const uint8_t *db_seq, const uint64_t *db_off,
                        uint64_t n_db, const uint32_t *pair_q, const uint32_t *pair_db,
                        uint64_t n_pairs, int32_t mode, const saln_nw_scoring *scoring,
                        saln_nw_result *results, uint32_t *cigar, const uint64_t *cigar_off);

/* -------------------------------------------------- NW: batched (device, plan)
 * For callers whose data is already resident in HBM (bench, multi-GPU
 * driver).  The plan is built once from host-side lengths; execute then only
 * launches kernels on `stream` (hipStream_t; NULL = the context's own
 * non-blocking stream; pass hipStreamLegacy for the legacy null stream).
 * Device buffers: q_seq/db_seq (same CSR byte layout as the host offsets
 * given to the plan), results[n_pairs], cigar[plan cigar words] (may be
 * NULL: traceback still runs, ops are not stored). */
typedef struct saln_nw_plan saln_nw_plan;

int saln_nw_plan_create(saln_context *ctx, const uint64_t *q_off, uint64_t n_q,
                        const uint64_t *db_off, uint64_t n_db, const uint32_t *pair_q,
                        const uint32_t *pair_db, uint64_t n_pairs, int32_t mode,
                        const saln_nw_scoring *scoring, saln_nw_plan **out);
/* The same plan storing the reference's full parent sets: one byte per cell
 * (7 parent bits: the {M,I,D} argmax set and the I / D extend/open parents,
 * needleman_wunsch_affine.rs:96-153 - what the all-blocks DFS :281-329
 * consumes), instead of the walk codes saln_nw_plan_create's fills store.
 * Execute fills, walks and writes the first printed CIGAR as before;
 * saln_nw_plan_dense_mask reads a pair's parent sets back. */
int saln_nw_plan_create_full(saln_context *ctx, const uint64_t *q_off, uint64_t n_q,
                             const uint64_t *db_off, uint64_t n_db, const uint32_t *pair_q,
                             const uint32_t *pair_db, uint64_t n_pairs, int32_t mode,
                             const saln_nw_scoring *scoring, saln_nw_plan **out);
/* Pair `pair`'s parent sets from the last execute of a synchronous full plan
 * (waits for it), as saln_nw_dense_mask lays them out: (len_db+1) x (len_q+1)
 * bytes. */
int saln_nw_plan_dense_mask(saln_nw_plan *plan, uint64_t pair, uint8_t *out);
/* The 4-bit walk codes a (non-full) plan's short-query fills store for pair
 * `pair` (parity tests): len_db x len_q bytes, cell (i, j) at (i-1) len_q +
 * j-1, bits set when the parent is ABSENT - 0 argI, 1 argD (M's predecessor:
 * I / D in max(M, I, D) at (i, j), :120-153), 2 I-open (M(i, j) + open
 * among the maxima of I(i, j+1), :108-119), 3 D-open (the same for D(i+1,
 * j), :96-107); in the last row bit 3 of the end cell is argM.  Last
 * synchronous execute; SALN_E_INVALID for a pair stored otherwise. */
int saln_nw_plan_walk_codes(saln_nw_plan *plan, uint64_t pair, uint8_t *out);
/* mask_bytes: HBM parent-mask workspace (owned by the plan);
 * cigar_words: required length of the device cigar buffer. */
int saln_nw_plan_info(const saln_nw_plan *plan, uint64_t *mask_bytes, uint64_t *cigar_words,
                      uint64_t *cells);
int saln_nw_cigar_offsets(const saln_nw_plan *plan, uint64_t *cigar_off /* n_pairs+1 */);
int saln_nw_execute(saln_nw_plan *plan, const uint8_t *d_q_seq, const uint8_t *d_db_seq,
                    saln_nw_result *d_results, uint32_t *d_cigar, void *stream);
/* Optional per-kernel timing (hipEvents recorded on the launch stream around
 * each kernel of every execute while enabled).  Names: "nw_fill", "nw_traceback". */
int saln_nw_plan_set_timing(saln_nw_plan *plan, int enable);
int saln_nw_plan_kernel_time(const saln_nw_plan *plan, const char *kernel, double *total_ms,
                             uint64_t *launches);
/* Pipelined mode: execute returns with the traceback still running on the
 * context's second stream, so the traceback of batch n overlaps the fill of
 * batch n+1 (the plan double-buffers its mask workspace).  Results of an
 * execute are complete only after saln_nw_plan_sync(plan, stream, ...) has
 * made `stream` wait for them; keep_latest = 1 leaves the most recent execute
 * pending (software pipelining). */
int saln_nw_plan_set_async(saln_nw_plan *plan, int enable);
/* Score-only mode (the all-vs-all C5 workload): no parent codes, no
 * traceback; results carry score and the reference's panic status
 * (end_states = printed = cigar_len = 0, flags bit 3 set). */
int saln_nw_plan_set_score_only(saln_nw_plan *plan, int enable);
int saln_nw_plan_sync(saln_nw_plan *plan, void *stream, int keep_latest);
/* The stream a pipelined plan's tracebacks run on (NULL: the context's
 * second stream), e.g. a CU-masked stream so that the walk of execute n and
 * the fill of execute n+1 use disjoint CUs (tools/cu_pipeline.py). */
int saln_nw_plan_set_tb_stream(saln_nw_plan *plan, void *stream);
/* Device-side status of the plan's executes.  Waits (host-blocking) for every
 * execute issued since the previous call, then returns the device error
 * flags they raised (SALN_FLAG_*) in *flags (may be NULL) and clears them:
 * read-and-clear, so each execute is reported exactly once.  Returns
 * SALN_E_DEVICE_WAIT when a flag is set, SALN_OK otherwise.  The host-buffer
 * entry points (saln_nw_align, saln_nw_align_batch, ...) check it themselves;
 * device-plan callers call it after their executes (the kernels cannot fail
 * a stream).  A column-stripe fill never hangs: its bounded wait sets the
 * flag and the launch drains with wrong values for that pair. */
int saln_nw_plan_status(saln_nw_plan *plan, uint32_t *flags);
/* Polls a column-stripe dependency wait may spend before it gives up
 * (default 2^24, each poll sleeping ~64 clocks).  Test hook: 0 makes any wait
 * that finds its row unpublished fail, which injects SALN_FLAG_WAIT_TIMEOUT. */
int saln_nw_plan_set_wait_limit(saln_nw_plan *plan, uint32_t polls);
/* Waits for the device, then returns the plan's blocks to its context. */
int saln_nw_plan_destroy(saln_nw_plan *plan);

/* ------------------------------------ NW: score-only all-vs-all (device, C5)
 * The pair loop `for d in db { for q in query { n_w_align(q, d) } }`
 * (main.rs:61-67) reduced to what a score-only caller keeps: for every pair
 * p = d * n_q + q (reference order) out[2p] = score, out[2p+1] = status
 * (SALN_OK | SALN_REF_PANIC_BOUNDARY).  No per-pair descriptors: short
 * queries (packed-i16 region) are grouped into length classes and every
 * class runs as one index space over (query, db record); other queries go
 * through an internal score-only plan.  q_off/db_off are host offsets; the
 * sequences and `out` (int32[2 * n_q * n_db]) live on the device. */
typedef struct saln_nw_avsa saln_nw_avsa;
int saln_nw_avsa_create(saln_context *ctx, const uint64_t *q_off, uint64_t n_q,
                        const uint64_t *db_off, uint64_t n_db, int32_t mode,
                        const saln_nw_scoring *scoring, saln_nw_avsa **out);
int saln_nw_avsa_execute(saln_nw_avsa *a, const uint8_t *d_q_seq, const uint8_t *d_db_seq,
                         int32_t *d_out, void *stream);
/* cells = sum over all pairs of len_q * len_db; fallback_pairs = pairs that
 * take the plan path. */
int saln_nw_avsa_info(const saln_nw_avsa *a, uint64_t *cells, uint64_t *fallback_pairs);
/* Launch geometry of a packed query class (fill variant 4-8; include/saln.h
 * has no variant enum, the numbers are nw_kernels.hip's): the most pairs one
 * launch takes and the workgroups (256 threads) that launch has.  Introspection
 * for tests: blocks * 256 must stay a 32-bit work-item count. */
int saln_nw_avsa_launch_geometry(int variant, uint64_t *chunk_pairs, uint64_t *grid_blocks);
/* saln_nw_plan_status of the internal plan (SALN_OK without one); the packed
 * classes have no inter-workgroup waits. */
int saln_nw_avsa_status(saln_nw_avsa *a, uint32_t *flags);
int saln_nw_avsa_destroy(saln_nw_avsa *a);

/* ------------------------- NW: one long pair split by columns (multi-GPU, f3)
 * The fill loop of one pair (needleman_wunsch_affine.rs:217-236) and its
 * traceback (:242-334) cut into column spans, one per GPU (SURVEY.md §8(f)
 * #3): span r owns query columns col_lo+1 .. col_hi (col_lo a multiple of
 * 256), keeps only its part of the 1 B/cell parent mask, and runs the row
 * fill's column stripes over every db row.  Its first stripe takes the
 * boundary entering column col_lo+1 from the span's INBOX column, its last
 * stripe publishes the boundary leaving column col_hi into its OUTBOX column;
 * a caller moves outbox rows of span r into the inbox of span r+1 while both
 * fills run (RCCL send/recv per row band, or a device copy).  Boundary
 * columns hold one 8-byte element per db row r at element r (the engine's
 * internal (H, I) form; an unpublished row reads 0x80000000 in its low word),
 * saln_nw_span_boundary_elems elements per column.
 *
 * The traceback crosses the spans right to left: the span holding the end
 * cell walks from it (entry SALN_SPAN_END) until the walk leaves its first
 * column; its exit is the entry of the span to the left; the span where the
 * walk ends reports kind SALN_SPAN_EXIT + event.  Concatenating the spans'
 * op words in walk order (last span first, runs of one op merged at the
 * seams) and reversing gives the pair's CIGAR. */
typedef struct saln_nw_span saln_nw_span;
/* walk cursor kinds (entry / exit) */
#define SALN_SPAN_M 0         /* state known: M, I or D at (i, j) */
#define SALN_SPAN_I 1
#define SALN_SPAN_D 2
#define SALN_SPAN_VIA_M 3     /* arrived at (i, j) by a diagonal step: state = its argmax */
#define SALN_SPAN_VIA_I 4     /* arrived by a horizontal step: state from (i, j+1)'s I bits */
#define SALN_SPAN_END 5       /* the pair's end cell, first end state (the reference's order) */
#define SALN_SPAN_EXIT 8      /* exit: the walk ended; + 0 origin, + 1 panic, + 2 dead end */
typedef struct {
    int32_t i, j;   /* cell (db row, query column) */
    int32_t kind;   /* SALN_SPAN_* */
    uint32_t end_states; /* exit of the end cell's span: the end cell's state set
                            (bit0 M, bit1 I, bit2 D), else 0 */
} saln_nw_span_cursor;
/* Elements (8 bytes each) of one boundary column for a db of len_db rows. */
uint64_t saln_nw_span_boundary_elems(uint64_t len_db);
/* Boundary columns (stripes + 1) of the span col_lo+1 .. col_hi: the size of a
 * caller-owned d_boundary is cols * saln_nw_span_boundary_elems(len_db)
 * elements (host-only, no device needed).  device_cols: the query columns of
 * every span that fills on the same device at the same time (0: this span
 * alone); the stripe width follows from it (64 columns while each stripe
 * has a SIMD of its own, else 128). */
uint64_t saln_nw_span_boundary_cols(uint64_t col_lo, uint64_t col_hi, uint64_t device_cols);
/* d_boundary: caller-owned device buffer of (stripes + 1) boundary columns
 * (saln_nw_span_info), column 0 the inbox, the last column the outbox; NULL:
 * the span allocates it. */
int saln_nw_span_create(saln_context *ctx, uint64_t len_q, uint64_t len_db, uint64_t col_lo,
                        uint64_t col_hi, uint64_t device_cols, const saln_nw_scoring *scoring,
                        void *d_boundary, saln_nw_span **out);
int saln_nw_span_info(const saln_nw_span *s, uint64_t *mask_bytes, uint64_t *boundary_cols,
                      uint64_t *ops_cap);
/* Device addresses of the inbox (column 0) and outbox (last column). */
int saln_nw_span_boundary(const saln_nw_span *s, void **inbox, void **outbox);
/* Presets both boundary columns to "unpublished" on `stream`.  Must precede
 * any write into the inbox and the fill. */
int saln_nw_span_reset(saln_nw_span *s, void *stream);
/* Launches the span's fill (q / db: the whole pair's sequences on the
 * device).  A span with col_lo > 0 waits, row by row, for its inbox. */
int saln_nw_span_fill(saln_nw_span *s, const uint8_t *d_q, const uint8_t *d_db, void *stream);
/* Launches a one-wave kernel that returns once outbox rows row_lo .. row_hi
 * are published (bounded by the wait limit: then the timeout flag is set),
 * so work queued behind it on `stream` may read them. */
int saln_nw_span_watch(saln_nw_span *s, uint64_t row_lo, uint64_t row_hi, void *stream);
/* Walks this span from `entry` (host-blocking, after the fill completed);
 * ops (host, ops_cap words) receive the run words in walk order (back to
 * front); *exit the cursor where the walk left the span or ended. */
int saln_nw_span_walk(saln_nw_span *s, const uint8_t *d_q, const uint8_t *d_db,
                      const saln_nw_span_cursor *entry, saln_nw_span_cursor *exit, uint32_t *ops,
                      uint64_t ops_cap, uint64_t *n_ops, void *stream);
/* The span holding the end cell: score and panic status of the pair once the
 * fill queued on `stream` has finished (host-blocking; SALN_E_INVALID on
 * another span). */
int saln_nw_span_score(saln_nw_span *s, int32_t *score, int32_t *status, void *stream);
/* As saln_nw_plan_status / saln_nw_plan_set_wait_limit for the span's fill
 * and watch waits. */
int saln_nw_span_status(saln_nw_span *s, uint32_t *flags);
int saln_nw_span_set_wait_limit(saln_nw_span *s, uint32_t polls);
int saln_nw_span_destroy(saln_nw_span *s);
/* Spans of one pair on ONE device (tests, the single-GPU emulation of the
 * multi-GPU chain): queues on `stream` a one-wave kernel that copies src's
 * outbox rows row_lo .. row_hi into dst's inbox as they are published (64
 * rows per round). */
int saln_nw_span_forward(saln_nw_span *src, saln_nw_span *dst, uint64_t row_lo, uint64_t row_hi,
                         void *stream);
/* Compute units of the context's device, and a stream whose kernels run only
 * on CUs cu_lo .. cu_hi-1 (hipExtStreamCreateWithCUMask): one device split
 * into per-span partitions. */
/* The walk over all n spans of a pair on ONE device at once: every span's
 * speculative stripe passes run together over a shared record table, linked
 * on the host from the end cell to the walk's end.  Returns SALN_OK with the
 * pair's CIGAR in `ops` (forward order, runs of one op merged across the
 * spans' seams: the words saln_nw_align gives when the walk printed) and the
 * final exit, SALN_SPAN_UNLINKED when the passes do not link (walk span by
 * span with saln_nw_span_walk), or an error. */
int saln_nw_spans_walk(saln_nw_span *const *spans, uint32_t n, const uint8_t *d_q,
                       const uint8_t *d_db, saln_nw_span_cursor *exit, uint32_t *ops,
                       uint64_t ops_cap, uint64_t *n_ops, void *stream);
int saln_device_cu_count(saln_context *ctx, uint32_t *n);
/* A stream on mask bits [cu_lo, cu_hi).  Bit c is a CU of XCD c mod n_xcd
 * (measured, profiles/r04_cu_map.json), so a range of 8k bits is k CUs per
 * XCD.  Ranges shorter than the XCD count are refused (SALN_E_INVALID): an
 * XCD left without a bit runs unmasked. */
int saln_stream_create_cu_range(saln_context *ctx, uint32_t cu_lo, uint32_t cu_hi, void **stream);
int saln_stream_destroy(saln_context *ctx, void *stream);
/* A stream on an arbitrary CU mask (bit c of word c / 32 = CU c in the
 * runtime's mask order, hipExtStreamCreateWithCUMask; an XCD with no bit set
 * runs unmasked, see saln_stream_create_cu_range). */
int saln_stream_create_cu_mask(saln_context *ctx, const uint32_t *mask, uint32_t n_words,
                               void **stream);
/* Diagnostic: launches n_blocks one-wave workgroups on `stream` (e.g. a
 * CU-masked one) and returns, per workgroup, the HW_ID register of its wave
 * (gfx9 layout: CU 11:8, SH 12, SE 15:13) and its XCC_ID (host arrays of
 * n_blocks).  tools/cu_map.py derives the mask bit -> (XCD, SE, CU) order. */
int saln_device_cu_probe(saln_context *ctx, void *stream, uint32_t n_blocks, uint32_t *hw_id,
                         uint32_t *xcc_id);

/* ----------------------------------------------------------------------- WFA
 * Replaces `pub fn wfa_align(seq1: &Record, seq2: &Record, mode: Mode)`
 * (wfa.rs:23-42) with the reference's exact (quirky) semantics: wavefront
 * tensors built by WaveFrontTensor::new (:225-420), extension of the newest
 * M front only (:127-139, :467-488), Ocean::trim (:490-623), convergence on
 * the newest tensor at (len_db-1, len_q-1) (:180-191), and the greedy rec_tr
 * traceback (:654-853).  seq1 = query, seq2 = db.  The reference loops
 * forever when it never converges; max_steps bounds the expand loop
 * (status SALN_NONCONVERGED), and max_width bounds a wavefront's width
 * (also SALN_NONCONVERGED).  Rust panics are statuses:
 * SALN_REF_PANIC_TRIM (rotate_left / expect / unwrap in trim),
 * SALN_REF_PANIC_SLICE (slice indexing in rec_tr). */
typedef struct {
    int32_t score;        /* printed score: wfs.len() at convergence (:33-38) */
    int32_t status;       /* SALN_OK | SALN_NOT_IMPLEMENTED | SALN_REF_PANIC_* | SALN_NONCONVERGED */
    uint32_t steps;       /* Ocean::expand calls */
    uint32_t aln_len1;    /* bytes of Alignment.seq1 / seq2 (traceback output) */
    uint32_t aln_len2;
    int32_t conv_offset;  /* converged element (:640): offset, state (0 M, 1 D, 2 I), */
    uint8_t conv_state;   /*   parents (np entries, same codes)                      */
    uint8_t conv_np;
    uint8_t conv_parents[3];
    uint8_t reserved[3];
} saln_wfa_result;        /* 32 bytes */

/* Batched wfa_align over pairs (same pair conventions as
 * saln_nw_align_batch).  aln (optional): per pair 2*aln_cap bytes at
 * aln_off[p] (seq1 then seq2, in the reference's push order, i.e. reversed).
 * max_steps = 0 selects 64; max_width = 0 selects 64. */
int saln_wfa_align_batch(saln_context *ctx, const uint8_t *q_seq, const uint64_t *q_off,
                         uint64_t n_q, const uint8_t *db_seq, const uint64_t *db_off,
                         uint64_t n_db, const uint32_t *pair_q, const uint32_t *pair_db,
                         uint64_t n_pairs, int32_t mode, uint32_t max_steps, uint32_t max_width,
                         saln_wfa_result *results, uint8_t *aln, const uint64_t *aln_off,
                         uint32_t aln_cap);

/* Everything the reference prints to stdout for one wfa_align call (the
 * `lo/hi` lines, `converged with score`, the traceback's debug lines, the
 * alignment and its Debug dump), up to the point where it would panic. */
int saln_wfa_render(saln_context *ctx, const uint8_t *q, uint64_t len_q, const uint8_t *d,
                    uint64_t len_db, int32_t mode, uint32_t max_steps, uint32_t max_width,
                    char *out, uint64_t cap, uint64_t *out_len, saln_wfa_result *result);

/* The same text for every pair of a batch (pair conventions as
 * saln_wfa_align_batch), each pair computed once: one GPU run of the batch
 * with its step logs and alignment rows, then host rendering.  Replaces the
 * size-probe + render pair of saln_wfa_render calls per pair that the pair
 * loop main.rs:61-74 would otherwise make.  Large batches run in chunks of
 * at most ~1 GB of alignment rows and step logs each. */
typedef struct saln_wfa_text saln_wfa_text;
int saln_wfa_render_batch(saln_context *ctx, const uint8_t *q_seq, const uint64_t *q_off,
                          uint64_t n_q, const uint8_t *db_seq, const uint64_t *db_off,
                          uint64_t n_db, const uint32_t *pair_q, const uint32_t *pair_db,
                          uint64_t n_pairs, int32_t mode, uint32_t max_steps, uint32_t max_width,
                          saln_wfa_text **out);
uint64_t saln_wfa_text_count(const saln_wfa_text *t);
/* text points into the handle (not NUL-terminated; len bytes), valid until
 * saln_wfa_text_free. */
int saln_wfa_text_get(const saln_wfa_text *t, uint64_t pair, const char **text, uint64_t *len,
                      saln_wfa_result *result);
void saln_wfa_text_free(saln_wfa_text *t);

/* Device-resident WFA batch (configs[2] / C3 measurement): plan once from host
 * offsets and a pair list (NULL = all-vs-all, reference order), then execute
 * on device sequences (same CSR layout) into device results[n_pairs].  No
 * alignment rows.  Pairs that reach a 64-step first pass are re-run with
 * max_steps; the results equal a single pass at max_steps. */
typedef struct saln_wfa_plan saln_wfa_plan;
int saln_wfa_plan_create(saln_context *ctx, const uint64_t *q_off, uint64_t n_q,
                         const uint64_t *db_off, uint64_t n_db, const uint32_t *pair_q,
                         const uint32_t *pair_db, uint64_t n_pairs, int32_t mode,
                         uint32_t max_steps, uint32_t max_width, saln_wfa_plan **out);
int saln_wfa_execute(saln_wfa_plan *plan, const uint8_t *d_q_seq, const uint8_t *d_db_seq,
                     saln_wfa_result *d_results, void *stream);
int saln_wfa_plan_destroy(saln_wfa_plan *plan);

/* ------------------------------------------- corrected gap-affine WFA (new)
 * NOT a reference-parity path.  The reference's
 * wfa_align (src/wfa.rs:23-42, above) defines no output for realistic inputs
 * (Ocean::trim panics at s = 20).  These entry points compute
 * what a gap-affine WFA is meant to: the minimum penalty of a global
 * alignment, mismatch * #mismatches + sum(gap_open + gap_extend * len) over
 * gaps, with the reference's penalties (wfa.rs:14-21) by default.  The
 * checker is the Gotoh DP (oracle/refaffine.c).
 * scores[p] >= 0: the penalty; -1: above max_score (max_score <= 0: no cap);
 * -2: the wavefront grew past 2,048 diagonals (i16 offsets; 1,024 for a
 * sequence longer than 32,000 bases). */
typedef struct {
    int32_t mismatch;   /* x = 4 */
    int32_t gap_open;   /* o = 2 */
    int32_t gap_extend; /* e = 6 */
} saln_wfa_penalties;   /* NULL = the reference's {4, 2, 6} */

int saln_wfa_affine_batch(saln_context *ctx, const uint8_t *q_seq, const uint64_t *q_off,
                          uint64_t n_q, const uint8_t *db_seq, const uint64_t *db_off,
                          uint64_t n_db, const uint32_t *pair_q, const uint32_t *pair_db,
                          uint64_t n_pairs, const saln_wfa_penalties *pen, int32_t max_score,
                          int32_t *scores);
/* Device-resident form (configs[2] measurement with the corrected engine):
 * plan from host offsets and a pair list (NULL = all-vs-all, reference
 * order), execute on device sequences into device scores[n_pairs]. */
typedef struct saln_wfa_affine_plan saln_wfa_affine_plan;
int saln_wfa_affine_plan_create(saln_context *ctx, const uint64_t *q_off, uint64_t n_q,
                                const uint64_t *db_off, uint64_t n_db, const uint32_t *pair_q,
                                const uint32_t *pair_db, uint64_t n_pairs,
                                const saln_wfa_penalties *pen, int32_t max_score,
                                saln_wfa_affine_plan **out);
int saln_wfa_affine_execute(saln_wfa_affine_plan *plan, const uint8_t *d_q_seq,
                            const uint8_t *d_db_seq, int32_t *d_scores, void *stream);
int saln_wfa_affine_plan_destroy(saln_wfa_affine_plan *plan);

/* --------------------------------------------------------------------- FASTA
 * Replaces `pub fn parse_fasta(path: PathBuf) -> Result<Records>`
 * (parse.rs:54-99): extension must be exactly fa|fasta|fna; '>' opens a record
 * whose name includes the '>'; bytes outside {A,G,C,T,N} in sequence lines are
 * dropped and reported (returns SALN_E_FASTA_CHARS with the records still
 * valid, like CharError{res,chars}). */
typedef struct saln_records saln_records;
int saln_parse_fasta(const char *path, saln_records **out, uint8_t *bad_chars, uint64_t bad_cap,
                     uint64_t *n_bad);
int saln_parse_fasta_buffer(const uint8_t *buf, uint64_t len, saln_records **out,
                            uint8_t *bad_chars, uint64_t bad_cap, uint64_t *n_bad);
uint64_t saln_records_count(const saln_records *r);
int saln_records_get(const saln_records *r, uint64_t i, const uint8_t **name, uint64_t *name_len,
                     const uint8_t **seq, uint64_t *seq_len);
void saln_records_free(saln_records *r);

#ifdef __cplusplus
}
#endif
#endif /* SALN_H */

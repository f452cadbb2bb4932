/*
 * ORACLE — test infrastructure only. Nothing in the product links, loads or
 * calls this code; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker.
 *
 * Plain-C restatement of the reference CPU algorithms of
 * Qw11111111111/SequenceAligning (Rust, snapshot 2025-02-13):
 *   - NW affine fill      src/needleman_wunsch_affine.rs:169-237 (+ :76-153)
 *   - NW DFS traceback    src/needleman_wunsch_affine.rs:242-334, Display :390-411
 *   - FASTA parser        src/parse.rs:54-106
 *   - WFA                 src/wfa.rs (see refwfa.c)
 *
 * Pinning: the reference is Rust and cannot be built here (no cargo/rustc;
 * SURVEY.md §8(c)).  NW parity is pinned only by the hand-traced KATs of
 * SURVEY.md §8.4 (the reference's own NW tests are empty stubs,
 * needleman_wunsch_affine.rs:458-470), i.e. NW parity is *unpinned by any
 * reference-run fixture*.  The parser is pinned by the reference's tests
 * parse.rs:166-251 and WFA by wfa.rs:994-1294 (test_initial etc.).
 */
#ifndef SALN_ORACLE_REFCPU_H
#define SALN_ORACLE_REFCPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define REF_SENTINEL (-32768) /* i16::MIN as i32, needleman_wunsch_affine.rs:174 */

/* Parent bit conventions (bit order == the reference's push order):
 *   pM: bit0 = M[x-1][y-1], bit1 = I[x-1][y-1], bit2 = D[x-1][y-1]   (:120-153)
 *   pI: bit0 = I[x][y-1] (extend), bit1 = M[x][y-1] (open)           (:108-119)
 *   pD: bit0 = D[x-1][y] (extend), bit1 = M[x-1][y] (open)           (:96-107)
 * Boundary: D[0][j>=1] has pD bit0 (parent D[0][j-1], :196),
 *           I[i>=1][0] has pI bit0 (parent I[i-1][0], :208).
 * All matrices are (ld+1) x (lq+1), row-major, index x*(lq+1)+y, x over db
 * (seq2), y over query (seq1) — ScoreMatrix::new(x=len_db, y=len_q) :428. */
typedef struct {
    size_t lq, ld;
    int32_t *M, *I, *D;
    uint8_t *pM, *pI, *pD;
} ref_nw_mats;

/* Allocate and fill; returns 0 on success.  Free with ref_nw_free. */
int ref_nw_fill(const uint8_t *q, size_t lq, const uint8_t *d, size_t ld, ref_nw_mats *out);
void ref_nw_free(ref_nw_mats *m);

/* Dense 7-bit cell code used for mask parity (same meaning as the product's
 * dense mask export):  bits0-2 = {M,I,D} that equal max(M,I,D) at (x,y),
 * bits3-4 = pI(x,y) {ext,open}, bits5-6 = pD(x,y) {ext,open}.
 * out has (ld+1)*(lq+1) bytes. */
void ref_nw_dense_mask(const ref_nw_mats *m, uint8_t *out);

/* Literal DFS traceback (needleman_wunsch_affine.rs:242-330).  Writes the
 * text the reference prints for this pair (without the timing line) into
 * out (truncated at out_cap; *out_len gets the full length).
 * Stops after max_pops stack pops (0 = unlimited).
 * Returns: 0 = DFS finished, 1 = panic (boundary index, :299/:303),
 *          2 = pop cap reached. *n_blocks = blocks printed. */
int ref_nw_traceback_dfs(const uint8_t *q, const uint8_t *d, const ref_nw_mats *m,
                         char *out, size_t out_cap, size_t *out_len,
                         uint64_t max_pops, uint64_t *n_blocks);
/* The same DFS stopping before the (max_blocks+1)-th printed block (rc 3;
 * 0 = no cap): the text of `saln --max-blocks N`. */
int ref_nw_traceback_dfs_blocks(const uint8_t *q, const uint8_t *d, const ref_nw_mats *m,
                                char *out, size_t out_cap, size_t *out_len, uint64_t max_pops,
                                uint64_t max_blocks, uint64_t *n_blocks);

/* Score = max(M,I,D)[ld][lq] (:247-250). end_states: bit0 M, bit1 I, bit2 D. */
int32_t ref_nw_score(const ref_nw_mats *m, uint8_t *end_states);

/* Memoised DAG restatement of the same DFS (order-preserving path counting):
 * *n_blocks = blocks printed before the first panic (saturating),
 * *panics = 1 if the DFS would panic.  Also returns the first printed block
 * as an op string (forward order; '=' 'X' 'I' 'D') into ops (cap ops_cap),
 * *ops_len = -1 if nothing is printed.  Returns 0. */
int ref_nw_dag_summary(const uint8_t *q, const uint8_t *d, const ref_nw_mats *m,
                       uint64_t *n_blocks, int *panics, char *ops, size_t ops_cap,
                       int64_t *ops_len);

/* Timed CPU baseline: fill + literal DFS over n pairs, output discarded.
 * Sequences are CSR (seq + offsets, n+1).  Returns cells processed. */
uint64_t ref_nw_run_pairs(const uint8_t *qs, const uint64_t *q_off, const uint8_t *ds,
                          const uint64_t *d_off, uint64_t n_pairs, uint64_t max_pops);
/* ref_nw_run_pairs, also counting the pairs whose DFS stopped at max_pops
 * (*capped, may be NULL) */
uint64_t ref_nw_run_pairs_capped(const uint8_t *qs, const uint64_t *q_off, const uint8_t *ds,
                                 const uint64_t *d_off, uint64_t n_pairs, uint64_t max_pops,
                                 uint64_t max_blocks, uint64_t *capped);
/* refmt.c: ref_nw_run_pairs over contiguous slices of the pairs on threads
 * (_capped: with the count of capped pairs) */
uint64_t ref_nw_run_pairs_mt_capped(const uint8_t *qs, const uint64_t *q_off, const uint8_t *ds,
                                    const uint64_t *d_off, uint64_t n_pairs, uint64_t max_pops,
                                    uint64_t max_blocks, int threads, uint64_t *capped);
/* the same with every pair's text written to fd in pair order (refmt.c) */
uint64_t ref_nw_run_pairs_text_mt(const uint8_t *qs, const uint64_t *q_off, const uint8_t *ds,
                                  const uint64_t *d_off, uint64_t n_pairs, uint64_t max_pops,
                                  uint64_t max_blocks, int threads, int fd, uint64_t chunk,
                                  uint64_t *bytes, uint64_t *capped);
uint64_t ref_nw_run_pairs_mt(const uint8_t *qs, const uint64_t *q_off, const uint8_t *ds,
                             const uint64_t *d_off, uint64_t n_pairs, uint64_t max_pops,
                             int threads);

/* refcheck.c: per-pair score, end states, panic status and first printed
 * alignment (CIGAR words (len << 4) | op, '=' 7 'X' 8 'I' 1 'D' 2; cig_len -1
 * when nothing is printed) for every pair of a CSR batch, on threads. */
int ref_nw_check_pairs_mt(const uint8_t *qs, const uint64_t *q_off, const uint8_t *ds,
                          const uint64_t *d_off, uint64_t n_pairs, const uint64_t *cig_off,
                          int32_t *score, uint8_t *end_states, uint8_t *panics, int32_t *cig_len,
                          uint32_t *cig, int threads);

/* Linear-memory score + end states + panic status of one pair with the
 * reference semantics (reflinear.c), on `threads` column stripes.  For
 * pairs too large for ref_nw_fill (C4).  Returns 0 on success. */
int ref_nw_score_linear(const uint8_t *q, size_t lq, const uint8_t *d, size_t ld, int threads,
                        int32_t *score, uint8_t *end_states, int *panics);

/* ref_nw_score_linear plus the first event of the reference DFS over stored
 * parent sets (1 B per cell of host memory): ops (forward, '=' 'X' 'I' 'D')
 * of the first printed alignment, *ops_len = -1 if nothing is printed (the
 * DFS panics first, or every path is sentinel-rooted); *dead_nodes = (cell,
 * state) nodes the DFS exhausted without a terminal before that event. */
int ref_nw_first_linear(const uint8_t *q, size_t lq, const uint8_t *d, size_t ld, int threads,
                        int32_t *score, uint8_t *end_states, int *panics, char *ops,
                        size_t ops_cap, int64_t *ops_len, uint64_t *dead_nodes);

/* FASTA parser restatement (parse.rs:54-99) on an in-memory buffer.
 * has_valid_ext: result of the extension check (:55-60) done by the caller.
 * Records are returned as a flat byte stream: for each record
 * [u32 name_len][name bytes][u32 seq_len][seq bytes].  Returns number of
 * records, or -1 for FastaError (bad extension).  *n_bad_chars = number of
 * dropped bytes, bad_chars receives them (cap bad_cap). */
int64_t ref_parse_fasta(const uint8_t *buf, size_t len, int has_valid_ext, uint8_t *rec_out,
                        size_t rec_cap, size_t *rec_len, uint8_t *bad_chars, size_t bad_cap,
                        size_t *n_bad_chars);

/* splitmix64 synthetic generator. */
uint64_t ref_splitmix64(uint64_t *state);

/* ---------------------------------------------------------------- WFA
 * ref_wfa_align: wfa_align(seq1 = q, seq2 = d, mode) (wfa.rs:23-42) with
 * release semantics.  out gets everything the reference prints to stdout
 * for the pair (the `lo/hi` lines, the convergence and traceback debug
 * lines, the alignment and its Debug dump).  max_steps caps the expand loop
 * (0 = unlimited; the reference can loop forever).  Returns res->status. */
enum {
    REF_WFA_OK = 0,
    REF_WFA_NOT_IMPLEMENTED = 1, /* non-global mode :26 */
    REF_WFA_PANIC_TRIM = 3,      /* Ocean::trim rotate_left / expect / unwrap :524-603 */
    REF_WFA_PANIC_SLICE = 4,     /* rec_tr slice indexing :695-844 */
    REF_WFA_NONCONVERGED = 5     /* max_steps reached */
};
typedef struct {
    int32_t status;
    uint64_t steps;    /* expand calls */
    int64_t score;     /* printed score wfs.len() */
    uint64_t aln_len1, aln_len2;
} ref_wfa_result;
int ref_wfa_align(const uint8_t *q, size_t lq, const uint8_t *d, size_t ld, int mode,
                  uint64_t max_steps, ref_wfa_result *res, char *out, size_t out_cap,
                  size_t *out_len);
/* WaveFrontTensor::new on flat-encoded tensors (refwfa.c) for the
 * reference's tensor tests; NULL = None.  Returns the encoded length. */
int64_t ref_wfa_tensor_new(const int32_t *o, const int32_t *e, const int32_t *x, int32_t *out,
                           char *txt_out, size_t txt_cap);
int ref_wfa_initial_converged(const uint8_t *q, size_t lq, const uint8_t *d, size_t ld);

#ifdef __cplusplus
}
#endif
#endif

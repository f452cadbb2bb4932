// Shared host/device definitions for the NW-affine engine.
//
// Scaled representation ("flag-in-LSB"): every score V of the reference
// recurrence (needleman_wunsch_affine.rs:76-94) is carried as V' = 2V + p,
// where p = 1 iff a reference boundary panic node (D[0][j>=1] :196, I[i>=1][0]
// :208) is reachable from this (cell,state) through the reference's parent
// pointers.  max() over scaled candidates returns the max score and ORs the
// flags of the tied maxima, which is exactly the "panic reachable" closure of
// the reference's DFS (:281-329).  Constants are added scaled by 2, which
// keeps the flag.  Equality with the max is tested against H' & ~1.
//
// The i32 fills (lanes, column stripes) carry a second, nested flag:
// V'' = 4V + 2a + p, a = 1 iff a DFS terminal (the origin, :283-286, or a
// panic node) is reachable ("alive").  Paths into the sentinel-valued roots
// M[0][j>=1], I[0][j], M[i>=1][0], D[i][0] (no parents, :172-216) are dead:
// the DFS drops them silently.  p implies a, so max() over (V, a, p) ORs both
// flags.  Walk codes test ties against H'' & ~1: among the tied parents the
// alive ones, if any; the greedy walk over those is the reference DFS's
// first path even where the sentinel competes (x + y > ~5,450).  Full codes
// (the reference's parent sets) test against & ~3.  A pair is sentinel-free
// (every maximum real, every cell alive) while the boundary values of its
// last column and row stay above the sentinel: then V' = 2V + p suffices.
#pragma once
#include <stdint.h>

#ifndef SALN_HD
#if defined(__HIPCC__)
#define SALN_HD __host__ __device__ __forceinline__
#else
#define SALN_HD inline
#endif
#endif

namespace saln {

constexpr int32_t kSentinel = -32768;  // i16::MIN as i32, needleman_wunsch_affine.rs:174
constexpr int kNumVariants = 9;        // fill kernel variants (nw_kernels.hip)
// plans with at least this many column-stripe waves use the packed stripe fill
constexpr uint64_t kStripePkMinWaves = 1024;
// polls a column-stripe dependency wait spends before it sets the plan's
// timeout flag (saln_nw_plan_set_wait_limit; each poll sleeps ~64 clocks)
constexpr uint32_t kWaitLimitDefault = 1u << 24;

struct Scoring {
    int32_t match, mismatch, gap_open, gap_extend;
};

// Cell-code bits (dense mask layout, include/saln.h saln_nw_dense_mask).
enum : uint8_t {
    kArgM = 1, kArgI = 2, kArgD = 4,
    kIExt = 8, kIOpen = 16,
    kDExt = 32, kDOpen = 64,
};

// One pair as the fill/traceback kernels see it (plan order).
struct NwPairDesc {
    uint64_t q_off, db_off;  // byte offsets into the query / db sequence buffers
    uint64_t mask_off;       // byte offset of this pair's segment (row 1, block 0) in the workspace
    uint64_t mask_rs;        // bytes from row i to row i+1 of the pair's mask
    uint64_t cigar_off;      // word offset of this pair's cigar (in results order)
    uint64_t scratch_off;    // int2 offset of the chunk-boundary column (multi-chunk pairs)
    uint64_t ops_off;        // word offset of the traceback's op stream (walker scratch)
    uint32_t mask_bs;        // bytes from column block b to b+1
    uint32_t len_q, len_db;
    uint32_t pair_id;        // index into results
    uint32_t variant;        // fill kernel variant (kernel geometry)
    uint32_t reserved;
    uint64_t mask_cs;        // bytes from query chunk c to c+1 (G*bs unless skewed)
};

// Speculative stripe walks of a long column-stripe pair (nw_kernels.hip,
// nw_traceback_coop_kernel<.., kSpec = true>): every 256-column walker stripe
// of the pair walks at once from an entry (cell, kind); pass 1 guesses the
// entries, pass k enters stripe s where pass k-1 left stripe s+1.
enum : int32_t {
    kSpecM = 0, kSpecI = 1, kSpecD = 2,  // state known
    kSpecViaM = 3,  // arrived by a diagonal step: state = argmax of the cell
    kSpecViaI = 4,  // arrived by a horizontal step: state from the I bits
    kSpecEnd = 5,   // the pair's end cell, first end state
    kSpecEv = 8,    // exit: walk ended (kSpecEv + event)
    kSpecNone = 16, // no entry (the walk ended in a stripe to the right)
};
constexpr uint32_t kSpecOpsCap = 2 * 256 + 8;  // run words per stripe (>= 2 per column + 2)
constexpr uint32_t kSpecMaxStripes = 4096;     // per pair (the link scan's LDS)
constexpr uint32_t kSpecMinStripes = 8;        // shorter pairs: the cooperative walker alone
constexpr uint32_t kSpecMaxPairs = 16;         // more column-stripe pairs walk in parallel anyway
struct SpecStripe {
    int32_t in_i, in_j, in_k;              // entry of the stored walk
    int32_t out_i[2], out_j[2], out_k[2];  // exit, per pass parity
    uint32_t nops;                         // run words (walk order, pending run last)
    uint32_t am_end;                       // last stripe: end cell argmax set
    int32_t base, k0;                      // link: walk-order slot of word 0, first word kept
    uint32_t open_w;                       // link: final value of the stripe's last word
};
struct SpecPair {
    uint32_t plan_idx, n_stripes, stripe_base, reserved;
};
struct SpecArgs {
    const uint2 *blocks;     // spec block -> (spec pair, stripe)
    const SpecPair *pairs;
    SpecStripe *stripes;
    uint32_t *ops;           // kSpecOpsCap words per stripe
    const uint32_t *done;    // plan index -> walk finished by the spec passes
    int32_t pass;
    // column-span walks (nw_span.cpp): span != 0 stops the walk only where
    // it leaves column span_c0 + 1 (the span's first), not at every stripe edge
    int32_t span, span_c0;
    // speculative passes over a span's stripes: stripe entry_s1 - 1 (the
    // span's rightmost) takes its entry from the record after it on every
    // pass (0: none)
    int32_t entry_s1;
};

// Kernel geometry of one fill variant: G lanes per pair, K query columns per
// lane, KD = ceil(K/4) mask dwords per lane-row segment (LB = 4*KD bytes).
// A pair's query is cut in chunks of W = G*K columns; column block
// b = (j-1)/K (chunk b/G, lane b%G).  Within a chunk, lane `lane` computes
// row r = t - lane + 1 at step t (t = 0 .. len_db+G-2).
// Mask layout (row-major, block-interleaved): the K codes of block b at row i
// are one LB-byte segment at mask_off + (i-1)*rs + b*bs.  A plan interleaves
// the segments of up to 64 consecutive pairs of a variant (one traceback
// wave): bs = n*LB and pair slot s sits at +s*LB, so the walker's per-lane
// loads of one (row, block) touch adjacent bytes and the fill's stores of a
// row are contiguous across the pairs of a wave.  A pair outside such a pack
// has bs = LB and rs = (blocks)*LB; in both, chunk stride cs = G*bs.
// Column-stripe pairs (G = 64, K = 4) are stored skewed instead, in the order
// the stripe wave writes them: the 64 lanes' code dwords of fill step t
// (lane l at row t-l+1) are the 256 contiguous bytes of line t of the
// stripe's region, so rs = 256, bs = 260 (next block: one row later, 4 bytes
// on) and cs = (len_db + 63) * 256.  The packed stripe fill (two int16
// halves per lane: 128 virtual lanes of 2 columns, virtual lane v = l + 64h
// at row t - v + 1 in step t) marks its layout with bs = 0: byte
// 4l + 2(col % 2) + h of line t, cs = (len_db + 127) * 256.
struct Geom {
    uint32_t G, K;
    SALN_HD uint32_t KD() const { return (K + 3) / 4; }
    SALN_HD uint32_t LB() const { return KD() * 4; }
    // 4-bit walk codes (nw_fill_pk_kernel kCodesNib): ceil(K/4) 16-bit
    // column-group halves per pair, two per dword, plus the row's db char
    SALN_HD uint32_t LBn() const { return 4 * ((K + 3) / 4 / 2 + 1); }
    SALN_HD uint32_t nib_char_byte() const {
        const uint32_t ng = (K + 3) / 4;
        return ng % 2 ? 4 * (ng / 2) + 2 : 4 * (ng / 2);
    }
    SALN_HD uint32_t W() const { return G * K; }
    SALN_HD uint32_t n_chunks(uint32_t len_q) const { return (len_q + W() - 1) / W(); }
    SALN_HD uint32_t n_blocks(uint32_t len_q) const { return n_chunks(len_q) * G; }
    SALN_HD uint32_t steps(uint32_t len_db) const { return len_db + G - 1; }
    // byte offset (from mask_off) of interior cell (i, j), 1-based
    SALN_HD uint64_t cell(uint32_t i, uint32_t j, uint64_t rs, uint32_t bs, uint64_t cs) const {
        if (bs == 0) {  // packed column stripes (nw_fill_stripe_pk_kernel): 256-byte lines
            const uint32_t jj = j - 1, o = jj % 256, v = o / 2;
            return (uint64_t)(jj / 256) * cs + (uint64_t)(i - 1 + v) * 256 + 4 * (v % 64) +
                   2 * (o % 2) + v / 64;
        }
        const uint32_t jj0 = j - 1, b = jj0 / K;
        return (uint64_t)(i - 1) * rs + (uint64_t)(b / G) * cs + (uint64_t)(b % G) * bs + jj0 % K;
    }
};

// ---------------------------------------------------------------- boundary
// Reference boundary values (needleman_wunsch_affine.rs:172-216), true scores.
SALN_HD int32_t d_row0(const Scoring &s, uint32_t j) {  // D[0][j], j >= 1
    return ((int32_t)j + 1) * s.gap_extend + s.gap_open;
}
SALN_HD int32_t i_col0(const Scoring &s, uint32_t i) {  // I[i][0], i >= 1
    return s.gap_open + ((int32_t)i + 1) * s.gap_extend;
}
SALN_HD int32_t imax(int32_t a, int32_t b) { return a > b ? a : b; }

// Scaled H'(0, j) and H'(i, 0).
SALN_HD int32_t hs_row0(const Scoring &s, uint32_t j) {
    return j == 0 ? 0 : imax(2 * kSentinel, 2 * d_row0(s, j) + 1);
}
SALN_HD int32_t hs_col0(const Scoring &s, uint32_t i) {
    return i == 0 ? 0 : imax(2 * kSentinel, 2 * i_col0(s, i) + 1);
}
// Scaled D'(1, j) (first-row D, from row 0) and I'(i, 1) (first-column I).
SALN_HD int32_t ds_row1(const Scoring &s, uint32_t j) {
    return imax(2 * kSentinel + 2 * s.gap_open, 2 * d_row0(s, j) + 1) + 2 * s.gap_extend;
}
SALN_HD int32_t is_col1(const Scoring &s, uint32_t i) {
    return imax(2 * kSentinel + 2 * s.gap_open, 2 * i_col0(s, i) + 1) + 2 * s.gap_extend;
}

// A pair whose boundary row / column never falls to the sentinel: no
// sentinel-derived value is ever a maximum, every path ends at the origin or
// a panic node (the packed fills and the packed stripes take only these).
SALN_HD bool sentinel_free(const Scoring &s, uint32_t len_q, uint32_t len_db) {
    const int32_t floor = kSentinel + imax(0, s.gap_open);  // also M[0][j] + open (D row 1)
    return (len_q == 0 || d_row0(s, len_q) > floor) && (len_db == 0 || i_col0(s, len_db) > floor);
}

// The i32 fills' V'' = 4V + 2a + p boundary values (origin alive, row-0 D and
// column-0 I alive panic nodes, the sentinel roots dead).
SALN_HD int32_t hs4_row0(const Scoring &s, uint32_t j) {
    return j == 0 ? 2 : imax(4 * kSentinel, 4 * d_row0(s, j) + 3);
}
SALN_HD int32_t hs4_col0(const Scoring &s, uint32_t i) {
    return i == 0 ? 2 : imax(4 * kSentinel, 4 * i_col0(s, i) + 3);
}
SALN_HD int32_t ds4_row1(const Scoring &s, uint32_t j) {
    return imax(4 * kSentinel + 4 * s.gap_open, 4 * d_row0(s, j) + 3) + 4 * s.gap_extend;
}
SALN_HD int32_t is4_col1(const Scoring &s, uint32_t i) {
    return imax(4 * kSentinel + 4 * s.gap_open, 4 * i_col0(s, i) + 3) + 4 * s.gap_extend;
}
// V'' -> V' (2V + p), the form the walkers and result kernels read.
SALN_HD int32_t x4_to_x2(int32_t v) { return ((v >> 2) << 1) | (v & 1); }

// Walk-code view of the boundary cells' bits: among tied candidates the
// alive ones (the sentinel roots are dead, row-0 D / column-0 I alive).
SALN_HD uint8_t argmax_row0_walk(const Scoring &s, uint32_t j) {
    if (j == 0) return kArgM;
    return d_row0(s, j) >= kSentinel ? kArgD : (uint8_t)(kArgM | kArgI);
}
SALN_HD uint8_t argmax_col0_walk(const Scoring &s, uint32_t i) {
    if (i == 0) return kArgM;
    return i_col0(s, i) >= kSentinel ? kArgI : (uint8_t)(kArgM | kArgD);
}
SALN_HD uint8_t ibits_col1_walk(const Scoring &s, uint32_t i) {  // open = M[i][0]: dead
    const int32_t ext = i_col0(s, i), open = kSentinel + s.gap_open;
    return (uint8_t)((ext >= open ? 1 : 0) | (open > ext ? 2 : 0));
}
SALN_HD uint8_t dbits_row1_walk(const Scoring &s, uint32_t j) {  // open = M[0][j]: dead
    const int32_t ext = d_row0(s, j), open = kSentinel + s.gap_open;
    return (uint8_t)((ext >= open ? 1 : 0) | (open > ext ? 2 : 0));
}

// argmax-set bits of boundary cells (the reference's tie sets).
SALN_HD uint8_t argmax_row0(const Scoring &s, uint32_t j) {
    if (j == 0) return kArgM;
    const int32_t dv = d_row0(s, j), h = imax(kSentinel, dv);
    return (uint8_t)((kSentinel == h ? (kArgM | kArgI) : 0) | (dv == h ? kArgD : 0));
}
SALN_HD uint8_t argmax_col0(const Scoring &s, uint32_t i) {
    if (i == 0) return kArgM;
    const int32_t iv = i_col0(s, i), h = imax(kSentinel, iv);
    return (uint8_t)((kSentinel == h ? (kArgM | kArgD) : 0) | (iv == h ? kArgI : 0));
}
// Parent bits of I(i,1) and D(1,j) (their producers are boundary cells).
SALN_HD uint8_t ibits_col1(const Scoring &s, uint32_t i) {
    const int32_t ext = i_col0(s, i), open = kSentinel + s.gap_open;
    return (uint8_t)((ext >= open ? 1 : 0) | (open >= ext ? 2 : 0));
}
SALN_HD uint8_t dbits_row1(const Scoring &s, uint32_t j) {
    const int32_t ext = d_row0(s, j), open = kSentinel + s.gap_open;
    return (uint8_t)((ext >= open ? 1 : 0) | (open >= ext ? 2 : 0));
}

// int2 elements per boundary column of a multi-chunk / column-stripe pair:
// rows 1..len_db, then the row fill's pad slots len_db + 1 .. len_db + 8
// (where its lanes other than 63 publish); a multiple of four elements.
SALN_HD uint64_t scratch_col(uint32_t len_db) { return ((uint64_t)len_db + 13) & ~(uint64_t)3; }

// Scaled end value H'(len_db, len_q) when a length is 0.
SALN_HD int32_t hs_boundary_end(const Scoring &s, uint32_t len_q, uint32_t len_db) {
    if (len_db == 0) return hs_row0(s, len_q);
    return hs_col0(s, len_db);
}

}  // namespace saln

// NW-affine fill + canonical traceback kernels for gfx950 (MI355X).
//
// Reference path: src/needleman_wunsch_affine.rs — ScoreTensor::fill :169-237
// (recurrences m_score/i_score/d_score :76-94, parent lists :96-153) and
// ScoreTensor::traceback :242-334.
//
// Fill geometry ("skewed row pipeline"): a group of G lanes (G = 16: one DPP
// row; G = 64: the whole wave) owns one pair.  Lane l owns K consecutive
// query columns of the current chunk and walks the db rows; at step t it
// computes row r = t - l + 1, so the left neighbour finished the same row one
// step earlier.  The only cross-lane traffic per step is two DPP shifts
// (the row's I candidate leaving the lane's last column and the last
// column's H), fused as update_dpp moves.  Each lane keeps its previous-row
// H and next-row D for its K columns in registers; nothing else of the matrix
// is stored except the parent code per cell (1 B/cell), one ceil(K/4)-dword
// segment per lane and step, in the block-interleaved row-major layout of
// nw_common.hpp (Geom): the segments of one row and block of the pairs of a
// pack (64 consecutive pairs of a variant) are adjacent.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "nw_common.hpp"
#include "nw_host.hpp"
#include "saln_options.hpp"
#include "saln.h"

namespace saln {
bool stripe_packed(const Scoring &sc, uint64_t n_waves, bool wide, const Options &o);
}

namespace saln {

// lane i <- lane i-1 within the group; the group's lane 0 keeps `old`.
template <int G>
__device__ __forceinline__ int32_t shr1(int32_t old, int32_t v) {
    static_assert(G == 16 || G == 64, "group must be a DPP row or the wave");
    if constexpr (G == 16)
        return __builtin_amdgcn_update_dpp(old, v, 0x111 /*row_shr:1*/, 0xf, 0xf, false);
    else
        return __builtin_amdgcn_update_dpp(old, v, 0x138 /*wave_shr:1*/, 0xf, 0xf, false);
}

// Workgroups are dispatched round-robin over the 8 XCDs (block i -> XCD
// i % 8).  The bpp workgroups that fill one pack (64 consecutive pairs whose
// mask rows are interleaved) are remapped onto one XCD, so the partial lines
// they write meet in one L2.  The grid is a multiple of 8*bpp.
// (i: the block index, blockIdx.x unless a grid-stride loop runs virtual blocks)
__device__ __forceinline__ uint32_t pack_block(uint32_t bpp, uint32_t i = blockIdx.x) {
    const uint32_t sup = 8u * bpp;
    const uint32_t r = i % sup;
    return i - r + (r % 8u) * bpp + r / 8u;
}
constexpr uint32_t blocks_per_pack(uint32_t pairs_per_block) {
    return pairs_per_block >= 64 ? 1u : 64u / pairs_per_block;
}

// --------------------------------------------------------------- traceback
struct GeomTable {
    Geom g[kNumVariants];
};

struct MaskCell {
    const uint8_t *m;
    Geom g;
    uint64_t rs;
    uint32_t bs;
    uint64_t cs;
    Scoring sc;
    // codes are stored inverted (bit set = parent absent); bit 7 = q == d
    __device__ uint8_t byte(uint32_t i, uint32_t j) const { return m[g.cell(i, j, rs, bs, cs)] ^ 0x7F; }
    // walk-code view: boundary cells from the alive-preferring formulas
    __device__ uint8_t argmax(uint32_t i, uint32_t j) const {
        if (i == 0) return argmax_row0_walk(sc, j);
        if (j == 0) return argmax_col0_walk(sc, i);
        return byte(i, j) & 7;
    }
    __device__ uint8_t ibits(uint32_t i, uint32_t j) const {  // i, j >= 1
        return j == 1 ? ibits_col1_walk(sc, i) : (byte(i, j - 1) >> 3) & 3;
    }
    __device__ uint8_t dbits(uint32_t i, uint32_t j) const {  // i, j >= 1
        return i == 1 ? dbits_row1_walk(sc, j) : (byte(i - 1, j) >> 5) & 3;
    }
};

enum { kStM = 0, kStI = 1, kStD = 2 };
enum { kEvOrigin = 0, kEvPanic = 1, kEvDead = 2 };

// End states in the order the reference DFS pops them (:251-280 push I, M, D).
__device__ __forceinline__ int first_end_state(uint32_t es) {
    return (es & kArgD) ? kStD : ((es & kArgM) ? kStM : kStI);
}
// The end states after `st` in that order (st itself and those before it removed).
__device__ __forceinline__ uint32_t end_states_after(uint32_t es, int st) {
    return st == kStD ? es & (kArgM | kArgI) : st == kStM ? es & kArgI : 0u;
}

struct WalkOut {
    int ev;
    uint32_t nops;
};

// Greedy walk from cell (i, j) in state st over walk codes (D > I > M in an M
// cell, open > extend in I / D; the tied alive parents, nw_common.hpp), run-
// length ops back to front into out.  '=' / 'X' from the sequences when
// given, else from the codes' eq bit.  A walk started at an alive state ends
// at the origin or a panic node; one started at a dead state (a sentinel-
// rooted end state) ends at a sentinel root (kEvDead).
__device__ WalkOut walk_greedy(const MaskCell &mc, int st, uint32_t i, uint32_t j,
                               const uint8_t *q, const uint8_t *d, uint32_t *out) {
    uint32_t nops = 0, run_op = 0, run_len = 0;
    int ev;
    for (;;) {
        uint32_t op;
        if (st == kStM) {
            if (i == 0 && j == 0) { ev = kEvOrigin; break; }
            if (i == 0 || j == 0) { ev = kEvDead; break; }
            const bool eq = q ? q[j - 1] == d[i - 1] : (mc.byte(i, j) >> 7) != 0;
            op = eq ? SALN_CIGAR_EQ : SALN_CIGAR_X;
            const uint8_t a = mc.argmax(i - 1, j - 1);
            --i;
            --j;
            st = (a & kArgD) ? kStD : ((a & kArgI) ? kStI : kStM);
        } else if (st == kStI) {
            if (j == 0) { ev = i >= 1 ? kEvPanic : kEvDead; break; }
            if (i == 0) { ev = kEvDead; break; }
            op = SALN_CIGAR_I;
            const uint8_t b = mc.ibits(i, j);
            --j;
            st = (b & 2) ? kStM : kStI;
        } else {
            if (i == 0) { ev = j >= 1 ? kEvPanic : kEvDead; break; }
            if (j == 0) { ev = kEvDead; break; }
            op = SALN_CIGAR_D;
            const uint8_t b = mc.dbits(i, j);
            --i;
            st = (b & 2) ? kStM : kStD;
        }
        if (op == run_op && run_len) {
            ++run_len;
        } else {
            if (run_len && out) out[nops] = (run_len << 4) | run_op;
            nops += run_len ? 1 : 0;
            run_op = op;
            run_len = 1;
        }
    }
    if (run_len) {
        if (out) out[nops] = (run_len << 4) | run_op;
        ++nops;
    }
    if (ev != kEvOrigin) nops = 0;
    if (out) {  // ops were produced back to front
        for (uint32_t a = 0, b = nops ? nops - 1 : 0; a < b; ++a, --b) {
            const uint32_t tmp = out[a];
            out[a] = out[b];
            out[b] = tmp;
        }
    }
    return WalkOut{ev, nops};
}

// The reference DFS's first path from the end states `es` (the tied set),
// tried in pop order D, M, I: the first that is not dead decides (printed at
// the origin, or a panic with nothing printed); all dead = nothing printed.
__device__ WalkOut walk_first(const MaskCell &mc, uint32_t es, uint32_t ld, uint32_t lq,
                              const uint8_t *q, const uint8_t *d, uint32_t *out) {
    WalkOut w{kEvDead, 0};
    while (es) {
        const int st = first_end_state(es);
        w = walk_greedy(mc, st, ld, lq, q, d, out);
        if (w.ev != kEvDead) break;
        es = end_states_after(es, st);
    }
    return w;
}

__device__ __forceinline__ saln_nw_result make_result(int32_t hend, WalkOut w, uint32_t es) {
    saln_nw_result r;
    r.score = hend >> 1;
    r.status = (hend & 1) ? SALN_REF_PANIC_BOUNDARY : SALN_OK;
    r.cigar_len = w.nops;
    r.end_states = (uint8_t)es;
    r.printed = w.ev == kEvOrigin ? 1 : 0;
    r.flags = (w.ev == kEvPanic && !(hend & 1)) ? 2 : 0;  // diagnostic: never set
    r.reserved = 0;
    return r;
}

// Canonical (first printed) alignment: the reference DFS pops end states in
// the order D, M, I (:251-280 push I, M, D) and parents in reverse push order
// (M: D>I>M; I: open>extend; D: open>extend).  Over walk codes (the alive
// tied parents) the first path is this greedy walk from the first end state
// that is not dead (walk_first).
__device__ __forceinline__ void walk_pair(const NwPairDesc &p, int32_t hend,
                                       const uint8_t *__restrict__ qs,
                                       const uint8_t *__restrict__ ds,
                                       const uint8_t *__restrict__ mask, Geom geo,
                                       saln_nw_result *__restrict__ results,
                                       uint32_t *__restrict__ cigar, Scoring sc) {
    const uint32_t lq = p.len_q, ld = p.len_db;
    const MaskCell mc{mask + p.mask_off, geo, p.mask_rs, p.mask_bs, p.mask_cs, sc};
    // the reference's end states (true ties: boundary formulas, or the last
    // row's codes, which the fills store unfiltered)
    const uint8_t es = ld == 0 ? argmax_row0(sc, lq)
                     : lq == 0 ? argmax_col0(sc, ld) : (mc.byte(ld, lq) & 7);
    const WalkOut w = walk_first(mc, es, ld, lq, qs + p.q_off, ds + p.db_off,
                                 cigar ? cigar + p.cigar_off : nullptr);
    results[p.pair_id] = make_result(hend, w, es);
}

// LDS-window walker (walk_pack_lds; segments of <= 16 bytes, i.e. K <= 16).
// Lock-step phases: every lane of the wave is in the same window phase S
// (0..W-1) with its target row == base - S (phases unrolled).  The windows live in LDS, filled by LDS-DMA (global_load_lds_dwordx{3,4}:
// lane l's bytes land at slot base + 16*l; the slot base is wave-uniform
// because all lanes are in the same phase).  Block b lives in window b % NW
// (WalkGeo); at the end of phase S every lane refills slot S of every window
// with row base-S-W of the blocks {B, .., B-NW+1} (B = its current block),
// so when the walk crosses into block B-1 the data is already resident.
// valid bits track which slots of each window hold the block currently
// assigned to it; a crossing that comes back faster than the refills falls
// back to a synchronous load.
// Decisions are table lookups on the raw code byte: three bits at a
// state-dependent offset index kNextLut (no branches on the state).  The
// walk records 3-bit ops (state | eq << 2, ten per word) and stores complete
// words at phase ends, before the DMAs; the CIGAR (forward
// order, run-length words) is produced from that stream after the walk.
// Exactly NW DMAs per phase (the init issues the same group per slot) keep
// >= NW*(W-1) younger VMEM operations behind any slot a phase reads, so the
// read waits with that vmcnt in the same asm statement (the compiler cannot
// hoist it or turn it into a conservative vmcnt(0)).  Extra VMEM operations
// (op-stream stores, fallback loads) only make that wait more conservative.
constexpr uint32_t kOpsPerWord = 10;                     // 3-bit ops per op-stream word

// Window geometry of the walker for K columns per block: NW windows (blocks
// B, .., B-NW+1 resident) of W slots (rows).  A slot holds 16 bytes per lane
// (the LDS-DMA lane stride, also for dwordx3).  Each phase end issues the NW
// DMAs (always) after the op-stream store (only when a word is complete), so
// a phase reads the slot its DMA filled W-1 phases earlier behind >= NW*(W-1)
// younger VMEM operations.  A phase waits for a DMA issued W-1 phases earlier,
// but at the C2 scale the walk is bound by the DMA stream itself, not by that
// latency: round 3 measured (NW x W) 2 x 4 0.26 ms, 2 x 8 0.28, 3 x 4 0.30,
// 3 x 6 0.30 (tools/exp_ab_c2.sh, one box), so the default is the leanest.
// NW = 3 keeps block B-2 resident too (no synchronous reload when a path
// crosses two blocks within W rows) and was slower.
// kNib: 4-bit walk codes (Geom::LBn-byte segments) and the pair's query
// staged in LDS after the windows: QC 16-byte chunks per lane, [chunk][lane]
// (the LDS-DMA order), enough for a variant of `cols` query columns at any
// 16-byte misalignment.
template <int K, bool kNib = false, uint32_t kCols = 0>
struct WalkGeo {
    static constexpr uint32_t LB = kNib ? 4 * ((K + 3) / 4 / 2 + 1) : (K + 3) / 4 * 4;
    static constexpr uint32_t NW = 2;
    static constexpr uint32_t W = K < 16 || kNib ? 4 : 8;
    static constexpr uint32_t SB = LB == 12 ? 12 : 16;        // DMA bytes per lane
    static constexpr uint32_t kSlotBytes = 64 * 16;          // one slot of a wave
    static constexpr uint32_t kWinBytes = W * kSlotBytes;    // one window of a wave
    static constexpr uint32_t QC = kNib ? (15 + kCols + 15) / 16 : 0;
    static constexpr uint32_t kWaveLds = NW * kWinBytes + QC * kSlotBytes;
    static constexpr uint32_t kVmcnt = NW * (W - 1);
    static_assert(LB <= 16, "LDS window slots hold 16 bytes per lane");
    static_assert((NW == 2 || NW == 3) && W >= 2 && W <= 8, "8 valid bits per window");
    static_assert(!kNib || kCols > 0, "4-bit walk: the variant's query width");
};

typedef __attribute__((address_space(3))) uint8_t lds_u8;

__device__ __forceinline__ uint32_t lds_off(const lds_u8 *p) { return (uint32_t)(uintptr_t)p; }

// A store the compiler can neither merge nor drop: the walker's vmcnt
// arithmetic counts every one of them.
__device__ __forceinline__ void counted_store(uint32_t *ptr, uint32_t v) {
    asm volatile("global_store_dword %0, %1, off" : : "v"(ptr), "v"(v) : "memory");
}

// Next state from the current state st (M, I, D, or 3 = at the end cell)
// and the three raw code bits at offset kLutShift(st): M reads bits 1-3
// (argI, argD; D > I > M), I bits 3-5 (I-open > extend), D bits 5-7 (D-open
// > extend), the end cell bits 0-2 (argM, argI, argD; D > M > I).
__host__ __device__ constexpr uint32_t next_state_raw(uint32_t st, uint32_t f) {
    const uint32_t pr = f ^ 7u;  // present bits (bit 2 of the D view is eq: unused)
    return st == 0 ? ((pr & 2) ? kStD : (pr & 1) ? kStI : kStM)
         : st == 1 ? ((pr & 2) ? kStM : kStI)
         : st == 2 ? ((pr & 2) ? kStM : kStD)
                   : ((pr & 4) ? kStD : (pr & 1) ? kStM : kStI);
}
__host__ __device__ constexpr uint64_t make_next_lut() {
    uint64_t l = 0;
    for (uint32_t st = 0; st < 4; ++st)
        for (uint32_t f = 0; f < 8; ++f) l |= (uint64_t)next_state_raw(st, f) << (16 * st + 2 * f);
    return l;
}
constexpr uint64_t kNextLut = make_next_lut();

// One 16-byte read of the lane's slot (the segment of its block at the
// phase's row), once at most N younger VMEM operations are outstanding.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <uint32_t N>
__device__ __forceinline__ u32x4 window_seg(uint32_t addr) {
    static_assert(N < 64, "vmcnt immediate");
    u32x4 v;
    asm volatile("s_waitcnt vmcnt(%2)\n\tds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(v) : "v"(addr), "n"(N) : "memory");
    return v;
}

template <typename F, uint32_t... I>
__device__ __forceinline__ void unroll_each(F &&f, std::integer_sequence<uint32_t, I...>) {
    (f(std::integral_constant<uint32_t, I>{}), ...);
}

// The walk (round 3: one iteration per row, and a shorter instruction stream
// than the round-2 walker; the windows, refills and counted waits are kept).  A
// wave iterates while any of its 64 lanes is still in the row, and an I step
// (a gap in the query: a move left) keeps a lane in its row, so the wave
// used to run ~2.8 iterations per row for ~1.05 per lane (PMC: 441 LDS reads
// per wave for ~157 rows).  Here an iteration reads the lane's whole segment
// (ds_read_b128) and, after the cell step of an M / D / end-cell state, walks
// an I run to its end within the block at once: the I-open bits of the
// segment's bytes (bit 4, stored inverted) are gathered into a mask whose
// highest set bit at or left of the lane's column is the cell where the run
// opens (at most nine cells per iteration, so the ops fit the accumulator).
// Only a run that leaves the block takes another iteration.
// - addresses are 64-bit lane pointers updated by adds: the row pointer of
//   the phase (one subtract per phase) and the block offsets held by window
//   0 / 1 (a crossing recomputes only the one it hands to block B-2);
// - the op stream is a 64-bit accumulator (stored 30 bits = ten ops at a time).
// kNib (round 4): 4-bit codes (nw_fill_pk_kernel kCodesNib).  The nibble of
// column col is read at the bit nib_bit(col) of dword col / 8; the lookup
// offsets become M 0 (argI, argD), I 1 (I-open), D 2 (D-open) instead of the
// byte's 1 / 3 / 5, so the same kNextLut decides; the end cell's state set
// is its nibble's argI, argD and (last row) argM-in-D-open bits; '=' / 'X'
// compare the query byte (LDS) with the row's db char in the segment.
template <int G, int K, bool kNib = false>
__device__ void walk_pack_lds(const NwPairDesc &p, int32_t hend, const uint8_t *__restrict__ mask,
                              uint32_t *__restrict__ ops_all, saln_nw_result *__restrict__ results,
                              uint32_t *__restrict__ cigar, Scoring sc, lds_u8 *win,
                              const uint8_t *__restrict__ qs) {
    using WG = WalkGeo<K, kNib, G * K>;
    constexpr Geom geo{G, K};
    constexpr uint32_t kW = WG::W, NW = WG::NW;
    constexpr uint32_t kWin = WG::kWinBytes, kSlot = WG::kSlotBytes;
    constexpr uint64_t kMask30 = (1u << 30) - 1u;
    const uint64_t rs = p.mask_rs, cs = p.mask_cs;
    const uint32_t bs = p.mask_bs;
    const uint8_t *__restrict__ m = mask + p.mask_off;
    uint32_t *out = cigar ? cigar + p.cigar_off : nullptr;
    uint32_t *const ops = ops_all + p.ops_off;
    // block b's segment at row 1, relative to m
    auto boff = [&](uint32_t b) __attribute__((always_inline)) {
        // (4-bit codes: queries of <= G * K columns, one chunk, b < G)
        if constexpr (kNib) return (uint64_t)(b * bs);
        else return (uint64_t)(b / G) * cs + (uint64_t)((b % G) * bs);
    };
    uint64_t acc = 0;        // pending 3-bit ops (state | eq << 2), oldest lowest
    uint32_t sh = 0, wi = 0; // acc's bit count; op words stored
    uint32_t ti = p.len_db, tj = p.len_q;
    uint32_t sidx = 3u * 16u, lsh = 0;  // kNextLut row of the state (3: end cell), its bits
    uint32_t walking = 1;
    uint32_t B = (tj - 1) / K, col = (tj - 1) % K;
    // block b lives in window b % NW: wc holds B, the windows below it (mod
    // NW) B-1 (and B-2); ow<w> is the block offset window w is loaded from
    uint32_t wc = B % NW;
    uint32_t valid = NW == 3 ? 0xFFFFFFu : 0xFFFFu;  // bit 8w + s: slot s of window w is current
    uint64_t ow0 = 0, ow1 = 0, ow2 = 0;
    auto set_ow = [&](uint32_t w, uint64_t o) __attribute__((always_inline)) {
        ow0 = w == 0 ? o : ow0;
        ow1 = w == 1 ? o : ow1;
        if constexpr (NW == 3) ow2 = w == 2 ? o : ow2;
    };
    auto get_ow = [&](uint32_t w) __attribute__((always_inline)) {
        return NW == 3 ? (w == 0 ? ow0 : w == 1 ? ow1 : ow2) : (w == 0 ? ow0 : ow1);
    };
    for (uint32_t b = 0; b < NW; ++b)  // blocks B, B-1, .. (clamped to block 0)
        set_ow((B + NW - b) % NW, boff(B >= b ? B - b : 0));
    const uint32_t wbase = lds_off(win) + (threadIdx.x & 63u) * 16u;
    // kNib: the query's 16-byte chunks (aligned; a chunk holding one of the
    // query's bytes never crosses into an unmapped page) into LDS, ahead of
    // every window DMA, so the counted waits below also cover them
    const uint32_t qa = (uint32_t)(p.q_off & 15u);
    lds_u8 *const qlds = win + NW * kWin;
    if constexpr (kNib) {
        const uint8_t *qg = qs + (p.q_off - qa);
        const uint32_t qlast = (qa + p.len_q - 1u) / 16u;
#pragma unroll
        for (uint32_t c = 0; c < WG::QC; ++c)
            __builtin_amdgcn_global_load_lds(qg + 16u * (c < qlast ? c : qlast),
                                             (__attribute__((address_space(3))) void *)(qlds + c * kSlot),
                                             16, 0, 0);
    }
    // query column j (1-based) of this lane's pair equals the db char dch
    auto qeq = [&](uint32_t j, uint32_t dch) __attribute__((always_inline)) {
        const uint32_t o = qa + j - 1u;
        return (uint32_t)qlds[(o >> 4) * kSlot + (threadIdx.x & 63u) * 16u + (o & 15u)] == dch;
    };
    // db char byte of a 4-bit segment (Geom::nib_char_byte)
    constexpr uint32_t kNG = (K + 3) / 4, kCB = kNG % 2 ? 4 * (kNG / 2) + 2 : 4 * (kNG / 2);
    // bit of column c's nibble in its dword (dword c / 8)
    auto nib_bit = [](uint32_t c) __attribute__((always_inline)) {
        return ((c & 4u) << 2) | ((c & 1u) << 3) | (c & 2u) << 1;
    };
    // kNib: the end cell's raw (absent) M, I, D bits from its nibble
    auto end_bits = [](uint32_t n4) __attribute__((always_inline)) {
        return ((n4 >> 3) & 1u) | ((n4 & 3u) << 1);
    };
    uint32_t wl = wbase + wc * kWin;  // my slot 0 in the current window
    // the phase's row pointer (row ti at a phase start), W rows ahead for the refills
    // (row counts on after the lane's walk ends; rows below 1 load row 1)
    const uint8_t *rp = m + (uint64_t)(ti - 1) * rs;
    int32_t row = (int32_t)ti;
    const uint64_t rsW = (uint64_t)kW * rs;
    auto dma = [&](auto win_c, auto slot_c, const uint8_t *a) __attribute__((always_inline)) {
        constexpr uint32_t w = decltype(win_c)::value, s = decltype(slot_c)::value;
        __builtin_amdgcn_global_load_lds(
            a, (__attribute__((address_space(3))) void *)(win + w * kWin + s * kSlot), WG::SB, 0,
            0);
    };
    // Slot S of both windows <- the row W phases ahead: the lane's block B
    // (window wc) while it walks, block B-1 only when the lane may cross into
    // it within W rows (col < W + 2: a diagonal path moves a column per row; a
    // longer I run takes ensure()'s synchronous reload).  The other lanes load
    // their pair's first segment (one line per pack, cached): every lane
    // issues exactly NW DMAs per phase, as the counted waits need, but a
    // finished lane or a far block costs no HBM request (round 5: the
    // walker's window loads were half of its co-run cost, a no-load timing
    // probe ran the pipelined C2 step 0.82-0.84 ms against 0.90-0.91).
    // Sets slot S's validity: wc's when walking, the other window's iff near.
    static_assert(NW == 2, "two windows: the lane's block and the one left of it");
    auto refill = [&](auto slot_c, const uint8_t *row) __attribute__((always_inline)) {
        constexpr uint32_t S = decltype(slot_c)::value;
        const bool near = walking && col < kW + 2u;
        const bool own0 = walking && wc == 0u, own1 = walking && wc == 1u;
        dma(std::integral_constant<uint32_t, 0>{}, slot_c, (own0 || near) ? row + ow0 : m);
        dma(std::integral_constant<uint32_t, 1>{}, slot_c, (own1 || near) ? row + ow1 : m);
        const uint32_t mine = 1u << (wc * 8u + S), other = 1u << ((wc ^ 1u) * 8u + S);
        valid = (valid | mine | (near ? other : 0u)) & ~(near ? 0u : other);
    };
    // slot S of the current window not refreshed since a crossing: load it now
    auto ensure = [&](auto slot_c) __attribute__((always_inline)) {
        constexpr uint32_t S = decltype(slot_c)::value;
        if (!((valid >> (wc * 8u + S)) & 1u)) {
            const uint8_t *a = rp + get_ow(wc);
            if (wc == 0) dma(std::integral_constant<uint32_t, 0>{}, slot_c, a);
            __builtin_amdgcn_sched_barrier(0);
            if (wc == 1) dma(std::integral_constant<uint32_t, 1>{}, slot_c, a);
            if constexpr (NW == 3) {
                __builtin_amdgcn_sched_barrier(0);
                if (wc == 2) dma(std::integral_constant<uint32_t, 2>{}, slot_c, a);
            }
            asm volatile("s_waitcnt vmcnt(0)" : : : "memory");
            valid |= 1u << (wc * 8u + S);
        }
    };
    auto flush = [&]() __attribute__((always_inline)) {
        counted_store(ops + wi, (uint32_t)(acc & kMask30));
        acc >>= 30;
        sh -= 30;
        ++wi;
    };
    // into block B-1 (the window below wc) at its last column; window wc takes B-NW
    auto cross = [&]() __attribute__((always_inline)) {
        set_ow(wc, boff(B >= NW ? B - NW : 0));
        valid &= ~(0xFFu << (wc * 8u));
        wc = wc == 0 ? NW - 1 : wc - 1;
        wl = wbase + wc * kWin;
        --B;
        col = K - 1;
    };
    auto pick = [](const u32x4 &v, uint32_t k) __attribute__((always_inline)) {
        if constexpr (WG::LB <= 8) return k == 0 ? v.x : v.y;
        else if constexpr (WG::LB <= 12) return k == 0 ? v.x : k == 1 ? v.y : v.z;
        else return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
    };
    // bit c set: the I-open parent of byte c is present (bit 4 clear); the
    // multiply gathers bits 4, 12, 20, 28 of a dword into bits 25..28
    auto iopen = [](uint32_t d) __attribute__((always_inline)) {
        return __builtin_amdgcn_ubfe((~d & 0x10101010u) * 0x00204081u, 25, 4);
    };
    // kNib: a 16-bit group half holds the I-open bits (nibble bit 2) of its
    // columns 0..3 at bits 2, 10, 6, 14; the multiply by 0x285 gathers them in
    // column order into bits 11..14 (a 24-bit multiply: full rate, where the
    // 32-bit one is quarter rate)
    auto iopen_n = [](uint32_t h) __attribute__((always_inline)) {
        return __builtin_amdgcn_ubfe((uint32_t)__umul24(~h & 0x4444u, 0x285u), 11, 4);
    };
    auto iopen_n8 = [&](uint32_t d) __attribute__((always_inline)) {
        return iopen_n(d) | (iopen_n(d >> 16) << 4);
    };
    auto iopen_mask = [&](const u32x4 &v) __attribute__((always_inline)) {
        if constexpr (kNib) {
            uint32_t pm = iopen_n8(v.x);
            if constexpr (K > 8) pm |= iopen_n8(v.y) << 8;
            if constexpr (K > 16) pm |= iopen_n8(v.z) << 16;
            return pm;
        } else {
            uint32_t pm = iopen(v.x) | (iopen(v.y) << 4);
            if constexpr (WG::LB > 8) pm |= iopen(v.z) << 8;
            if constexpr (WG::LB > 12) pm |= iopen(v.w) << 12;
            return pm;
        }
    };
    constexpr uint32_t kOnes3 = 0x09249249u;  // op I (1) in each of nine 3-bit slots
    auto phase = [&](auto slot_c) __attribute__((always_inline)) {
        constexpr uint32_t S = decltype(slot_c)::value;
        // the row W phases ahead (rows below 1 load row 1: the count stays exact)
        const uint8_t *ahead = row > (int32_t)kW ? rp - rsW : m;
        if (walking) {
            ensure(slot_c);
            for (;;) {
                if (sh >= 30) flush();  // at most 30 bits per iteration follow
                const u32x4 seg = window_seg<WG::kVmcnt>(wl + S * kSlot);
                if (sidx != 16u) {  // a cell step in state M, D or at the end cell
                    uint32_t f3, eqb;
                    if constexpr (kNib) {
                        const uint32_t dw = pick(seg, col >> 3);
                        f3 = sidx == 48u ? end_bits(__builtin_amdgcn_ubfe(dw, nib_bit(col), 4))
                                         : __builtin_amdgcn_ubfe(dw, nib_bit(col) + lsh, 3);
                        const uint32_t dch = __builtin_amdgcn_ubfe(pick(seg, kCB >> 2), (kCB & 3u) * 8u, 8);
                        eqb = qeq(tj, dch) ? 1u : 0u;
                    } else {
                        const uint32_t dw = pick(seg, col >> 2), b8 = (col & 3u) * 8u;
                        f3 = __builtin_amdgcn_ubfe(dw, b8 + lsh, 3);
                        eqb = __builtin_amdgcn_ubfe(dw, b8 + 7u, 1);
                    }
                    const uint32_t nx = (uint32_t)(kNextLut >> (f3 * 2u + sidx)) & 3u;
                    acc |= (uint64_t)(nx | (eqb << 2)) << sh;
                    sh += 3;
                    sidx = nx * 16u;
                    lsh = kNib ? nx : 2u * nx + 1u;
                    const bool up = nx != kStI, left = nx != kStD;
                    ti -= up ? 1u : 0u;
                    tj -= left ? 1u : 0u;
                    const bool done = ti == 0 || tj == 0;
                    bool crossed = false;
                    if (left && !done) {
                        if (col == 0) {
                            cross();
                            crossed = true;
                        } else {
                            --col;
                        }
                    }
                    if (up || done) {
                        walking = done ? 0u : 1u;
                        break;
                    }
                    if (crossed) {  // the run goes on in the other window
                        ensure(slot_c);
                        continue;
                    }
                }
                // state I at column col: extends up to the first present I-open
                const uint32_t lo = col >= 8u ? col - 8u : 0u;
                const uint32_t pm = iopen_mask(seg) & ((2u << col) - 1u) & (~0u << lo);
                if (pm) {  // opens at c1: ops I x (col - c1), then M, diagonal from c1
                    const uint32_t c1 = 31u - (uint32_t)__builtin_clz(pm), n = col - c1;
                    uint32_t eqb;
                    if constexpr (kNib)
                        eqb = qeq(tj - n, __builtin_amdgcn_ubfe(pick(seg, kCB >> 2), (kCB & 3u) * 8u, 8))
                                  ? 1u : 0u;
                    else
                        eqb = __builtin_amdgcn_ubfe(pick(seg, c1 >> 2), (c1 & 3u) * 8u + 7u, 1);
                    acc |= (uint64_t)((kOnes3 & ((1u << (3u * n)) - 1u)) | (eqb << (3u * n + 2u)))
                           << sh;
                    sh += 3u * (n + 1u);
                    sidx = 0;
                    lsh = kNib ? 0u : 1u;
                    ti -= 1;
                    tj -= n + 1u;
                    const bool done = ti == 0 || tj == 0;
                    if (!done) {
                        if (c1 == 0) cross();
                        else col = c1 - 1u;
                    }
                    walking = done ? 0u : 1u;
                    break;
                }
                const uint32_t n = col - lo + 1u;  // extends through column lo
                acc |= (uint64_t)(kOnes3 & ((1u << (3u * n)) - 1u)) << sh;
                sh += 3u * n;
                tj -= n;
                if (tj == 0) {
                    walking = 0;
                    break;
                }
                if (lo == 0) cross();
                else col = lo - 1u;
                ensure(slot_c);
            }
        }
        if (sh >= 30) flush();
        refill(slot_c, ahead);
        rp -= rs;
        --row;
    };
    // the first W rows; then exactly NW DMAs per phase, for every lane still walking
    unroll_each([&](auto slot_c) __attribute__((always_inline)) {
        constexpr uint32_t S = decltype(slot_c)::value;
        refill(slot_c, ti > S ? rp - (uint64_t)S * rs : m);
    }, std::make_integer_sequence<uint32_t, kW>{});
    while (walking) unroll_each(phase, std::make_integer_sequence<uint32_t, kW>{});
    const uint32_t st = sidx / 16u;
    int ev, bst;
    if (st == kStM && ti == 0 && tj == 0) {
        ev = kEvOrigin;
    } else {
        if (st == kStM) {
            const uint8_t a = ti == 0 ? argmax_row0_walk(sc, tj) : argmax_col0_walk(sc, ti);
            bst = (a & kArgD) ? kStD : ((a & kArgI) ? kStI : kStM);
        } else if (st == kStI) {
            bst = (ibits_col1_walk(sc, ti) & 2) ? kStM : kStI;
        } else {
            bst = (dbits_row1_walk(sc, tj) & 2) ? kStM : kStD;
        }
        if (bst == kStD && ti == 0 && tj >= 1) ev = kEvPanic;
        else if (bst == kStI && tj == 0 && ti >= 1) ev = kEvPanic;
        else ev = kEvDead;
    }
    // the reference's end states: the last row's codes are stored unfiltered
    // (kNib: the end cell's nibble, argM in its D-open bit)
    uint32_t es;
    if constexpr (kNib) {
        const uint32_t c = (p.len_q - 1) % K, b = (p.len_q - 1) / K;
        const uint32_t w = *reinterpret_cast<const uint32_t *>(
            m + (uint64_t)(p.len_db - 1) * rs + boff(b) + 4u * (c >> 3));
        es = ~end_bits(__builtin_amdgcn_ubfe(w, nib_bit(c), 4)) & 7u;
    } else {
        es = (m[geo.cell(p.len_db, p.len_q, rs, bs, cs)] ^ 0x7Fu) & 7u;
    }
    uint32_t nops = 0;
    bool retried = false;
    // (4-bit codes are written by the packed fills only: sentinel-free pairs,
    // no dead end state)
    if (!kNib && ev == kEvDead) {
        // the first end state is sentinel-rooted (i32 lanes pairs only): the
        // DFS goes on with the next tied end states (walk_first, byte loads)
        const uint32_t rest = end_states_after(es, first_end_state(es));
        if (rest) {
            const MaskCell mc{m, geo, rs, bs, cs, sc};
            const WalkOut w = walk_first(mc, rest, p.len_db, p.len_q, nullptr, nullptr, out);
            ev = w.ev;
            nops = w.nops;
            retried = true;
        }
    }
    // CIGAR: the op stream read back in forward order (last recorded op
    // first), a run at a time: each word's ten 3-bit ops become 2-bit classes
    // (0 '=', 1 I, 2 D, 3 X) with a few mask operations, the class changes
    // between neighbouring slots are a bit mask, and the loop visits the runs
    // (clz of the changes below the current slot) instead of the ops; the next
    // word's load is issued a word ahead.
    if (ev == kEvOrigin && !retried) {
        const uint32_t nrec = wi * kOpsPerWord + sh / 3;
        if (sh) counted_store(ops + wi, (uint32_t)(acc & kMask30));
        if (sh > 30) counted_store(ops + wi + 1, (uint32_t)(acc >> 30));
        asm volatile("s_waitcnt vmcnt(0)" : : : "memory");
        constexpr uint32_t kSlots = 0x09249249u;  // bit 0 of each 3-bit slot
        constexpr uint32_t kOpOf = (SALN_CIGAR_X << 12) | (SALN_CIGAR_D << 8) |
                                   (SALN_CIGAR_I << 4) | SALN_CIGAR_EQ;  // by class
        static_assert(SALN_CIGAR_X < 16 && SALN_CIGAR_EQ < 16, "4-bit CIGAR ops");
        uint32_t run_cls = 4u, run_len = 0;
        int32_t w = (int32_t)((nrec - 1u) / kOpsPerWord);
        uint32_t word = ops[w], nxt = w > 0 ? ops[w - 1] : 0u;
        uint32_t top = (nrec - 1u) % kOpsPerWord;
        for (; w >= 0; --w, top = kOpsPerWord - 1) {
            const uint32_t cur = word;
            word = nxt;
            nxt = w >= 2 ? ops[w - 2] : 0u;
            const uint32_t s0 = cur & kSlots, s1 = (cur >> 1) & kSlots, e = (cur >> 2) & kSlots;
            const uint32_t xm = ~(s0 | s1 | e) & kSlots;  // M without the '=' bit: X
            const uint32_t c0 = s0 | xm, c1 = s1 | xm;    // class bits 0, 1 per slot
            // slot k (k < top) starts a new run below slot k+1
            const uint32_t chg = ((c0 ^ (c0 >> 3)) | (c1 ^ (c1 >> 3))) & kSlots &
                                 ((1u << (3u * top)) - 1u);
            int32_t pos = (int32_t)top;  // the highest slot not yet counted
            for (;;) {
                const uint32_t below = chg & ((1u << (3u * (uint32_t)pos)) - 1u);
                const int32_t b = below ? (31 - __builtin_clz(below)) / 3 : -1;  // next run's top slot
                const uint32_t cls = ((c0 >> (3u * (uint32_t)pos)) & 1u) |
                                     (((c1 >> (3u * (uint32_t)pos)) & 1u) << 1);
                const uint32_t len = (uint32_t)(pos - b);
                if (cls != run_cls) {
                    if (run_len) {
                        if (out) out[nops] = (run_len << 4) | ((kOpOf >> (4u * run_cls)) & 15u);
                        ++nops;
                    }
                    run_cls = cls;
                    run_len = 0;
                }
                run_len += len;
                if (b < 0) break;
                pos = b;
            }
        }
        if (run_len) {
            if (out) out[nops] = (run_len << 4) | ((kOpOf >> (4u * run_cls)) & 15u);
            ++nops;
        }
    }
    results[p.pair_id] = make_result(hend, WalkOut{ev, nops}, es);
}

// Per-variant traceback for filled pairs whose segments fit an LDS slot.
// kNib: 4-bit codes; two waves per workgroup (the query staging doubles the
// LDS of a wave).
template <int G, int K, bool kNib = false>
constexpr uint32_t tb_lds_threads() { return kNib ? 128u : 256u; }
template <int G, int K, bool kNib>
__global__ __launch_bounds__(256) void nw_traceback_lds_kernel(
    const NwPairDesc *__restrict__ pairs, uint32_t first, uint32_t n,
    const uint8_t *__restrict__ mask, const int32_t *__restrict__ end_h,
    uint32_t *__restrict__ ops, saln_nw_result *__restrict__ results,
    uint32_t *__restrict__ cigar, Scoring sc, const uint8_t *__restrict__ qs) {
    constexpr uint32_t kWave = WalkGeo<K, kNib, G * K>::kWaveLds;
    __shared__ __attribute__((aligned(16))) uint8_t win_all[tb_lds_threads<G, K, kNib>() / 64u * kWave];
    // The walk is a latency-bound chain that shares SIMDs with the VALU-bound
    // fill of the next batch in pipelined plans.  Issue priority against the
    // table fills (priority 2): above them for a lane's first pair, below
    // them for the next ones (a grid that walks two pairs per lane beside the
    // next fill).  Above throughout, the walk took 0.63 ms and the co-run fill
    // 0.84; below throughout, the walk outlasted the fill (0.83 against 0.74);
    // first above, then below: fill 0.82, walk 0.79, C2 step 0.861-0.865 ->
    // 0.844-0.852 ms (round 6, profiles/r06_prio_ab.jsonl, five calls).
    __builtin_amdgcn_s_setprio(3);
    lds_u8 *win = (lds_u8 *)(win_all + (threadIdx.x / 64u) * kWave);
    // a lane per pair; a grid smaller than the pairs walks them in turns (the
    // wave's lanes start their next pairs together, after the last of the
    // previous ones has finished)
    const uint32_t stride = gridDim.x * blockDim.x;
    bool later = false;
    for (uint32_t rel = blockIdx.x * blockDim.x + threadIdx.x; rel < n; rel += stride) {
        if (later) __builtin_amdgcn_s_setprio(1);
        later = true;
        const uint32_t idx = first + rel;
        const NwPairDesc p = pairs[idx];
        walk_pack_lds<G, K, kNib>(p, end_h[idx], mask, ops, results, cigar, sc, win, qs);
    }
}

// One walker per pair.  Pairs with an empty side have no mask and take the
// boundary-only walk.
__global__ __launch_bounds__(256) void nw_traceback_kernel(
    const NwPairDesc *__restrict__ pairs, uint32_t first, uint32_t n,
    const uint8_t *__restrict__ qs, const uint8_t *__restrict__ ds,
    const uint8_t *__restrict__ mask, const int32_t *__restrict__ end_h,
    saln_nw_result *__restrict__ results, uint32_t *__restrict__ cigar, Scoring sc,
    GeomTable gt) {
    const uint32_t idx = first + blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= first + n) return;
    const NwPairDesc p = pairs[idx];
    const Geom geo = gt.g[p.variant];
    walk_pair(p, p.len_q && p.len_db ? end_h[idx] : hs_boundary_end(sc, p.len_q, p.len_db), qs,
              ds, mask, geo, results, cigar, sc);
}

// ------------------------------------------------ render batches: next event
// What the reference DFS (needleman_wunsch_affine.rs:281-329) meets after the
// first printed alignment, decided on the GPU from a full-code plan's parent
// sets (saln_nw_render_batch: a pair whose text this decides is rendered from
// its CIGAR, with no mask download and no host DFS).  The DFS stack holds,
// when the first path reaches the origin, the parents each node of that path
// did not take (pushed in the order M, I, D / extend, open and popped in
// reverse) and, at the bottom, the tied end states after the first (:247-280);
// the next pop is the not-taken parent of the deepest node that has one.  In a
// sentinel-free pair every node reaches a terminal (the origin or a panic
// node), so the next event is the first terminal of the greedy walk from that
// parent: the origin = a second block, a panic node = the panic.  Codes:
// 0 none (exactly one block), 1 a second block, 2 a panic after the first
// block, 3 not decided here (sentinel-rooted subtrees: the host DFS decides).
// Pairs with nothing printed need no next event (0).
__global__ __launch_bounds__(256) void nw_next_event_kernel(
    const NwPairDesc *__restrict__ pairs, uint32_t n, const uint8_t *__restrict__ mask,
    const saln_nw_result *__restrict__ results, Scoring sc, GeomTable gt,
    uint8_t *__restrict__ next) {
    const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n) return;
    const NwPairDesc p = pairs[idx];
    const saln_nw_result r = results[p.pair_id];
    uint8_t out = kNextNone;
    if (r.printed && p.len_q && p.len_db) {
        if (!sentinel_free(sc, p.len_q, p.len_db)) {
            out = kNextHost;
        } else {
            const MaskCell mc{mask + p.mask_off, gt.g[p.variant], p.mask_rs, p.mask_bs, p.mask_cs, sc};
            int st = first_end_state(r.end_states);
            const uint32_t rest = end_states_after(r.end_states, st);
            int ast = rest ? first_end_state(rest) : -1;  // the next pop: an end state ...
            uint32_t ai = p.len_db, aj = p.len_q;
            uint32_t i = p.len_db, j = p.len_q;
            // ... unless a node of the first path left a parent (the deepest wins)
            for (uint32_t guard = 0; !(i == 0 && j == 0) && guard <= p.len_q + p.len_db; ++guard) {
                int ps[3];
                uint32_t pi[3], pj[3];
                int np = 0;
                auto push = [&](int s2, uint32_t i2, uint32_t j2) {
                    ps[np] = s2;
                    pi[np] = i2;
                    pj[np] = j2;
                    ++np;
                };
                if (i == 0 || j == 0) break;  // (a printed first path meets no other boundary cell)
                if (st == kStM) {
                    const uint8_t a = mc.argmax(i - 1, j - 1);
                    if (a & kArgM) push(kStM, i - 1, j - 1);
                    if (a & kArgI) push(kStI, i - 1, j - 1);
                    if (a & kArgD) push(kStD, i - 1, j - 1);
                } else if (st == kStI) {
                    const uint8_t b = mc.ibits(i, j);
                    if (b & 1) push(kStI, i, j - 1);
                    if (b & 2) push(kStM, i, j - 1);
                } else {
                    const uint8_t b = mc.dbits(i, j);
                    if (b & 1) push(kStD, i - 1, j);
                    if (b & 2) push(kStM, i - 1, j);
                }
                if (np == 0) break;
                if (np >= 2) {
                    ast = ps[np - 2];
                    ai = pi[np - 2];
                    aj = pj[np - 2];
                }
                st = ps[np - 1];
                i = pi[np - 1];
                j = pj[np - 1];
            }
            if (!(i == 0 && j == 0 && st == kStM)) {
                out = kNextHost;  // (not the printed path: leave it to the host DFS)
            } else if (ast >= 0) {
                const WalkOut w = walk_greedy(mc, ast, ai, aj, nullptr, nullptr, nullptr);
                out = w.ev == kEvOrigin ? kNextBlock : w.ev == kEvPanic ? kNextPanic : kNextHost;
            }
        }
    }
    next[p.pair_id] = out;
}

hipError_t launch_next_event(const NwPairDesc *pairs, uint32_t n, const uint8_t *mask,
                             const saln_nw_result *results, Scoring sc, uint8_t *next,
                             hipStream_t stream) {
    if (!n) return hipSuccess;
    GeomTable gt;
    for (int v = 0; v < kNumVariants; ++v) gt.g[v] = variant_geom(v);
    nw_next_event_kernel<<<dim3((n + 255) / 256), dim3(256), 0, stream>>>(pairs, n, mask, results,
                                                                       sc, gt, next);
    return hipGetLastError();
}

// ------------------------------------------- long pairs: cooperative walker
// One wave per pair (column-stripe pairs, K = 4).  The same greedy walk as
// walk_pair, but a step run is resolved by the whole wave at once: in state
// M lane l looks at the l-th diagonal step (eq bit of cell (i-l, j-l), next
// state from the argmax bits of (i-l-1, j-l-1)); in I / D lane l looks at the
// l-th extend step.  A ballot of "the run ends after my step" gives the run
// length, so a 64-step stretch of the path costs one round of LDS reads
// instead of 64 dependent ones.  The codes come from an LDS window over the
// stripe holding the current cell, rows [i-rows+1, i]: in the skewed stripe
// layout (nw_common.hpp) that is one contiguous run of lines, copied by
// LDS-DMA (1 KB per instruction) when a run would leave it.  A step into the
// previous stripe takes the current cell's eq bit from the old window and the
// rest from the new one.  CIGAR words are emitted back to front (uniform
// scalar run-length state) and reversed at the end.  The window height is the
// launch's choice (dynamic LDS of (rows + 64) lines): tall for a few long
// pairs (fewer reloads), short for batches (more waves per CU).
constexpr int32_t kCoopLine = 256;  // bytes per line (one stripe step)
constexpr int32_t kCoopSlack = 64;  // rows loaded beyond a diagonal crossing of the stripe

// kLay: 1 the
// packed stripe layout (bs == 0): virtual lane v = (c - c0) / 2 of row r sits
// on line r - 1 + v (127 lines of skew); 2 the row-major 256-column tiles of
// nw_fill_rows_kernel (no skew: row r is line r - 1).
// kSpec: one block per walker stripe of a long pair (SpecArgs, nw_common.hpp):
// the walk starts at the stripe's entry and stops where it leaves the stripe
// (the crossing step is the stripe's last op) or ends; it writes its run
// words and exit to the stripe's record.  A pass whose entry equals the one
// of the stored walk keeps it (the walk is a function of (cell, state)).
template <int NWV, int kLay, bool kSpec = false>
__global__ __launch_bounds__(64 * NWV) void nw_traceback_coop_kernel(
    const NwPairDesc *__restrict__ pairs, uint32_t first, const uint8_t *__restrict__ mask,
    const int32_t *__restrict__ end_h, saln_nw_result *__restrict__ results,
    uint32_t *__restrict__ cigar, Scoring sc, int32_t kCoopRows,
    const uint8_t *__restrict__ qs, const uint8_t *__restrict__ ds, SpecArgs sa) {
    static_assert(kLay == 1 || kLay == 2, "round 1's skewed i32 stripe layout is retired");
    constexpr bool kPk = kLay == 1;
    constexpr int32_t kSkew = kLay == 1 ? 127 : 0;  // lines from a row's first to its last block
    // kCoopRows + kSkew lines, rounded up to whole 4-line DMAs; then the
    // request words wave 0 posts to the loader waves
    extern __shared__ __attribute__((aligned(16))) uint8_t win[];
    int32_t *req = reinterpret_cast<int32_t *>(win + (kCoopRows + kSkew + 1) * kCoopLine);
    // kLay 2: the row fill's walk codes carry no eq bit; '=' / 'X' come from
    // the sequence bytes of the window, staged beside it: q[c_lo-2 ..
    // c_lo+254] (the stripe's columns and the one before) and d[r_lo-2 .. i-1]
    uint8_t *qwin = win + (kCoopRows + kSkew + 1) * kCoopLine + 16;
    uint8_t *dwin = qwin + 272;
    const int32_t lane = (int32_t)threadIdx.x % 64, wv = (int32_t)threadIdx.x / 64;
    uint32_t idx = first + blockIdx.x;
    SpecStripe *rec = nullptr;
    int32_t ei = 0, ej = 0, ek = 0, s_id = 0;  // kSpec: entry, stripe
    if constexpr (kSpec) {
        const uint2 b = sa.blocks[blockIdx.x];
        const SpecPair sp = sa.pairs[b.x];
        idx = sp.plan_idx;
        s_id = (int32_t)b.y;
        rec = sa.stripes + sp.stripe_base + b.y;
    } else if (sa.done && sa.done[idx]) {
        return;  // walked by the speculative passes
    }
    const NwPairDesc p = pairs[idx];
    const uint8_t *__restrict__ m = mask + p.mask_off;
    if constexpr (kSpec) {
        // every wave reads the same entry (nothing writes it in this pass)
        const int32_t lqp = (int32_t)p.len_q, ldp = (int32_t)p.len_db;
        const int32_t par = (sa.pass - 1) & 1, cur = sa.pass & 1;
        if (sa.entry_s1 && s_id == sa.entry_s1 - 1) {  // a span's rightmost stripe: its given entry
            ei = rec[1].out_i[par];
            ej = rec[1].out_j[par];
            ek = rec[1].out_k[par];
        } else if (s_id == (lqp - 1) / kCoopLine) {
            ei = ldp;
            ej = lqp;
            ek = kSpecEnd;
        } else if (sa.pass == 1) {  // guess: the proportional row, state M
            ej = kCoopLine * (s_id + 1);
            ei = (int32_t)min((int64_t)ldp, max((int64_t)1, (int64_t)ej * ldp / lqp));
            ek = kSpecM;
        } else {
            ei = rec[1].out_i[par];
            ej = rec[1].out_j[par];
            ek = rec[1].out_k[par];
        }
        if (ek >= kSpecEv) {  // the walk ends to the right of this stripe
            if (threadIdx.x == 0) {
                rec->in_k = kSpecNone;
                rec->out_k[cur] = kSpecNone;
                rec->nops = 0;
            }
            return;
        }
        if (sa.pass > 1 && rec->in_i == ei && rec->in_j == ej && rec->in_k == ek) {
            if (threadIdx.x == 0) {  // same entry: the stored walk stands
                rec->out_i[cur] = rec->out_i[par];
                rec->out_j[cur] = rec->out_j[par];
                rec->out_k[cur] = rec->out_k[par];
            }
            return;
        }
    }
    int32_t r_lo = 1, c_lo = 1;  // window: rows [r_lo, i], the stripe's columns [c_lo, c_lo+255]
    // Wave w's share of the window for cell (i, j): every NWV-th 4-line DMA.
    auto dma = [&](int32_t i, int32_t j, int32_t w) __attribute__((always_inline)) {
        const int32_t s = (j - 1) / kCoopLine;
        c_lo = s * kCoopLine + 1;
        // a near-diagonal path leaves the stripe after j - c_lo + 1 rows:
        // load those plus some slack for gaps, not the whole window height
        r_lo = max(1, i - min(kCoopRows, j - c_lo + 1 + kCoopSlack) + 1);
        // lines r_lo-1 .. i-1+kSkew of stripe s (row r of lane l is line r-1+l)
        const int32_t t_lo = r_lo - 1, t_hi = i - 1 + kSkew;
        const uint8_t *reg = m + (uint64_t)s * p.mask_cs;
        typedef __attribute__((address_space(3))) void lds_v;
        for (int32_t mm = w; 4 * mm <= t_hi - t_lo; mm += NWV) {
            const int32_t t = min(t_lo + 4 * mm + lane / 16, t_hi);  // clamped: stay in the region
            __builtin_amdgcn_global_load_lds(reg + (uint64_t)t * kCoopLine + 16 * (lane % 16),
                                             (lds_v *)(win + 4 * mm * kCoopLine), 16, 0, 0);
        }
        if constexpr (kLay == 2) {
            const int32_t lqp = (int32_t)p.len_q, ldp = (int32_t)p.len_db;
            for (int32_t k = w * 64 + lane; k < 257; k += NWV * 64) {
                const int32_t jq = c_lo - 2 + k;  // q index
                qwin[k] = jq >= 0 && jq < lqp ? qs[p.q_off + jq] : 0;
            }
            for (int32_t k = w * 64 + lane; k <= i - r_lo + 1; k += NWV * 64) {
                const int32_t id = r_lo - 2 + k;  // d index
                dwin[k] = id >= 0 && id < ldp ? ds[p.db_off + id] : 1;
            }
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): my share has landed
    };
    // Waves 1.. only load windows: wait for a request (i, j), or i < 0 = done.
    if (wv > 0) {
        for (;;) {
            __syncthreads();
            const int32_t qi = req[0], qj = req[1];
            if (qi < 0) return;
            dma(qi, qj, wv);
            __syncthreads();
        }
    }
    const int32_t hend = end_h[idx];
    const int32_t lq = (int32_t)p.len_q, ld = (int32_t)p.len_db;
    auto load = [&](int32_t i, int32_t j) __attribute__((always_inline)) {
        if (NWV > 1) {
            if (lane == 0) {
                req[0] = i;
                req[1] = j;
            }
            __syncthreads();
        }
        dma(i, j, 0);
        if (NWV > 1)
            __syncthreads();  // every share has landed
        else
            __builtin_amdgcn_wave_barrier();
    };
    // code byte of interior cell (r, c) inside the window, bits 0-6 present-sets
    auto code = [&](int32_t r, int32_t c) __attribute__((always_inline)) {
        const int32_t o = c - c_lo;
        if constexpr (kPk) {
            const int32_t v = o >> 1;
            return (uint32_t)win[(r - r_lo + v) * kCoopLine + 4 * (v & 63) + 2 * (o & 1) + (v >> 6)] ^
                   0x7Fu;
        }
        if constexpr (kLay == 2) return (uint32_t)win[(r - r_lo) * kCoopLine + o] ^ 0x7Fu;
        return (uint32_t)win[(r - r_lo + (o >> 2)) * kCoopLine + o] ^ 0x7Fu;
    };
    int32_t i = kSpec ? ei : ld, j = kSpec ? ej : lq;
    load(i, j);
    // the reference's end states (the last row's codes are unfiltered), tried
    // in the DFS's pop order: a walk from a sentinel-rooted end state dead-ends
    // and the next one is walked (walk_first)
    uint32_t am_end = 0, es_left = 0;
    int32_t st;
    if (!kSpec || ek == kSpecEnd) {
        am_end = code(i, j) & 7u;
        es_left = am_end;
        st = first_end_state(es_left);
        es_left = end_states_after(es_left, st);
    } else if (ek == kSpecViaM) {  // the step into (i, j) was diagonal: its argmax
        const uint32_t a = i == 0 ? argmax_row0_walk(sc, (uint32_t)j) : code(i, j) & 7u;
        st = (a & kArgD) ? kStD : ((a & kArgI) ? kStI : kStM);
    } else if (ek == kSpecViaI) {  // horizontal: the I bits of (i, j+1) sit at (i, j)
        st = ((code(i, j) >> 3) & 2u) ? kStM : kStI;
    } else {
        st = ek;
    }
    int32_t xi = 0, xj = 0, xk = kSpecNone;  // kSpec: exit
    uint32_t *out = kSpec ? sa.ops + (uint64_t)(rec - sa.stripes) * kSpecOpsCap
                          : cigar ? cigar + p.cigar_off : nullptr;
    uint32_t nops = 0, run_op = 0, run_len = 0;
    // The pending run is stored at out[nops] unconditionally (every lane, one
    // address): when it merges or is empty the slot is simply rewritten later.
    auto push = [&](uint32_t op, uint32_t len) __attribute__((always_inline)) {
        const bool merge = run_op == op;
        if (out) out[nops] = (run_len << 4) | run_op;
        nops += (!merge && run_len) ? 1u : 0u;
        run_len = merge ? run_len + len : len;
        run_op = op;
    };
    int ev;
    for (;;) {
        if (i == 0 || j == 0) {  // every end of the walk is on row or column 0
            if (st == kStM) ev = i == 0 && j == 0 ? kEvOrigin : kEvDead;
            else if (st == kStI) ev = j == 0 && i >= 1 ? kEvPanic : kEvDead;
            else ev = i == 0 && j >= 1 ? kEvPanic : kEvDead;
            if (kSpec || ev != kEvDead || !es_left) break;  // kSpec: the link checks
            // dead end state: restart from the next tied end state
            st = first_end_state(es_left);
            es_left = end_states_after(es_left, st);
            i = ld;
            j = lq;
            nops = run_op = run_len = 0;
            load(i, j);
            continue;
        }
        // steps l whose reads stay in the window (row / column 0 come from
        // the boundary formulas)
        const int32_t lim_i = r_lo == 1 ? i - 1 : i - 1 - r_lo;
        const int32_t lim_j = c_lo == 1 ? j - 1 : j - 1 - c_lo;
        if (i < r_lo || j < c_lo || (st != kStI && lim_i < 0)) {
            load(i, j);  // anchored at row i: lim_i >= 0 afterwards
            continue;
        }
        // j == c_lo > 1 and the step reads column j-1: one step, lane 0,
        // that column from global memory
        const bool edge = st != kStD && lim_j < 0;
        uint32_t eq0 = 0;
        if constexpr (kSpec) {
            // the crossing step is this stripe's last op (a span walk: only
            // where it leaves the span's first column)
            if (edge && (!sa.span || c_lo - 1 <= sa.span_c0)) {
                if (st == kStM) {
                    push((kLay == 2 ? qwin[j - c_lo + 1] == dwin[i - r_lo + 1] : (code(i, j) >> 7) != 0)
                             ? SALN_CIGAR_EQ : SALN_CIGAR_X, 1);
                    xi = i - 1;
                    xk = kSpecViaM;
                } else {
                    push(SALN_CIGAR_I, 1);
                    xi = i;
                    xk = kSpecViaI;
                }
                xj = j - 1;
                ev = -1;
                break;
            }
        }
        // q == d of cell (r, c) inside the window (kLay 2: from the staged bytes)
        auto eqbit = [&](int32_t r, int32_t c) __attribute__((always_inline)) -> uint32_t {
            if constexpr (kLay == 2)
                return qwin[c - c_lo + 1] == dwin[r - r_lo + 1] ? 1u : 0u;
            else
                return code(r, c) >> 7;
        };
        if (edge) {  // j == c_lo > 1: this step reads column j-1 of the previous stripe
            if (st == kStM) eq0 = eqbit(i, j);  // (i, j) leaves the window now
            load(i, j - 1);
        }
        int32_t lmax = edge ? 0 : st == kStM ? min(lim_i, lim_j) : st == kStI ? lim_j : lim_i;
        lmax = min(lmax, 63);
        // Every lane reads and decides (no divergent branches around the LDS
        // reads); lanes past lmax read outside the window - LDS returns 0 for
        // out-of-range addresses and their decisions are masked by `stop`.
        bool stop;
        int32_t nxt;
        uint32_t eq = 0;
        if (st == kStM) {  // wave-uniform
            const int32_t ni = i - lane - 1, nj = j - lane - 1;
            const uint32_t cn = code(ni, nj);
            eq = edge ? eq0 : eqbit(i - lane, j - lane);
            const uint32_t ab = ni == 0 ? argmax_row0_walk(sc, (uint32_t)nj)
                                        : argmax_col0_walk(sc, (uint32_t)ni);
            const uint32_t a = (ni == 0 || nj == 0) ? ab : cn & 7u;
            nxt = (a & kArgD) ? kStD : ((a & kArgI) ? kStI : kStM);
            stop = nxt != kStM || ni == 0 || nj == 0;
        } else if (st == kStI) {
            const int32_t cj = j - lane;
            const uint32_t cc = code(i, cj - 1);
            const uint32_t b = cj == 1 ? ibits_col1_walk(sc, (uint32_t)i) : (cc >> 3) & 3u;
            nxt = (b & 2) ? kStM : kStI;
            stop = nxt != kStI || cj == 1;
        } else {
            const int32_t ci = i - lane;
            const uint32_t cc = code(ci - 1, j);
            const uint32_t b = ci == 1 ? dbits_row1_walk(sc, (uint32_t)j) : (cc >> 5) & 3u;
            nxt = (b & 2) ? kStM : kStD;
            stop = nxt != kStD || ci == 1;
        }
        stop = stop || lane >= lmax;
        const uint64_t sb = __builtin_amdgcn_ballot_w64(stop);
        const int32_t L = __builtin_ctzll(sb);  // last step of this run (lane lmax always stops)
        const uint32_t n = (uint32_t)L + 1;
        if (st == kStM) {
            const uint64_t lm = n >= 64 ? ~0ull : ((1ull << n) - 1);
            const uint64_t e = __builtin_amdgcn_ballot_w64(eq != 0) & lm;
            const uint64_t bnd = (e ^ (e << 1)) & lm & ~1ull;  // steps whose op differs from the previous
            const uint32_t cur0 = (e & 1) ? SALN_CIGAR_EQ : SALN_CIGAR_X;
            const uint32_t other = cur0 == SALN_CIGAR_EQ ? SALN_CIGAR_X : SALN_CIGAR_EQ;
            const uint32_t k = (uint32_t)__builtin_popcountll(bnd);
            // segment 0 (up to the first boundary) joins or follows the pending run
            push(cur0, k ? (uint32_t)__builtin_ctzll(bnd) : n);
            if (k) {
                // the pending run ends at the first boundary; segments 1..k-1
                // are written in parallel by their boundary lanes; the last
                // segment is the new pending run
                if (out) out[nops] = (run_len << 4) | run_op;
                ++nops;
                if ((bnd >> lane) & 1) {
                    const uint32_t m = (uint32_t)__builtin_popcountll(bnd & ((1ull << lane) - 1)) + 1;
                    if (m < k && out) {
                        const uint32_t nb = (uint32_t)__builtin_ctzll(bnd & ~((2ull << lane) - 1));
                        out[nops + m - 1] = ((nb - (uint32_t)lane) << 4) | ((m & 1) ? other : cur0);
                    }
                }
                nops += k - 1;
                run_op = (k & 1) ? other : cur0;
                run_len = n - (uint32_t)(63 - __builtin_clzll(bnd));
            }
            i -= (int32_t)n;
            j -= (int32_t)n;
        } else if (st == kStI) {
            push(SALN_CIGAR_I, n);
            j -= (int32_t)n;
        } else {
            push(SALN_CIGAR_D, n);
            i -= (int32_t)n;
        }
        st = __builtin_amdgcn_readlane(nxt, L);
    }
    if (NWV > 1) {  // release the loader waves
        if (lane == 0) req[0] = -1;
        __syncthreads();
    }
    if (run_len) {
        if (lane == 0 && out) out[nops] = (run_len << 4) | run_op;
        ++nops;
    }
    if constexpr (kSpec) {
        if (lane == 0) {
            const int32_t cur = sa.pass & 1;
            rec->in_i = ei;
            rec->in_j = ej;
            rec->in_k = ek;
            rec->out_i[cur] = xi;
            rec->out_j[cur] = xj;
            rec->out_k[cur] = ev < 0 ? xk : kSpecEv + ev;
            rec->nops = nops;
            rec->am_end = am_end;
        }
        return;
    }
    if (ev != kEvOrigin) nops = 0;
    if (out && nops > 1) {  // words were produced back to front
        __builtin_amdgcn_s_waitcnt(0x0F70);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        for (uint32_t a = (uint32_t)lane; a < nops / 2; a += 64) {
            const uint32_t x = out[a], y = out[nops - 1 - a];
            out[a] = y;
            out[nops - 1 - a] = x;
        }
    }
    if (lane == 0) {
        saln_nw_result r = make_result(hend, WalkOut{ev, nops}, am_end);
        results[p.pair_id] = r;
    }
}

// Link of the speculative stripe walks of one pair (one block): the passes'
// walks form the sequential walk when, from the last stripe (entered at the
// end cell) down to the stripe t where the walk ends, each stripe's stored
// walk started where the final pass left the stripe after it.  Then the
// stripes' run words, concatenated in walk order with runs of one op merged
// across stripe boundaries, are the walk's CIGAR back to front: a block scan
// places each stripe's words (base, k0, the merged value of its last word)
// and nw_spec_copy_kernel writes them.  Otherwise, or when the walk ends dead
// (the next tied end state would be walked), the cooperative walker runs.
__global__ __launch_bounds__(256) void nw_spec_link_kernel(
    const NwPairDesc *__restrict__ pairs, SpecArgs sa, uint32_t *__restrict__ done,
    const int32_t *__restrict__ end_h, saln_nw_result *__restrict__ results,
    uint32_t *__restrict__ strict_err) {
    __shared__ uint32_t s_n[kSpecMaxStripes], s_first[kSpecMaxStripes], s_last[kSpecMaxStripes];
    __shared__ uint8_t s_k0[kSpecMaxStripes];
    __shared__ uint32_t s_part[256];
    __shared__ int32_t t_sh, bad_sh;
    const SpecPair sp = sa.pairs[blockIdx.x];
    const int32_t S = (int32_t)sp.n_stripes, P = sa.pass & 1;
    SpecStripe *rec = sa.stripes + sp.stripe_base;
    const uint32_t *ops = sa.ops + (uint64_t)sp.stripe_base * kSpecOpsCap;
    const int32_t tid = (int32_t)threadIdx.x;
    if (tid == 0) {
        t_sh = -1;
        bad_sh = 0;
    }
    __syncthreads();
    for (int32_t s = tid; s < S; s += 256)
        if (rec[s].out_k[P] >= kSpecEv) atomicMax(&t_sh, s);
    __syncthreads();
    const int32_t t = t_sh;
    const int32_t tk = t >= 0 ? rec[t].out_k[P] : kSpecNone;
    bool bad = t < 0 || tk == kSpecNone || tk == kSpecEv + kEvDead;
    for (int32_t s = max(t, 0) + tid; !bad && s < S - 1; s += 256) {
        const SpecStripe &a = rec[s], &b = rec[s + 1];
        if (a.in_i != b.out_i[P] || a.in_j != b.out_j[P] || a.in_k != b.out_k[P]) bad_sh = 1;
    }
    __syncthreads();
    const uint32_t idx = sp.plan_idx;
    if (bad || bad_sh) {
        if (tid == 0) {
            done[idx] = 0u;
            if (strict_err) atomicOr(strict_err, 2u);  // SALN_SPEC_STRICT: report the fallback
        }
        return;
    }
    for (int32_t s = tid; s < S; s += 256) {
        const uint32_t n = s >= t ? rec[s].nops : 0u;
        s_n[s] = n;
        s_first[s] = n ? ops[(uint64_t)s * kSpecOpsCap] : 0u;
        s_last[s] = n ? ops[(uint64_t)s * kSpecOpsCap + n - 1] : 0u;
        if (s < t) rec[s].k0 = (int32_t)n;  // nothing to copy
    }
    __syncthreads();
    // Walk order is stripe S-1 down to t.  After a non-empty stripe the open
    // (last) output word has the op of the stripe's last word whether or not
    // the stripe merged into it, so stripe s merges its first word (k0 = 1)
    // iff its op is that of stripe s+1's last word (every stripe above t
    // holds its crossing step, so s+1 is never empty).  A stripe starts
    // c = n - k0 output words; base(s) = (words of the stripes above) - k0.
    for (int32_t s = tid; s < S; s += 256)
        s_k0[s] = (s >= t && s < S - 1 && s_n[s] && (s_first[s] & 15u) == (s_last[s + 1] & 15u))
                      ? 1u : 0u;
    __syncthreads();
    // suffix sums of c over chunks of consecutive stripes (walk order)
    const int32_t C = (S + 255) / 256;
    const int32_t u0 = tid * C, u1 = min(S, u0 + C);  // u = S - 1 - s
    uint32_t part = 0;
    for (int32_t u = u0; u < u1; ++u) part += s_n[S - 1 - u] - s_k0[S - 1 - u];
    s_part[tid] = part;
    __syncthreads();
    for (int32_t d = 1; d < 256; d <<= 1) {  // inclusive scan of the chunk sums
        const uint32_t v = tid >= d ? s_part[tid - d] : 0u;
        __syncthreads();
        s_part[tid] += v;
        __syncthreads();
    }
    uint32_t g = s_part[tid] - part;  // words before my chunk
    for (int32_t u = u0; u < u1; ++u) {
        const int32_t s = S - 1 - u;
        const uint32_t n = s_n[s], k0 = s_k0[s];
        rec[s].base = (int32_t)g - (int32_t)k0;
        rec[s].k0 = (int32_t)k0;
        if (n > k0) {  // my last word opens an output word: add the first words merged into it
            uint32_t len = s_last[s] >> 4;
            for (int32_t r = s - 1; r >= t && s_k0[r]; --r) {
                len += s_first[r] >> 4;
                if (s_n[r] != 1u) break;
            }
            rec[s].open_w = (len << 4) | (s_last[s] & 15u);
        }
        g += n - k0;
    }
    if (tid == 255) {
        const uint32_t N = s_part[255];
        const NwPairDesc p = pairs[idx];
        const int ev = tk - kSpecEv;
        results[p.pair_id] = make_result(end_h[idx], WalkOut{ev, ev == kEvOrigin ? N : 0u},
                                         rec[S - 1].am_end);
        done[idx] = 1u;
    }
}

// Writes the linked stripes' run words front to back (one block per stripe).
__global__ __launch_bounds__(64) void nw_spec_copy_kernel(
    const NwPairDesc *__restrict__ pairs, SpecArgs sa, const saln_nw_result *__restrict__ results,
    uint32_t *__restrict__ cigar) {
    const uint2 b = sa.blocks[blockIdx.x];
    const SpecPair sp = sa.pairs[b.x];
    if (!sa.done[sp.plan_idx]) return;
    const NwPairDesc p = pairs[sp.plan_idx];
    const int32_t N = (int32_t)results[p.pair_id].cigar_len;
    const SpecStripe &r = sa.stripes[sp.stripe_base + b.y];
    const int32_t n = (int32_t)r.nops;
    if (N == 0 || r.k0 >= n) return;
    const uint32_t *w = sa.ops + (uint64_t)(sp.stripe_base + b.y) * kSpecOpsCap;
    uint32_t *out = cigar + p.cigar_off;
    for (int32_t k = r.k0 + (int32_t)threadIdx.x; k < n; k += 64)
        out[N - 1 - (r.base + k)] = k == n - 1 ? r.open_w : w[k];
}

template <int K>
struct MaskWords {
    uint32_t w[(K + 3) / 4];
};


// ----------------------------------------------------- long pairs: stripes
// One wave per column stripe of G*K = 64*K columns; all stripes of a pair run
// concurrently as a pipeline down the rows (the "anti-diagonal tiling across
// CUs" of configs[3]).  Stripe c's last lane publishes, per row, the H and
// I-candidate leaving its last column as one 64-bit agent-coherent store into
// scratch column c, which the host preset to kColEmpty: each row is its own
// publication, so the producer never waits for its stores (a progress counter
// behind a vmcnt(0) cost ~1 us per 32 rows on the critical path, 11 % of
// configs[3]).  Stripe c+1 polls 32-row blocks of that column with
// agent-coherent loads until no lane sees the preset.  (A release/acquire
// pair would write back and invalidate the whole L2 at every publication.)
// Work items
// are ordered pair-major, chunk-ascending, so a stripe's predecessor always
// has a lower workgroup id and has been dispatched before it (no deadlock);
// a bounded spin turns a lost dependency into an error flag instead of a hang.
constexpr uint32_t kPub = 32;
// the boundary column's preset (H word): no fill value comes near INT32_MIN
constexpr uint32_t kColEmpty = 0x80000000u;
// err[0]: flags (bit 0: a dependency wait timed out), err[1]: the polls a
// wait may spend before it gives up (the plan's wait limit, default 2^24;
// tests set it to 0 to inject a timeout)

// ------------------------------------------------------- packed-i16 fill
// Two pairs per lane group: pair A in the low 16 bits of every register,
// pair B in the high 16 bits, so every v_pk_* instruction advances two cells.
//
// Representation: X~(r,c) = X'(r,c) + alpha*r + beta*c, X' the flag-in-LSB
// scaled score (nw_common.hpp).  With alpha + beta = -2*match the diagonal
// step is M~ = H~(r-1,c-1) - pen*[q != d] (pen = 2*(match - mismatch)); with
// beta = -2*gap_extend the I recurrence is a bare max: I~(r,c+1) =
// max(M~ + 2*gap_open, I~); D~(r+1,c) = max(M~ + 2*gap_open, D~) + 2*ge + alpha.
// All parent decisions compare values of the same cell, where the offsets
// cancel.  Offsets are even, so the panic flag in the LSB survives.
// Mismatch detection: chars are carried as c << 5, so (q ^ d) is 0 on a match
// and >= 32 otherwise; pen = min_u16(q ^ d, pen_max).
// Parent codes come from sign bits of same-cell differences (1 = parent
// absent): v_perm's sign-replicating selectors (8..11) gather two signs per
// pair into 0x00/0xFF bytes, v_and_or weights them into bit positions.
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ s16x2 as_s2(uint32_t x) { return __builtin_bit_cast(s16x2, x); }
__device__ __forceinline__ uint32_t as_u(s16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ s16x2 spl(int32_t v) { return s16x2{(short)v, (short)v}; }
__device__ __forceinline__ uint32_t pk2(int32_t lo, int32_t hi) {
    return ((uint32_t)lo & 0xFFFFu) | ((uint32_t)hi << 16);
}
__device__ __forceinline__ s16x2 vmax(s16x2 a, s16x2 b) { return __builtin_elementwise_max(a, b); }
// Biased pair word: each half holds v + 32768 (an unsigned 16-bit number
// ordered like v).  Inside the packed region every value stays in
// [-30000, 30000], so 32-bit adds / subtracts of these words never carry or
// borrow across the halves (SWAR: one full-rate v_add/v_sub_u32 per two
// cells), and a half's bit 15 of a 32-bit difference is the sign of that
// half's difference; the low half's borrow only lowers the high half by 1,
// which the comparisons below tolerate by never letting a high half be 0.
__device__ __forceinline__ uint32_t pkb(int32_t lo, int32_t hi) {
    return ((uint32_t)(lo + 32768) & 0xFFFFu) | ((uint32_t)(hi + 32768) << 16);
}
__device__ __forceinline__ uint32_t umax2(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a),
                                                                  __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t umin2(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a),
                                                                  __builtin_bit_cast(u16x2, b)));
}
// constant c in both halves, as the 32-bit addend that adds c to each half
// of a biased word (for c < 0 it is the two's complement of |c| * 0x10001)
__device__ __forceinline__ uint32_t cst2(int32_t c) { return (uint32_t)c * 0x10001u; }

// lane <- lane-1 of the same group; a group's first lane takes `bnd`.
template <int G>
__device__ __forceinline__ uint32_t gshift(uint32_t bnd, uint32_t v, bool group_start) {
    uint32_t s;
    if constexpr (G <= 16)
        s = __builtin_amdgcn_update_dpp(bnd, v, 0x111 /*row_shr:1*/, 0xf, 0xf, false);
    else
        s = __builtin_amdgcn_update_dpp(bnd, v, 0x138 /*wave_shr:1*/, 0xf, 0xf, false);
    if constexpr (G == 16 || G == 64) return s;
    return group_start ? bnd : s;
}

// Sign bytes of one code source t over two columns: the (A, B) halves of
// s_t at columns k-1 (lo) and k (hi) -> 0x00/0xFF bytes [A_k-1, B_k-1, A_k, B_k].
__device__ __forceinline__ uint32_t col_pair_signs(uint32_t hi, uint32_t lo) {
    return __builtin_amdgcn_perm(hi, lo, 0x0B0A0908u);
}

// (m & a) | (~m & b) as one v_bitop3_b32 (truth table 0xCA over m, a, b).
// Written as the gfx950 builtin: plain C makes the compiler turn a chain of
// these into an and per source plus or3s, and inline asm (round 2) made it
// pad dependent ops with s_nop (it cannot see an asm instruction's hazards).
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
    return __builtin_amdgcn_bitop3_b32(m, a, b, 0xCA);
}

// Merge the sign-byte words of the code sources (bit t of every cell byte
// from source t) with a v_bfi chain: each step keeps the bits below the next
// source and takes the rest from it.  Walk codes have no sources for bits 3
// and 5; those bits then hold a copy of the next source (the walker never
// reads them in walk mode).  argM (bit 0) is only read at the end cell; rows
// that hold no end cell get a copy of bit 1 there.
template <bool kArgMBit>
__device__ __forceinline__ uint32_t merge_walk(const uint32_t (&p)[8]) {
    uint32_t r = kArgMBit ? bfi(0x01010101u, p[0], p[1]) : p[1];
    r = bfi(0x03030303u, r, p[2]);
    r = bfi(0x07070707u, r, p[4]);
    r = bfi(0x1F1F1F1Fu, r, p[6]);
    return bfi(0x7F7F7F7Fu, r, p[7]);
}
__device__ __forceinline__ uint32_t merge_full(const uint32_t (&p)[8]) {
    uint32_t r = bfi(0x01010101u, p[0], p[1]);
    r = bfi(0x03030303u, r, p[2]);
    r = bfi(0x07070707u, r, p[3]);
    r = bfi(0x0F0F0F0Fu, r, p[4]);
    r = bfi(0x1F1F1F1Fu, r, p[5]);
    r = bfi(0x3F3F3F3Fu, r, p[6]);
    return bfi(0x7F7F7F7Fu, r, p[7]);
}

template <int K>
struct PkMask {
    uint32_t w[(K + 3) / 4];
};
// h[k] for a lane-varying k < K: a select tree over the bits of k (one
// condition per level, ceil(log2 K) of them) instead of K compares, which
// would each hold a lane mask (SGPR pressure, spills for K = 19).
template <int K>
__device__ __forceinline__ uint32_t pick_col(const uint32_t (&h)[K], int k) {
    uint32_t v[K];
#pragma unroll
    for (int i = 0; i < K; ++i) v[i] = h[i];
    int n = K;
#pragma unroll
    for (int bit = 0; (1 << bit) < K; ++bit) {
        const bool b = (k >> bit) & 1;
#pragma unroll
        for (int i = 0; 2 * i < n; ++i) v[i] = 2 * i + 1 < n ? (b ? v[2 * i + 1] : v[2 * i]) : v[2 * i];
        n = (n + 1) / 2;
    }
    return v[0];
}
// One pair's 4-bit walk-code segment of K columns (Geom::LBn bytes).
template <int K>
struct NibSeg {
    uint32_t w[(K + 3) / 4 / 2 + 1];
};

// kCodes: kCodesWalk stores walk codes only (argM/argI/argD, I-open, D-open,
// eq) - the
// bits the device walker reads; the extend bits (3, 5) are left 0.  Full
// codes (every parent set) are kept for the dense-mask / render paths.
// kCodesNib (round 4): 4-bit walk codes, two cells per byte - bit 0 argI,
// 1 argD, 2 I-open, 3 D-open, each set when the parent is ABSENT - plus the
// row's db char in the segment; no eq bit (the walker compares the query
// byte, staged in LDS, with that char).  The end cell's state set needs
// argM: in a pair's last row the walker reads only I-open (a cell there is
// entered from its right neighbour or is the end cell), so the end cell's
// lane stores argM in the D-open bit of that row.  Layout of a
// segment (Geom::LBn): the 4-column groups g = c / 4 as 16-bit halves, two
// per dword, in each half the nibble of column c at bit 8 (c & 1) +
// 4 ((c >> 1) & 1); then the db char at byte Geom::nib_char_byte.
enum { kCodesWalk = 0, kCodesFull = 1, kCodesNone = 2, kCodesNib = 3 };

// Where the packed fill gets its pairs and puts the end values.
// PlanSrc: the plan's sorted descriptor table; the scaled end value goes to
// end_h for the traceback / score-results kernels.
struct PlanSrc {
    const NwPairDesc *pairs;
    uint32_t first;
    int32_t *end_h;
    __device__ __forceinline__ NwPairDesc pair(uint32_t i) const { return pairs[first + i]; }
    __device__ __forceinline__ void end(uint32_t i, const NwPairDesc &, int32_t h) const {
        end_h[first + i] = h;
    }
};

// AvsaSrc: score-only all-vs-all (configs[4]) without descriptors.  Pair
// k = base + i of a query class is (class query k % nq, db record k / nq) -
// both pairs of a lane group usually share the db record; the result
// {score, status} goes straight to out[d * nq_total + q], the reference's
// db-outer / query-inner order (main.rs:61-62).
struct AvsaSrc {
    const uint64_t *q_off, *d_off;  // full CSR offsets (n+1)
    const uint32_t *q_ids, *d_ids;  // the class's queries, the non-empty db records
    uint32_t nq;                    // queries in the class
    uint32_t nq_total;
    uint64_t base;
    int2 *out;
    __device__ __forceinline__ NwPairDesc pair(uint32_t i) const {
        const uint64_t k = base + i;
        const uint32_t qi = q_ids[k % nq], di = d_ids[k / nq];
        NwPairDesc p{};
        p.q_off = q_off[qi];
        p.db_off = d_off[di];
        p.len_q = (uint32_t)(q_off[qi + 1] - p.q_off);
        p.len_db = (uint32_t)(d_off[di + 1] - p.db_off);
        p.mask_off = (uint64_t)di * nq_total + qi;  // result slot (no mask in this mode)
        return p;
    }
    __device__ __forceinline__ void end(uint32_t, const NwPairDesc &p, int32_t h) const {
        out[p.mask_off] = make_int2(h >> 1, (h & 1) ? SALN_REF_PANIC_BOUNDARY : SALN_OK);
    }
};

// The same index space paired for a shared query profile (round 4): pair k is
// (class query (k/2) % nq, db record 2*((k/2)/nq) + k%2), so the two pairs of
// a lane group (2g, 2g+1) hold one query against two neighbouring db records
// (the db list is sorted by length: the halves stay balanced).  nd_pairs
// counts whole db pairs; an odd last db record goes through AvsaSrc.
struct AvsaSrcP : AvsaSrc {
    __device__ __forceinline__ NwPairDesc pair(uint32_t i) const {
        const uint64_t k = base + i, j = k >> 1;
        const uint32_t qi = q_ids[j % nq], di = d_ids[2 * (j / nq) + (k & 1)];
        NwPairDesc p{};
        p.q_off = q_off[qi];
        p.db_off = d_off[di];
        p.len_q = (uint32_t)(q_off[qi + 1] - p.q_off);
        p.len_db = (uint32_t)(d_off[di + 1] - p.db_off);
        p.mask_off = (uint64_t)di * nq_total + qi;
        return p;
    }
};

// KS: mask block width (the layout's K, the walker's geometry): a lane's K
// columns are stored as K/KS segments of KS codes.  KS < K lets a narrower
// lane group (G*K = the same width, fewer lanes: less pipeline skew, per-step
// overhead spread over more columns) write the layout of the wider one.
//
// kRebase: pairs whose db is too long for one int16 frame (packed_ok_rebase).
// Every kRebaseSteps steps all carried values drop by the column-0 drift of
// that many rows, (2*gap_extend + alpha) * kRebaseSteps (even: flags
// survive), so a value at step t is X~ - (2*ge + alpha) * r0(t), r0(t) = t
// rounded down to the period; a lane's rows are then within period + G of
// r0 and the values within the bound of a (period + G)-row pair.  Parent
// codes compare values of one cell (frame-free); group-start inputs and end
// values convert with r0(t).
constexpr int kRebaseSteps = 64;
// The column term of the frame bound is one-sided (a row's values exceed its
// column-0 value by up to c*(2|m| + 4|ge|) and fall below it by at most a
// small constant): the frame is centred on half the widest chunk's term.
__host__ __device__ inline int32_t rebase_center(const Scoring &sc, int32_t W) {
    const int32_t m = sc.match < 0 ? -sc.match : sc.match;
    const int32_t ge = sc.gap_extend < 0 ? -sc.gap_extend : sc.gap_extend;
    return (W * (2 * m + 4 * ge) / 2) & ~1;
}

// (Built for one wave per SIMD: at 124 VGPRs it runs 4; built for 5, 96
// VGPRs, it spills 26 registers: C2 fill 0.97 -> 1.57 ms, round 1.)
// The 8 x 19 fill with 4-bit codes needs ~183 VGPRs in its generic steps
// (the steady loop ~126): built for 3 waves per SIMD instead of 2.
template <int G, int K, int kCodes>
constexpr int pk_min_waves() { return kCodes == 3 /* kCodesNib */ && G == 8 ? 3 : 1; }
// kProf (score-only all-vs-all, AvsaSrcP): both halves hold one query, so a
// column's penalty for the row's two db chars is one v_perm of a per-column
// profile (the penalty against A, C, T, G in bytes 0-3; code = (char >> 1) & 3)
// with a per-step selector from the row word, instead of an xor and a packed
// min (and the wait state after the min).  Valid while every query and db
// byte is one of A, C, G, T (the launch checks the sequences on the device).
// kTab (4-bit walk codes, one frame; round 4): alpha = beta = -2*gap_extend,
// so neither gap extension adds anything (D~(r+1,c) = max(M~ + 2*gap_open,
// D~), no per-column add) and the diagonal step is M~ = H~(r-1,c-1) + bonus,
// bonus = 2*match - 4*gap_extend on a match and 2*mismatch - 4*gap_extend
// otherwise (both in [0, 255]: pk_tab_ok), one v_perm of a constant table
// selected by (q code ^ d code) in each half's low byte; the row word holds
// the db codes with 0x0C (v_perm's zero byte) in each half's high byte.
// Codes are (char >> 1) & 3 for A, C, T, G; a wave with any other byte in its
// pairs returns before its first step (fill_pk_body returns 1) and its
// kernel marks the launch in its plan's bail word; the fallback launch behind
// it (kTabMode 2: the generic 4-bit-code body) runs only when the word holds
// its launch, and then only in the waves that found such a byte.  Every value
// stays within the packed bound: X~ = X' + 2|ge|(r + c) lies in
// [-(4|go| + ...), rows (2|m| + 2|ge|) + 2|ge| lq] (X' is at least its
// all-gap path, at most its all-match one).
constexpr int32_t kFreeBias = 4096;
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
// max of three words of two biased halves read as positive normal f16 (one
// v_pk_maximum3_f16); exact only inside the extension-free frame's window
__device__ __forceinline__ uint32_t hmax3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_bit_cast(
        uint32_t, __builtin_elementwise_maximum(__builtin_bit_cast(f16x2, a),
                                                __builtin_elementwise_maximum(
                                                    __builtin_bit_cast(f16x2, b),
                                                    __builtin_bit_cast(f16x2, c))));
}

// A step's row input: the packed db word of its row.
struct RowIn {
    uint32_t w;
};

// Returns (per lane; wave-uniform over the lanes that hold pairs): 0 filled
// (or no pair), 1 the table body left the wave's pairs to the fallback launch
// (a byte other than A, C, G, T), 2 the fallback body found nothing to do.
template <int G, int K, int kCodes, typename Src, int KS, bool kRebase = false, bool kProf = false,
          int kTabMode = 0>
__device__ __forceinline__ int fill_pk_body(Src src, uint32_t count, const uint8_t *__restrict__ qs,
                                            const uint8_t *__restrict__ ds,
                                            uint8_t *__restrict__ mask, Scoring sc,
                                            uint32_t ld_max, bool sc_steady,
                                            uint32_t vblock = ~0u) {
    // table body (kTabMode 1; 4: the same at scale 4, below); kTabMode 2: the
    // generic body of its bail-outs
    constexpr bool kTab = kTabMode == 1 || kTabMode == 4 || kTabMode == 5;
    // kTabMode 5 (round 6): the table body with row profiles.  A step builds
    // its row's two profiles - the bonus of every query code against the
    // row's db char of pair A (lo) and of pair B (hi): cmm in each byte, cm in
    // byte code(char) - with one v_lshl_add each from the staged word
    // [8 code(A), 0x60, 8 code(B), 0x60], so a column's bonus is one v_perm
    // with a per-column selector of its query codes instead of an xor and a
    // v_perm (~19 fewer VALU per step for K = 19).  The staged word >> 3 is
    // the table body's [code(A), 0x0C, code(B), 0x0C] (the segment's chars).
    // (A first version staged both profiles in LDS, 10 B per row: fill -4.5 %
    // alone, but three fill workgroups then took the CU's LDS and the
    // pipelined walk lost its room: C2 step 0.86 -> 0.99 ms.)
    constexpr bool kRowProf = kTabMode == 5;
    // the extension-free frame (alpha = beta = -2*gap_extend, M~ = H~ + bonus):
    // the table body, and kTabMode 3 = query profiles holding bonuses
    constexpr bool kFree = kTab || kTabMode == 3;
    // kTabMode 4 (round 6): values carried as V = 4x + p instead of 2x + p
    // (bit 1 always 0).  The walk tests then have a strict margin on both
    // sides: argI present <=> (H - 2) - I < 0 (present: -2 + p_H - p_I in
    // [-2, -1], since a tied I's flag is in H's; absent: >= 4 - 2 - 1), I-open
    // present <=> (tO + 2) - I >= 1 (absent <= -4 + 3), so each is one full-rate
    // 32-bit v_sub_u32 on the pair word (a low half's borrow lowers the high
    // half by 1, which neither margin minds) instead of a quarter-rate
    // v_pk_sub_i16, and the flag masks (H & ~1, tO | 1) become the two adds.
    constexpr bool kS4 = kTabMode == 4;
    constexpr int kSc = kS4 ? 4 : 2;  // value scale
    // 2V + p (the boundary helpers, the end values) <-> kSc V + p
    auto up = [](int32_t v2) -> int32_t { return kS4 ? (v2 >> 1) * 4 + (v2 & 1) : v2; };
    static_assert(kTabMode != 3 || kProf, "kTabMode 3: query profiles");
    // The extension-free frame's values lie in a narrow window above about
    // -(6|go| + 6|ge|) (pk_free_ok): biased by kFreeBias they are the bit
    // patterns of positive normal halves, [0x0400, 0x7BFF], whose order is
    // their integer order, so H = max(M, I, D) is one v_pk_maximum3_f16.
    constexpr int32_t kBias = kFree ? kFreeBias : 32768;
    auto pkx = [](int32_t lo, int32_t hi) {
        return ((uint32_t)(lo + kBias) & 0xFFFFu) | ((uint32_t)(hi + kBias) << 16);
    };
    static_assert(!kProf || (kCodes == kCodesNone && !kRebase), "profiles: score-only, one frame");
    static_assert(!kTab || ((kCodes == kCodesNib || kCodes == kCodesNone || kCodes == kCodesFull) &&
                            !kRebase && !kProf && !(kS4 && kCodes == kCodesFull)),
                  "tables: 4-bit codes, full codes (scale 2) or score-only, one frame");
    constexpr int GPB = 256 / G;
    constexpr Geom geo{G, K};
    extern __shared__ uint32_t drow[];  // [GPB][G + ld_max + G] packed db chars (dch) per row
    const int lane = threadIdx.x % G;
    // (vblock: the block of a grid-stride launch, nw_fill_pk_tabfb_kernel)
    const uint32_t gi = pack_block(blocks_per_pack(2 * GPB), vblock == ~0u ? blockIdx.x : vblock) * GPB +
                        threadIdx.x / G;
    const uint32_t ia = 2 * gi, ib = 2 * gi + 1;
    if (ia >= count) return 0;  // whole group
    const bool hasB = ib < count;
    const NwPairDesc pa = src.pair(ia);
    NwPairDesc pb = pa;
    if (hasB) pb = src.pair(ib);
    const int ldA = (int)pa.len_db, ldB = hasB ? (int)pb.len_db : 0;
    const int lqA = (int)pa.len_q, lqB = hasB ? (int)pb.len_q : 0;
    const uint8_t *__restrict__ qA = qs + pa.q_off;
    const uint8_t *__restrict__ qB = qs + pb.q_off;
    const uint8_t *__restrict__ dA = ds + pa.db_off;
    const uint8_t *__restrict__ dB = ds + pb.db_off;
    const int ldM = ldA > ldB ? ldA : ldB;
    const int32_t beta = -kSc * sc.gap_extend;
    const int32_t alpha = kFree ? beta : -2 * sc.match - beta;
    const uint32_t kPen = cst2(2 * (sc.match - sc.mismatch));  // 0 < pen <= 32
    const uint32_t kOpen = cst2(kSc * sc.gap_open);
    const uint32_t kDstep = cst2(2 * sc.gap_extend + alpha);
    const int32_t drift = kFree ? 0 : 2 * sc.gap_extend + alpha;  // column-0 X~ per row
    // kTab: the diagonal bonus by (q code ^ d code) and the chars of codes 0-3
    const uint32_t cm = (uint32_t)(kSc * sc.match + alpha + beta) & 0xFFu;
    const uint32_t cmm = (uint32_t)(kSc * sc.mismatch + alpha + beta) & 0xFFu;
    const uint32_t kBonus = cm | cmm * 0x01010100u;
    const uint32_t kProfBase = cmm * 0x01010101u, kProfStep = cm - cmm;  // kRowProf
    const uint32_t kCmm2 = cmm * 0x00010001u;  // full codes' eq sign in the free frame
    constexpr uint32_t kAcgt = 'A' | 'C' << 8 | 'T' << 16 | 'G' << 24;
    auto acgt = [](uint32_t c) { return c == 'A' || c == 'C' || c == 'G' || c == 'T'; };
    bool bad = false;  // kTabMode: a byte other than A, C, G, T in this lane's share
    const uint32_t kRebaseAdd = cst2(-drift * kRebaseSteps);
    const int32_t ctr = kRebase ? rebase_center(sc, G * K) : 0;  // frame centring (kRebase)
    const bool gstart = lane == 0;

    const int col0 = lane * K;  // my columns: col0+1 .. col0+K
    // loop-carried state is kept as plain dwords (2 x i16) so the compiler
    // does not split it into halves
    uint32_t qc[K], Hp[K], Dn[K];
    const uint32_t pen1 = 2 * (sc.match - sc.mismatch);  // kProf: the mismatch byte
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int j = col0 + k + 1;
        if constexpr (kProf && kFree) {  // bonus against A, C, T, G; padding: all mismatch
            const uint32_t qch = j <= lqA ? (uint32_t)qA[j - 1] : 0u;
            qc[k] = (qch == 'A' ? cm : cmm) | (qch == 'C' ? cm : cmm) << 8 |
                    (qch == 'T' ? cm : cmm) << 16 | (qch == 'G' ? cm : cmm) << 24;
        } else if constexpr (kProf) {  // penalty against A, C, T, G (codes 0-3); padding: all mismatch
            const uint32_t qch = j <= lqA ? (uint32_t)qA[j - 1] : 0u;
            qc[k] = (qch == 'A' ? 0u : pen1) | (qch == 'C' ? 0u : pen1 << 8) |
                    (qch == 'T' ? 0u : pen1 << 16) | (qch == 'G' ? 0u : pen1 << 24);
        } else if constexpr (kTab) {  // codes in bytes 0 / 2 (padding: code 0)
            const uint32_t ca = j <= lqA ? (uint32_t)qA[j - 1] : 'A';
            const uint32_t cb = j <= lqB ? (uint32_t)qB[j - 1] : 'A';
            bad |= !acgt(ca) || !acgt(cb);
            // kRowProf: the v_perm selector of the row profiles (A: bytes 0-3
            // of the lo dword, B: bytes 4-7 = the hi dword; 0x0C = zero byte)
            qc[k] = kRowProf ? (((ca >> 1) & 3u) | 0x0C00u | (((cb >> 1) & 3u) + 4u) << 16 | 0x0C000000u)
                             : (((ca >> 1) & 3u) | ((cb >> 1) & 3u) << 16);
        } else {
            const uint32_t ca = j <= lqA ? (uint32_t)qA[j - 1] << 5 : 0xE000u;
            const uint32_t cb = j <= lqB ? (uint32_t)qB[j - 1] << 5 : 0xE000u;
            if constexpr (kTabMode == 2) bad |= (j <= lqA && !acgt(ca >> 5)) || (j <= lqB && !acgt(cb >> 5));
            qc[k] = ca | (cb << 16);
        }
        const int32_t h0 = up(hs_row0(sc, (uint32_t)j)) + beta * j - ctr;     // H~(0, j)
        const int32_t d1 = up(ds_row1(sc, (uint32_t)j)) + alpha + beta * j - ctr;  // D~(1, j)
        Hp[k] = pkx(h0, h0);
        Dn[k] = pkx(d1, d1);
    }
    uint32_t hd = pkx(up(hs_row0(sc, (uint32_t)col0)) + beta * col0 - ctr,
                      up(hs_row0(sc, (uint32_t)col0)) + beta * col0 - ctr);  // H~(r-1, col0)
    uint32_t pubF = 0, pubH = 0;
    // db chars of both pairs, staged once per group in LDS as the packed
    // (A << 5 | B << 21) word of each row; a step reads its row's word from
    // LDS (lgkmcnt), so no global load sits in the step loop next to the
    // mask stores (vmcnt).  Rows are padded by G words on both sides, so the
    // skewed row index r-1 of any lane at any step addresses the row without
    // a clamp (the pad words are only read by steps whose body is skipped).
    // kRebase (long db): the row's two chars as a 16-bit (A | B << 8) word,
    // half the LDS, widened in the step (one v_perm and a shift)
    uint32_t *__restrict__ myrow = drow + (threadIdx.x / G) * (ld_max + 2 * G) + G;
    uint16_t *__restrict__ myrow16 = reinterpret_cast<uint16_t *>(drow) +
                                     (threadIdx.x / G) * (ld_max + 2 * G) + G;
    for (int i = lane; i < ldM; i += G) {
        const uint32_t ca = i < ldA ? (uint32_t)dA[i] : 0u;
        const uint32_t cb = i < ldB ? (uint32_t)dB[i] : 0u;
        if constexpr (kRebase) {
            if constexpr (kTabMode == 2) bad |= (i < ldA && !acgt(ca)) || (i < ldB && !acgt(cb));
            myrow16[i] = (uint16_t)(ca | (cb << 8));
        } else if constexpr (kRowProf) {
            bad |= (i < ldA && !acgt(ca)) || (i < ldB && !acgt(cb));
            myrow[i] = ((ca >> 1) & 3u) << 3 | ((cb >> 1) & 3u) << 19 | 0x60006000u;
        } else if constexpr (kTab) {
            bad |= (i < ldA && !acgt(ca)) || (i < ldB && !acgt(cb));
            myrow[i] = ((ca >> 1) & 3u) | ((cb >> 1) & 3u) << 16 | 0x0C000C00u;
        } else {
            if constexpr (kTabMode == 2) bad |= (i < ldA && !acgt(ca)) || (i < ldB && !acgt(cb));
            myrow[i] = (ca << 5) | (cb << 21);
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" : : : "memory");
    __builtin_amdgcn_wave_barrier();
    if constexpr (kTab) {
        if (__builtin_amdgcn_ballot_w64(bad)) return 1;  // the wave is left to the fallback launch
    } else if constexpr (kTabMode == 2) {
        if (!__builtin_amdgcn_ballot_w64(bad)) return 2;  // done by the table launch
    }
    // end-cell owners
    const int lA = (lqA - 1) / K, kA = (lqA - 1) % K;
    const int lB = hasB ? (lqB - 1) / K : -1, kB = hasB ? (lqB - 1) % K : 0;
    // the step at which this lane holds a pair's end cell (row ld, its last column), or -1
    const int tEA = lane == lA ? ldA + lane - 1 : -1;
    const int tEB = lane == lB ? ldB + lane - 1 : -1;
    // this lane's segment of row r = t - lane + 1 (block = lane), advanced
    // by one row per step (64-bit adds instead of a row multiply per store)
    static_assert(K % KS == 0 && (KS % 2 == 0 || KS == K), "segments hold whole column pairs");
    constexpr int NS = K / KS;  // mask segments per lane and row
    uint8_t *__restrict__ mA = mask + pa.mask_off + (uint64_t)(lane * NS) * pa.mask_bs -
                               (int64_t)lane * (int64_t)pa.mask_rs;
    uint8_t *__restrict__ mB = mask + pb.mask_off + (uint64_t)(lane * NS) * pb.mask_bs -
                               (int64_t)lane * (int64_t)pb.mask_rs;
    const uint32_t *__restrict__ rowp = myrow - lane;  // word of row r-1 at step 0
    const uint16_t *__restrict__ rowp16 = myrow16 - lane;
    const int T = (int)geo.steps((uint32_t)ldM);
    // Walk codes: a lane whose columns all lie past a pair's query stores
    // nothing for it (no walker reads past column len_q; 16 x 10 groups on
    // 150-column queries: one store of 16 saved).  Full codes keep every
    // segment defined.
    constexpr bool kWalkCodes = kCodes == kCodesWalk || kCodes == kCodesNib;
    static_assert(kCodes != kCodesNib || KS == K, "4-bit codes: one segment per lane");
    const int ldAs = (kWalkCodes && col0 >= lqA) ? 0 : ldA;
    const int ldBs = (kWalkCodes && col0 >= lqB) ? 0 : ldB;
    // Previous-row H: step t reads Hin (row r-1) and writes Hout (row r); a
    // two-step unroll swaps two arrays (no register rotation).
    uint32_t HpB[K];

    // kSteady (steps where every lane holds a row of both pairs below their
    // last row): no per-lane activity test, no end cells, so the row result
    // is computed straight into Hout (no copies through a divergent branch)
    // Steady steps of the single-frame fill also take their row's db word
    // from the caller (read a step ahead) and the group-start inputs from
    // running packed values (the boundary column is linear inside the pair's
    // rows: sentinel-free), advanced by one row's drift per step.
    uint32_t sF = 0, sH = 0;
    const uint32_t kRowAdd = cst2(drift);
    auto step = [&](int t, uint32_t(&Hin)[K], uint32_t(&Hout)[K], auto steady_c, RowIn row_in)
                    __attribute__((always_inline)) {
        constexpr bool kSteady = decltype(steady_c)::value;
        constexpr bool kRun = kSteady && !kRebase;  // running inputs, prefetched db word
        const int r = t - lane + 1;
        uint32_t dch;
        if constexpr (kRun)
            dch = row_in.w;
        else if constexpr (kRebase)  // [A, 0, B, 0] << 5
            dch = __builtin_amdgcn_perm(0u, (uint32_t)rowp16[t], 0x0C010C00u) << 5;
        else
            dch = rowp[t];
        // kRowProf: the row's profiles (v_lshl_add: the shift takes bits 4:0)
        uint32_t prof_lo = 0, prof_hi = 0;
        if constexpr (kRowProf) {
            prof_lo = (kProfStep << (dch & 31u)) + kProfBase;
            prof_hi = (kProfStep << ((dch >> 16) & 31u)) + kProfBase;
        }
        int32_t base = 0;  // frame of step t (kRebase)
        if constexpr (kRebase) {
            base = drift * (t & -kRebaseSteps) + ctr;
            if ((t & (kRebaseSteps - 1)) == 0 && t > 0) {  // wave-uniform
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    Hin[k] += kRebaseAdd;
                    Dn[k] += kRebaseAdd;
                }
                hd += kRebaseAdd;
                pubF += kRebaseAdd;
                pubH += kRebaseAdd;
            }
        }
        // group-start inputs for row t+1: I~(r,1) and H~(r,0) (same for A and B)
        const int32_t rb = t + 1;
        uint32_t gF, gH;
        if constexpr (kRun) {
            gF = sF;
            gH = sH;
            sF += kRowAdd;
            sH += kRowAdd;
        } else {
            const int32_t bF = up(is_col1(sc, (uint32_t)rb)) + alpha * rb + beta - base;
            const int32_t bH = up(hs_col0(sc, (uint32_t)rb)) + alpha * rb - base;
            gF = pkx(bF, bF);
            gH = pkx(bH, bH);
        }
        const uint32_t inF = gshift<G>(gF, pubF, gstart);
        const uint32_t inH = gshift<G>(gH, pubH, gstart);
        if (kSteady || (r >= 1 && r <= ldM)) {
            uint32_t F = inF;
            PkMask<KS> wa[NS], wb[NS];
            // code words of column pairs: bytes [A_2c, B_2c, A_2c+1, B_2c+1]
            uint32_t cw[(K + 1) / 2];
            uint32_t prv[8];  // sign sources of the previous (even) column
            // 4-bit codes: column-group words, the group's first column pair
            // (low nibbles), the previous column's four sources
            uint32_t nw[(K + 3) / 4], nlo = 0, nprv[4];
            // kNib end-cell steps: the half (A low, B high) whose last row
            // this lane computes now takes argM in its D-open bit
            const uint32_t endsel = (t == tEA ? 0x0000FFFFu : 0u) | (t == tEB ? 0xFFFF0000u : 0u);
            // argM (bit 0) is only ever read at a pair's end cell: the wave
            // computes it on the steps where one of its lanes holds one.
            // kProf: bytes 0 / 2 select the profile byte of the A / B db char
            // (dch = A << 5 | B << 21), bytes 1 / 3 zero
            const uint32_t psel = kProf ? (((dch >> 6) & 0x00030003u) | 0x0C000C00u) : 0u;
            auto columns = [&](auto with_argm) __attribute__((always_inline)) {
            constexpr bool kM = decltype(with_argm)::value;
            uint32_t diag = hd;  // H~(r-1, c-1) of column k
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint32_t hdk = diag;
                diag = Hin[k];
                const uint32_t pen = kProf     ? __builtin_amdgcn_perm(0u, qc[k], psel)
                                     : kRowProf ? __builtin_amdgcn_perm(prof_hi, prof_lo, qc[k])
                                     : kTab     ? __builtin_amdgcn_perm(0u, kBonus, qc[k] ^ dch)
                                                : umin2(qc[k] ^ dch, kPen);
                const uint32_t M = kFree ? hdk + pen : hdk - pen;
                const uint32_t I = F, D = Dn[k];
                const uint32_t H = kFree ? hmax3(M, I, D) : umax2(M, umax2(I, D));
                const uint32_t tO = M + kOpen;
                if constexpr (kCodes == kCodesNib) {
                    // the four walk decisions as signs (set = parent absent):
                    // argI, argD (ties against the flag-free H), I-open, D-open
                    // (kS4: argI / argD signs set = present, inverted in the merge)
                    uint32_t s4[4];
                    if constexpr (kS4) {
                        const uint32_t Hm = H - 0x00020002u;
                        const uint32_t tO2 = M + (kOpen + 0x00020002u);
                        s4[0] = Hm - I;
                        s4[1] = Hm - D;
                        s4[2] = tO2 - I;
                        s4[3] = tO2 - D;
                        // argM: M - (H - 2) is >= 1 when present, <= -1 when absent
                        if constexpr (kM) s4[3] = bfi(endsel, M - Hm, s4[3]);
                    } else {
                    const uint32_t Hc = H & 0xFFFEFFFEu;
                    const uint32_t tOr = tO | 0x00010001u;
                    auto psub = [](uint32_t a, uint32_t b) { return as_u(as_s2(a) - as_s2(b)); };
                    s4[0] = psub(I, Hc);
                    s4[1] = psub(D, Hc);
                    s4[2] = psub(tOr, I);
                    s4[3] = psub(tOr, D);
                    if constexpr (kM) s4[3] = bfi(endsel, psub(M, Hc), s4[3]);
                    }
                    if (k % 2 == 0 && k < K - 1) {
#pragma unroll
                        for (int u = 0; u < 4; ++u) nprv[u] = s4[u];
                    } else {
                        // sign bytes [A_k-1, B_k-1, A_k, B_k] per source (a lone
                        // last column: [A_k, B_k, 0, 0]); a group's first column
                        // pair goes to the low nibbles, its second to the high
                        uint32_t pw[4];
#pragma unroll
                        // (a lone last column's missing neighbour: signs clear after
                        // the merge, so kS4's inverted sources get set ones here)
                        for (int u = 0; u < 4; ++u)
                            pw[u] = k % 2 ? col_pair_signs(s4[u], nprv[u])
                                          : col_pair_signs(kS4 && u < 2 ? 0x80008000u : 0u, s4[u]);
                        const int cp = k / 2, g = cp / 2;
                        // m ? a : b, or m ? ~a : ~b (kS4: argI / argD signs inverted)
                        auto bfi01 = [](uint32_t m, uint32_t a, uint32_t b) {
                            return kS4 ? __builtin_amdgcn_bitop3_b32(m, a, b, 0x35) : bfi(m, a, b);
                        };
                        if (cp % 2 == 0) {
                            uint32_t lo = bfi01(0x01010101u, pw[0], pw[1]);
                            lo = bfi(0x03030303u, lo, pw[2]);
                            lo = bfi(0x07070707u, lo, pw[3]);
                            if (cp == (K - 1) / 2) nw[g] = lo;
                            else nlo = lo;
                        } else {
                            uint32_t x = bfi01(0x10101010u, pw[0], pw[1]);
                            x = bfi(0x30303030u, x, pw[2]);
                            x = bfi(0x70707070u, x, pw[3]);
                            nw[g] = bfi(0x0F0F0F0Fu, nlo, x);
                        }
                    }
                } else if constexpr (kCodes != kCodesNone) {
                // Sign set <=> parent absent.  Same-cell differences of biased
                // halves are the unbiased differences, taken with v_pk_sub
                // (no borrow between halves); extend/open ties are decided on
                // the flag-free order: with X = 2x+f, tO = 2o+g,
                // ext <=> x >= o <=> X >= (tO & ~1),  open <=> o >= x <=> (tO | 1) >= X.
                const uint32_t Hc = H & 0xFFFEFFFEu;
                const uint32_t tOr = tO | 0x00010001u;
                auto psub = [](uint32_t a, uint32_t b) { return as_u(as_s2(a) - as_s2(b)); };
                uint32_t sg[8];
                sg[0] = kM ? psub(M, Hc) : 0u;
                sg[1] = psub(I, Hc);
                sg[2] = psub(D, Hc);
                sg[4] = psub(tOr, I);
                sg[6] = psub(tOr, D);
                // sign <=> q == d (bit 7): pen is 0 or pen_max >= 2 in both
                // halves (the low half's borrow moves the high half from
                // pen_max - 1 to pen_max - 2 or from -1 to -2)
                // (the extension-free frame's bonus: cm on a match, cmm < cm
                // otherwise, so cmm - bonus is negative exactly on a match)
                sg[7] = kFree ? psub(kCmm2, pen) : pen - 0x00010001u;
                if constexpr (kCodes == kCodesFull) {
                    const uint32_t tOc = tO & 0xFFFEFFFEu;
                    sg[3] = psub(I, tOc);
                    sg[5] = psub(D, tOc);
                } else {
                    sg[3] = sg[5] = 0u;
                }
                if (k % 2 == 0 && k < K - 1) {
#pragma unroll
                    for (int t = 0; t < 8; ++t) prv[t] = sg[t];
                } else {
                    uint32_t pw[8];
#pragma unroll
                    for (int t = 0; t < 8; ++t)
                        pw[t] = k % 2 ? col_pair_signs(sg[t], prv[t]) : col_pair_signs(0u, sg[t]);
                    cw[k / 2] = kCodes == kCodesFull ? merge_full(pw) : merge_walk<kM>(pw);
                }
                }
                F = umax2(tO, I);
                Dn[k] = kFree ? umax2(tO, D) : umax2(tO, D) + kDstep;
                Hout[k] = H;
            }
            };
            if constexpr (kWalkCodes && kSteady) {
                columns(std::false_type{});
            } else if constexpr (kWalkCodes) {
                const bool endcell = t == tEA || t == tEB;
                if (__builtin_amdgcn_ballot_w64(endcell))
                    columns(std::true_type{});
                else
                    columns(std::false_type{});
            } else {
                columns(std::true_type{});
            }
            hd = inH;
            pubF = F;
            pubH = Hout[K - 1];
            if constexpr (kCodes == kCodesNib) {
                // group words [A_c0|A_c2, B_c0|B_c2, A_c1|A_c3, B_c1|B_c3]
                // -> per-pair halves, two groups per dword; the db chars
                // (dch = A << 5 | B << 21) rotated to bytes 0 / 2
                constexpr int NG = (K + 3) / 4, ND = NG / 2 + 1;
                const uint32_t rot = kRowProf ? __builtin_amdgcn_perm(0u, kAcgt, dch >> 3)
                                     : kTab   ? __builtin_amdgcn_perm(0u, kAcgt, dch)
                                              : __builtin_amdgcn_alignbit(dch, dch, 5);
                NibSeg<K> na, nb;
#pragma unroll
                for (int d = 0; d < NG / 2; ++d) {
                    na.w[d] = __builtin_amdgcn_perm(nw[2 * d + 1], nw[2 * d], 0x06040200u);
                    nb.w[d] = __builtin_amdgcn_perm(nw[2 * d + 1], nw[2 * d], 0x07050301u);
                }
                if constexpr (NG % 2) {
                    na.w[ND - 1] = __builtin_amdgcn_perm(rot, nw[NG - 1], 0x0C040200u);
                    nb.w[ND - 1] = __builtin_amdgcn_perm(rot, nw[NG - 1], 0x0C060301u);
                } else {
                    na.w[ND - 1] = rot & 0xFFu;
                    nb.w[ND - 1] = __builtin_amdgcn_ubfe(rot, 16, 8);
                }
                if (kSteady ? ldAs != 0 : r <= ldAs) *reinterpret_cast<NibSeg<K> *>(mA) = na;
                if (kSteady ? ldBs != 0 : r <= ldBs) *reinterpret_cast<NibSeg<K> *>(mB) = nb;
            } else if constexpr (kCodes != kCodesNone) {
                // column-pair words [A A' ..] -> per-pair words of 4 columns,
                // per segment of KS columns
#pragma unroll
                for (int sg = 0; sg < NS; ++sg) {
#pragma unroll
                    for (int w = 0; w < (KS + 3) / 4; ++w) {
                        const uint32_t lo = cw[sg * KS / 2 + 2 * w];
                        const uint32_t hi = 2 * w + 1 < (KS + 1) / 2 ? cw[sg * KS / 2 + 2 * w + 1] : 0u;
                        wa[sg].w[w] = __builtin_amdgcn_perm(hi, lo, 0x06040200u);
                        wb[sg].w[w] = __builtin_amdgcn_perm(hi, lo, 0x07050301u);
                    }
                }
                // (steady: r < min(ldA, ldB), so only the lane's columns decide)
                if (kSteady ? ldAs != 0 : r <= ldAs) {
#pragma unroll
                    for (int sg = 0; sg < NS; ++sg)
                        *reinterpret_cast<PkMask<KS> *>(mA + (uint64_t)sg * pa.mask_bs) = wa[sg];
                }
                if (kSteady ? ldBs != 0 : r <= ldBs) {
#pragma unroll
                    for (int sg = 0; sg < NS; ++sg)
                        *reinterpret_cast<PkMask<KS> *>(mB + (uint64_t)sg * pb.mask_bs) = wb[sg];
                }
            }
            // (end values in the 2V + p form the walkers and results read)
            auto down = [](int32_t v) -> int32_t { return kS4 ? (v >> 2) * 2 + (v & 1) : v; };
            if (!kSteady && t == tEA) {
                const int32_t e = (int32_t)(pick_col<K>(Hout, kA) & 0xFFFFu) - kBias;
                src.end(ia, pa, down(e + base - alpha * ldA - beta * lqA));
            }
            if (!kSteady && t == tEB) {
                const int32_t e = (int32_t)(pick_col<K>(Hout, kB) >> 16) - kBias;
                src.end(ib, pb, down(e + base - alpha * ldB - beta * lqB));
            }
        } else if (&Hout != &Hin) {
#pragma unroll
            for (int k = 0; k < K; ++k) Hout[k] = Hin[k];  // lane idle: keep row r-1
        }
        mA += pa.mask_rs;
        mB += pb.mask_rs;
    };
    // steps [tS0, tS1) are steady: every lane at a row in [1, min(ldA, ldB) - 1]
    // (bounds even: the ping-pong pairs keep their parity)
    const std::false_type G0;
    const std::true_type S1;
    const int ldm = ldA < (hasB ? ldB : ldA) ? ldA : (hasB ? ldB : ldA);
    const int tS0 = min((G + 1) & ~1, T & ~1);
    const int tS1 = sc_steady ? max(tS0, tS0 + ((ldm - 1 - tS0) & ~1) * (ldm - 1 > tS0 ? 1 : 0)) : tS0;
    int t = 0;
    const RowIn z{};
    // the steady loop's row inputs, read a step ahead
    auto rowin = [&](int tt) __attribute__((always_inline)) {
        if constexpr (kRebase) return z;
        else return RowIn{rowp[tt]};
    };
    for (; t < tS0; t += 2) {
        step(t, Hp, HpB, G0, z);
        step(t + 1, HpB, Hp, G0, z);
    }
    if (tS1 > tS0) {
        if constexpr (!kRebase) {
            const int32_t rb = tS0 + 1;
            const int32_t bF = up(is_col1(sc, (uint32_t)rb)) + alpha * rb + beta;
            const int32_t bH = up(hs_col0(sc, (uint32_t)rb)) + alpha * rb;
            sF = pkx(bF, bF);
            sH = pkx(bH, bH);
        }
        RowIn d0 = rowin(t);
        for (; t < tS1; t += 2) {
            const RowIn d1 = rowin(t + 1);
            step(t, Hp, HpB, S1, d0);
            d0 = rowin(t + 2);
            step(t + 1, HpB, Hp, S1, d1);
        }
    }
    for (; t + 1 < T; t += 2) {
        step(t, Hp, HpB, G0, z);
        step(t + 1, HpB, Hp, G0, z);
    }
    if (t < T) step(t, Hp, HpB, G0, z);
    return 0;
}

template <int G, int K, int kCodes, typename Src, int KS, bool kRebase = false>
__global__ __launch_bounds__(256, (pk_min_waves<G, K, kCodes>())) void nw_fill_pk_kernel(
    Src src, uint32_t count, const uint8_t *__restrict__ qs, const uint8_t *__restrict__ ds,
    uint8_t *__restrict__ mask, Scoring sc, uint32_t ld_max, bool sc_steady) {
    fill_pk_body<G, K, kCodes, Src, KS, kRebase>(src, count, qs, ds, mask, sc, ld_max, sc_steady);
}

// 4-bit walk codes with table penalties (kTabMode 1, nw.pk_tab), and the
// launch behind it for the waves whose pairs hold a byte other than A, C, G, T
// (kTabMode 2).  A bailing wave stores the launch's epoch in its plan's bail
// word (one per mask workspace; the plan numbers its launches, and the
// launches of one workspace run in stream order); the fallback launch runs
// only when that word holds its epoch.  Two kernels, not one with both
// bodies: together they spill.
// kCodes: kCodesNib, or kCodesFull (round 6: every parent set, row profiles only)
template <int G, int K, typename Src, int kScale = 2, int kCodes = kCodesNib>
__global__ __launch_bounds__(256, (pk_min_waves<G, K, kCodes>())) void nw_fill_pk_tab_kernel(
    Src src, uint32_t count, const uint8_t *__restrict__ qs, const uint8_t *__restrict__ ds,
    uint8_t *__restrict__ mask, Scoring sc, uint32_t ld_max, uint32_t *__restrict__ bail,
    uint32_t epoch) {
    // kScale: 2 or 4 (the value scale); 3: scale 2 with row profiles (kTabMode 5)
    // (issue priority 2: between a pipelined walk's first pairs and its
    // later ones, nw_traceback_lds_kernel)
    __builtin_amdgcn_s_setprio(2);
    const int st = fill_pk_body<G, K, kCodes, Src, K, false, false,
                                kScale == 4 ? 4 : kScale == 3 ? 5 : 1>(src, count, qs, ds, mask,
                                                                       sc, ld_max, true);
    if (__builtin_amdgcn_ballot_w64(st == 1) && (threadIdx.x & 63u) == 0) *bail = epoch;
}
// (kRebaseGeneric: the fallback of a launch whose dbs need the rebasing frame;
// the extension-free table body has no drift and needs none)
// A grid-stride launch over the table launch's `vblocks` blocks (64
// workgroups instead of one per block: the launch behind every table fill
// mostly finds its word unset, and its workgroups' dispatch was its time - a
// full grid of waves that only read the word took 42 us per C2 step, 512
// workgroups 27 us; round 6).
constexpr uint32_t kTabFbBlocks = 64;
template <int G, int K, typename Src, bool kRebaseGeneric, int kCodes = kCodesNib>
__global__ __launch_bounds__(256, (pk_min_waves<G, K, kCodes>())) void nw_fill_pk_tabfb_kernel(
    Src src, uint32_t count, const uint8_t *__restrict__ qs, const uint8_t *__restrict__ ds,
    uint8_t *__restrict__ mask, Scoring sc, uint32_t ld_max, const uint32_t *__restrict__ bail,
    uint32_t epoch, uint32_t vblocks) {
    if (__builtin_amdgcn_readfirstlane(*bail) != epoch) return;
    for (uint32_t vb = blockIdx.x; vb < vblocks; vb += gridDim.x)
        fill_pk_body<G, K, kCodes, Src, K, kRebaseGeneric, false, 2>(src, count, qs, ds, mask, sc,
                                                                      ld_max, true, vb);
}

// Score-only all-vs-all of the other query classes with table penalties in
// the extension-free frame (nw.pk_tab); *generic (nw_acgt_check_kernel earlier
// on the stream) selects the xor body when a byte is not A, C, G or T.
// kRebaseGeneric: dbs too long for the original frame's single int16 window
// (the extension-free frame has no drift, so its table body needs no
// rebasing); the xor body then rebases.
template <int G, int K, bool kRebaseGeneric>
__global__ __launch_bounds__(256, (pk_min_waves<G, K, kCodesNone>())) void nw_fill_avsa_tab_kernel(
    AvsaSrc src, uint32_t count, const uint8_t *__restrict__ qs, const uint8_t *__restrict__ ds,
    Scoring sc, uint32_t ld_max, bool sc_steady, const uint32_t *__restrict__ generic) {
    if (__builtin_amdgcn_readfirstlane(*generic))
        fill_pk_body<G, K, kCodesNone, AvsaSrc, K, kRebaseGeneric, false, 0>(
            src, count, qs, ds, nullptr, sc, ld_max, sc_steady);
    else
        fill_pk_body<G, K, kCodesNone, AvsaSrc, K, false, false, 1>(src, count, qs, ds, nullptr, sc,
                                                                    ld_max, sc_steady);
}

// Score-only all-vs-all with query profiles; *generic (set by
// nw_acgt_check_kernel earlier on the stream) selects the xor path when a
// sequence byte is not one of A, C, G, T.
// kFree: profiles of bonuses in the extension-free frame (nw.pk_tab, pk_tab_ok).
template <int G, int K, bool kFree>
__global__ __launch_bounds__(256) void nw_fill_avsa_prof_kernel(
    AvsaSrcP src, uint32_t count, const uint8_t *__restrict__ qs, const uint8_t *__restrict__ ds,
    Scoring sc, uint32_t ld_max, bool sc_steady, const uint32_t *__restrict__ generic) {
    if (__builtin_amdgcn_readfirstlane(*generic))
        fill_pk_body<G, K, kCodesNone, AvsaSrcP, K, false, false>(src, count, qs, ds, nullptr, sc,
                                                                  ld_max, sc_steady);
    else
        fill_pk_body<G, K, kCodesNone, AvsaSrcP, K, false, true, kFree ? 3 : 0>(
            src, count, qs, ds, nullptr, sc, ld_max, sc_steady);
}

// flag |= 1 when a byte of seq[0, n) is not A, C, G or T
__global__ __launch_bounds__(256) void nw_acgt_check_kernel(const uint8_t *__restrict__ seq,
                                                            uint64_t n, uint32_t *__restrict__ flag) {
    bool bad = false;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint8_t c = seq[i];
        bad |= c != 'A' && c != 'C' && c != 'G' && c != 'T';
    }
    if (__builtin_amdgcn_ballot_w64(bad) && (threadIdx.x & 63u) == 0) atomicOr(flag, 1u);
}

// Column-stripe fill (declared with the stripe protocol above), i32 lanes.
// Representation: X~(r,c) = X'(r,c) + alpha*r + beta*c as in the packed
// fill (beta = -2*gap_extend, alpha = -2*match - beta): M~ = H~(r-1,c-1) -
// pen*[q != d], I~(r,c+1) = max(M~ + 2*gap_open, I~), D~(r+1,c) = max(M~ +
// 2*gap_open, D~) + 2*gap_extend + alpha.  i32 carries the reference's
// literal -32768 sentinel exactly (the boundary functions apply it; the
// offsets are linear, so no value is clamped anywhere).
// Parent codes from sign bits of same-cell differences (sign set <=> parent
// absent, flag-free comparisons as in the packed fill); per source, two
// v_perm gather the bit-31 signs of the four columns into 0x00/0xFF bytes and
// a v_bfi chain merges the sources.
// kArgM = false (walk codes of rows that hold no end cell): bit 0 (argM,
// read only at the end cell) is not gathered; merge_walk copies bit 1 there.
// kEq = false (walk codes of the row fill): no eq bit (bit 7), the
// cooperative walker compares the sequence bytes instead.
template <int kCodes, bool kArgM, bool kEq = true>
__device__ __forceinline__ uint32_t stripe_code_word(const uint32_t (&s)[8][4]) {
    uint32_t w[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        if ((t == 0 && kCodes != kCodesFull && !kArgM) || (t == 7 && kCodes != kCodesFull && !kEq) ||
            ((t == 3 || t == 5) && kCodes != kCodesFull)) {
            w[t] = 0u;
            continue;
        }
        w[t] = __builtin_amdgcn_perm(s[t][1], s[t][0], 0x0C0C0B09u) |
               __builtin_amdgcn_perm(s[t][3], s[t][2], 0x0B090C0Cu);
    }
    if constexpr (kCodes == kCodesFull) return merge_full(w);
    if constexpr (!kEq) {  // merge_walk without its last (eq) step
        uint32_t r = kArgM ? bfi(0x01010101u, w[0], w[1]) : w[1];
        r = bfi(0x03030303u, r, w[2]);
        r = bfi(0x07070707u, r, w[4]);
        return bfi(0x1F1F1F1Fu, r, w[6]);
    }
    return merge_walk<kArgM>(w);
}
template <int kCodes>
__device__ __forceinline__ uint32_t stripe_code_word(const uint32_t (&s)[8][4]) {
    return stripe_code_word<kCodes, true>(s);
}

// ------------------------------------- long pairs: row-synchronous stripes
// One wave per stripe of 64*K columns (K = 1, 2, 4), all 64 lanes on the same
// row at the same step.  A stripe then has no internal skew: its right
// neighbour starts row r as soon as row r's boundary arrives (lag = one
// hand-off, not the 64 + 32 steps of nw_fill_stripe_kernel), so stripes can
// be narrow and many (C4: 1,563 waves of 64 columns instead of 391 of 256).
// Within a row, M~ = H~(r-1, c-1) - pen and D~ come from the previous row;
// in the transformed recurrence (nw_fill_stripe_kernel) I~(r, c+1) =
// max(I~(r, c), M~(r, c) + open) is the row's running max of the gap-open
// candidates: a lane-local prefix over its K columns, a 64-lane DPP prefix max
// of the lane totals (row_shr 1/2/4/8, row_bcast 15/31) and the I entering
// from the left stripe.  i32 with V'' = 4V + 2a + p (nw_common.hpp).
// Mask layout: 256-column tiles, row-major inside a tile (bs = 4, rs = 256):
// cell (i, j) at (j-1)/256 * cs + (i-1) * 256 + (j-1) % 256, so a stripe's
// row is 64K contiguous bytes.  Codes are built four cells at a time
// (stripe_code_word): K = 4 one row, K = 2 two rows, K = 1 four rows.
// Hand-off: the stripe's last lane stores (H~, I~) leaving its last column
// per row as one 64-bit agent-coherent store into boundary column g (preset
// to kColEmpty); stripe g+1 polls kRowsBlk-row blocks (nw_fill_stripe_kernel).
constexpr int32_t kNegInf = INT32_MIN;
constexpr uint32_t kRowsOff = 0;  // boundary row r at element r of the column
constexpr uint32_t kRowsGrp = 8;  // rows per boundary group (4: slower, rounds 2 and 4)

// inclusive prefix max over the wave's 64 lanes (lane order).  `fill`:
// independent work placed inside the chain, where each dependent DPP step
// would otherwise wait two issue slots (s_nop)
template <class Fill>
__device__ __forceinline__ int32_t wave_prefix_max(int32_t v, Fill &&fill) {
    v = max(v, __builtin_amdgcn_update_dpp(kNegInf, v, 0x111 /*row_shr:1*/, 0xf, 0xf, false));
    fill();
    v = max(v, __builtin_amdgcn_update_dpp(kNegInf, v, 0x112 /*row_shr:2*/, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(kNegInf, v, 0x114 /*row_shr:4*/, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(kNegInf, v, 0x118 /*row_shr:8*/, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(kNegInf, v, 0x142 /*row_bcast:15*/, 0xa, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(kNegInf, v, 0x143 /*row_bcast:31*/, 0xc, 0xf, false));
    return v;
}

// One-wave workgroups, one stripe each (n_waves of them; round 4: four-wave
// groups ran C4 in 21.2 ms against 14.2).  Placement (kPlace):
// 0  wave v = workgroup v; the dispatcher may stack stripes on a SIMD.
// 1  (kPlaceLone) every wave reserves the whole register file of its SIMD (an
//    AGPR clobber puts the allocation past 256 VGPR+AGPR per lane: one wave
//    per SIMD, MI355X_MICROARCH.md's occupancy table), so no two stripes
//    share a SIMD.  The dispatcher otherwise stacks them: 196 one-wave groups
//    on a 64-CU mask landed on 128 SIMDs (tools/cu_occupancy.py), and a stripe
//    that shares its SIMD slows the whole row chain (a span of the 4-span
//    chain alone: 19.8 ms against 12.1 for the 8-span one's).  Used when the
//    launch's stripes fit the SIMDs; waves past them wait for a SIMD, and
//    since workgroups dispatch in order the resident stripes are always the
//    leftmost unfinished ones.
// 2  (kPlaceXcd) lone, and XCD-local neighbours: workgroups are dispatched
//    round-robin over the 8 XCDs (workgroup b -> XCD b % 8), so wave v =
//    (b % 8) * xcd_run + b / 8 puts runs of xcd_run consecutive stripes on
//    one XCD and only 7 hand-offs cross XCDs.  Valid only when every stripe of
//    the launch is resident at once (a stripe's left neighbour may have a
//    later workgroup id): the host takes it when every XCD's SIMDs (of the
//    stream's CU mask) hold its run (xcd_fit).  A stripe whose consumer runs
//    on its own XCD publishes with plain stores, which keep the line in the
//    XCD's L2 where the consumer's sc1 load finds it (the hand-off rules in
//    DESIGN.md §3); every other stripe publishes sc1 (write-through, visible
//    to any XCD).  "Its own XCD" is checked, not assumed (HIP promises no
//    workgroup-to-XCD placement; the b % 8 round-robin is observed,
//    MI355X_MICROARCH.md "Workgroup dispatch"): each wave posts {epoch, its
//    XCC_ID} in its slot of the launch's err buffer with an sc1 store, and a
//    producer reads its consumer's slot with sc1 loads before the row loop;
//    anything but a match within the bound publishes sc1.
constexpr int kPlaceShared = 0, kPlaceLone = 1, kPlaceXcd = 2;
template <int K, int kCodes, bool kMinPen, int kPlace>
__global__ __launch_bounds__(64) void nw_fill_rows_kernel(
    const NwPairDesc *__restrict__ pairs, const uint2 *__restrict__ work,
    const uint8_t *__restrict__ qs, const uint8_t *__restrict__ ds, uint8_t *__restrict__ mask,
    int2 *__restrict__ scratch, uint32_t *__restrict__ err, int32_t *__restrict__ end_h,
    Scoring sc, uint32_t n_waves, uint32_t xcd_run, uint32_t epoch) {
    static_assert(K == 1 || K == 2, "4 cells per code word (K = 4, 256-column stripes: slower, round 2)");
    constexpr int S = 4 / K;   // stripes per 256-column chunk (work item)
    constexpr int W = 64 * K;  // stripe width (4 / K rows per code word)
    if constexpr (kPlace != kPlaceShared) asm volatile("" : : : "a255");
    const int lane = (int)(threadIdx.x & 63u);
    // (readfirstlane: the slot is wave-uniform, so everything derived from it
    // stays in SGPRs: the publication base is an asm "s" operand)
    const uint32_t v = __builtin_amdgcn_readfirstlane(
        kPlace == kPlaceXcd ? (blockIdx.x & 7u) * xcd_run + (blockIdx.x >> 3) : blockIdx.x);
    if (v >= n_waves) return;  // (whole wave: no group barrier in this kernel)
    // plain publication: my consumer (stripe v + 1, when it is one) runs on my
    // XCD, seen in its slot (err[2 + v + 1]: {epoch, XCC_ID}, posted by its
    // lane 0 at its start; a stale epoch or a bounded wait that expires: sc1).
    // The launch's last stripe publishes sc1: a span's outbox is read by a
    // relay kernel, a copy or RCCL, none of them in this XCD's L2.
    bool plain_pub = false;
    if constexpr (kPlace == kPlaceXcd) {
        uint32_t *const slots = err + 2;
        const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 15u;  // HW_REG_XCC_ID
        const uint32_t me = (epoch << 4) | xcc;
        if (lane == 0) asm volatile("global_store_dword %0, %1, off sc1" : : "v"(slots + v), "v"(me) : "memory");
        if ((v + 1) % xcd_run != 0 && v + 1 < n_waves) {
            uint32_t got = 0;
            for (uint32_t k = 0; k < 4096u; ++k) {  // (the consumer is resident: microseconds)
                asm volatile("global_load_dword %0, %1, off sc1\n\ts_waitcnt vmcnt(0)"
                             : "=v"(got) : "v"(slots + v + 1) : "memory");
                if ((got >> 4) == ((epoch << 4) >> 4)) break;
                __builtin_amdgcn_s_sleep(2);
            }
            plain_pub = __builtin_amdgcn_readfirstlane(got) == me;
        }
    }
    const uint2 wk = work[v / S];
    const NwPairDesc p = pairs[wk.x];
    const uint32_t g = wk.y * S + v % S;  // stripe index
    const uint32_t lq = p.len_q, ld = p.len_db;
    const uint32_t c0 = g * W;  // the stripe's columns c0+1 .. c0+W
    if (c0 >= lq) return;
    const uint32_t nst = (lq + W - 1) / W;
    const int2 *__restrict__ scr_in = g > 0 ? scratch + p.scratch_off + (uint64_t)(g - 1) * scratch_col(ld) : nullptr;
    // (the last stripe too, into a column nobody reads: a fixed VMEM count per group)
    int2 *__restrict__ scr_out = scratch + p.scratch_off + (uint64_t)g * scratch_col(ld);
    (void)nst;
    const int32_t beta = -4 * sc.gap_extend;
    const int32_t alpha = -4 * sc.match - beta;
    const int32_t pen_max = 4 * (sc.match - sc.mismatch);
    const int32_t kOpen = 4 * sc.gap_open;
    const int32_t kDstep = 4 * sc.gap_extend + alpha;
    constexpr int32_t kTieOr = kCodes == kCodesFull ? 3 : 1;
    const uint32_t col0 = c0 + (uint32_t)lane * K;  // my columns col0+1 .. col0+K
    uint32_t qc[K];
    int32_t Hp[K], Dn[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t j = col0 + k + 1;
        qc[k] = j <= lq ? (uint32_t)qs[p.q_off + j - 1] << 8 : 0xFFFFFF00u;
        Hp[k] = hs4_row0(sc, j) + beta * (int32_t)j;
        Dn[k] = ds4_row1(sc, j) + alpha + beta * (int32_t)j;
    }
    int32_t hb_prev = hs4_row0(sc, c0) + beta * (int32_t)c0;  // H~(r-1, c0): lane 0's diagonal
    // stripes with a left neighbour: the loaded boundary rows stay in lanes
    // 0..7 (cH_v, the previous group's in cH_prev_v); row q of a group takes
    // H~(r-1, c0) from lane q-1 with one DPP row_shl instead of a readlane
    int32_t cH_v = hb_prev, cH_prev_v = hb_prev;
    // my bytes of row 1 in the 256-column tile layout
    uint8_t *mrow = mask + p.mask_off + (uint64_t)(c0 / 256) * p.mask_cs + (col0 % 256);
    typedef const __attribute__((address_space(4))) uint32_t cu32;  // constant: scalar loads
    const uint8_t *d = ds + p.db_off;
    cu32 *dw = (cu32 *)((uintptr_t)d & ~(uintptr_t)3);
    const uint32_t doff = 8u * (uint32_t)((uintptr_t)d & 3);
    const uint32_t last_dw = ((uint32_t)ld - 1 + (uint32_t)((uintptr_t)d & 3)) >> 2;
    uint32_t dnidx = min(1u, last_dw);
    uint32_t dcur = dw[0], dnxt = dw[dnidx];

    bool failed = false;
    // SALN_ROWS_BCAST 2: the group's publication base (row r0) and my offset
    // from it: 0 for lane 63, the pad slots ld + 1 .. ld + 8 for the others
    const int2 *pub_base = scr_out;
    uint32_t pub_voff = 0;
    const uint32_t jend = lq - 1;
    const bool end_lane = jend / W == g && (uint32_t)lane == (jend % W) / K;
    const uint32_t k_end = jend % K;
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the query chars
    uint32_t sg[8][4];  // sign words of the current code word's four cells
    constexpr bool kCodesHere = kCodes != kCodesNone;
    // one row: r (1-based), its db char, the left boundary (H~(r, c0), I~
    // entering column c0+1) and u = its slot in the code word (compile time)
    // m: the row may be the last one (argM bits and the reference's tie
    // sets for the end states); every other row stores walk codes without
    // argM, tied against H'' & ~1 with no per-row test
    auto row = [&](uint32_t r, uint32_t dch, int32_t bH, int32_t bI, auto u_c, auto q_c,
                   auto m_c, auto &&fill, auto vb_c, auto plain_c) __attribute__((always_inline)) {
        constexpr int u = decltype(u_c)::value;
        constexpr int q = decltype(q_c)::value;  // row in its boundary group
        constexpr bool kM = decltype(m_c)::value;
        const int32_t hm = (kCodes == kCodesFull || (kM && r == ld)) ? ~3 : ~1;
        int32_t M[K], tO[K], P[K], Dv[K];
        uint32_t s6[K];  // D-open signs (sg[6] is written after the chain: the
                         // chain's filler may still read the previous rows' sg)
        int32_t hbv;  // lane 0: H~(r-1, c0)
        if constexpr (decltype(vb_c)::value) {
            if constexpr (q == 0)
                hbv = __builtin_amdgcn_update_dpp(0, cH_prev_v, 0x107 /*row_shl:7*/, 0xf, 0xf, true);
            else if constexpr (q == 1)
                hbv = cH_v;
            else
                hbv = __builtin_amdgcn_update_dpp(0, cH_v, 0x100 + (q - 1) /*row_shl*/, 0xf, 0xf, true);
        } else {
            hbv = hb_prev;
        }
        int32_t diag = __builtin_amdgcn_update_dpp(hbv, Hp[K - 1], 0x138 /*wave_shr:1*/, 0xf, 0xf, false);
        uint32_t x[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            x[k] = qc[k] ^ dch;
            const int32_t pen = kMinPen ? (int32_t)min(x[k], (uint32_t)pen_max) : (x[k] ? pen_max : 0);
            M[k] = (k == 0 ? diag : Hp[k - 1]) - pen;
            tO[k] = M[k] + kOpen;
            P[k] = k == 0 ? tO[0] : max(P[k - 1], tO[k]);
            // what does not need the row's I: the D step and its open sign
            // (independent of the prefix chain below, so they can fill its slots)
            Dv[k] = Dn[k];
            s6[k] = (uint32_t)((tO[k] | kTieOr) - Dv[k]);
            Dn[k] = max(tO[k], Dv[k]) + kDstep;
        }
        const int32_t S_incl = wave_prefix_max(P[K - 1], fill);
        const int32_t Ein = max(__builtin_amdgcn_update_dpp(kNegInf, S_incl, 0x138, 0xf, 0xf, false), bI);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int32_t I = k == 0 ? Ein : max(Ein, P[k - 1]);
            const int32_t D = Dv[k];
            const int32_t H = max(M[k], max(I, D));
            if constexpr (kCodesHere) {
                const int32_t Hc = H & hm;
                const int32_t tOr = tO[k] | kTieOr;
                const int e = u * K + k;  // cell slot in the code word (unrolled: constant)
                sg[0][e] = (kCodes == kCodesFull || kM) ? (uint32_t)(M[k] - Hc) : 0u;
                sg[1][e] = (uint32_t)(I - Hc);
                sg[2][e] = (uint32_t)(D - Hc);
                sg[4][e] = (uint32_t)(tOr - I);
                sg[6][e] = s6[k];
                sg[7][e] = kCodes == kCodesFull ? x[k] - 1u : 0u;  // sign <=> q == d (full codes)
                if constexpr (kCodes == kCodesFull) {
                    const int32_t tOc = tO[k] & ~3;
                    sg[3][e] = (uint32_t)(I - tOc);
                    sg[5][e] = (uint32_t)(D - tOc);
                } else {
                    sg[3][e] = sg[5][e] = 0u;
                }
            }
            Hp[k] = H;
        }
        hb_prev = bH;
        // (H~, I~) leaving the stripe's last column (lane 63's values)
        {   // every lane stores its own (H~, I~) with one instruction: lane 63
            // at row r of the column, the others at a pad slot past the db
            // (pub_voff, set per group); no readlane, no exec change, the
            // row's address an immediate offset from the group's base
            const int32_t iv = max(S_incl, bI);
            const uint64_t val = (uint64_t)(uint32_t)Hp[K - 1] | ((uint64_t)(uint32_t)iv << 32);
            const uint32_t vo = pub_voff;  // (asm operands take locals, not captures)
            const int2 *pb = pub_base;
            // (a 64-bit store has no data hazard with the VALU around it)
            if constexpr (decltype(plain_c)::value)
                asm volatile("global_store_dwordx2 %0, %1, %2 offset:%3"
                             : : "v"(vo), "v"(val), "s"(pb), "i"(8 * q) : "memory");
            else
                asm volatile("global_store_dwordx2 %0, %1, %2 offset:%3 sc1"
                             : : "v"(vo), "v"(val), "s"(pb), "i"(8 * q) : "memory");
        }
    };
    // store the code word of rows r0 .. r0+(4/K)-1 (n of them valid)
    auto put = [&](uint32_t r0, uint32_t n, auto m_c) __attribute__((always_inline)) {
        if constexpr (kCodesHere) {
            const uint32_t wv = stripe_code_word<kCodes, decltype(m_c)::value, false>(sg);
            uint8_t *a = mrow + (uint64_t)(r0 - 1) * 256;
            if constexpr (K == 2) {
                *reinterpret_cast<uint16_t *>(a) = (uint16_t)wv;
                if (n > 1) *reinterpret_cast<uint16_t *>(a + 256) = (uint16_t)(wv >> 16);
            } else {
                a[0] = (uint8_t)wv;
                if (n > 1) a[256] = (uint8_t)(wv >> 8);
                if (n > 2) a[512] = (uint8_t)(wv >> 16);
                if (n > 3) a[768] = (uint8_t)(wv >> 24);
            }
        }
    };
    auto nofill = []() __attribute__((always_inline)) {};
    const std::integral_constant<int, 0> u0;
    const std::integral_constant<int, 1> u1;
    const std::integral_constant<int, 2> u2;
    const std::integral_constant<int, 3> u3;
    // The left boundary arrives per four-row group: when a group starts,
    // lanes 0-3 load the next group's four rows (agent-coherent sc1 loads,
    // issued as inline asm so that the compiler adds no wait of its own: its
    // wait would be a vmcnt(0) on every outstanding store); the next group
    // waits for exactly that load with a counted vmcnt: a group issues eight
    // VMEM operations after it (four mask stores, four boundary stores: every
    // stripe publishes, the last one into a column nobody reads; score-only:
    // the four boundary stores), so vmcnt(7) (3) covers it.  The count must
    // be exact - a load still in flight after its wait would land in
    // registers the compiler has reused.  Rows not yet published are
    // re-polled with ordinary (compiler-waited) loads.
    auto rows = [&](auto F, auto PL) __attribute__((always_inline)) {
        constexpr bool kFirst = decltype(F)::value;
        const std::integral_constant<bool, !kFirst> VB;  // boundary rows kept in cH_v
        constexpr uint32_t kG = kRowsGrp;  // rows per boundary group
        uint64_t nv = 0;  // lanes 0..kG-1: (H~, I~) of the next group's rows
        // only the group's own rows.  (A round-2 branch-free variant in which
        // every lane loaded a clamped row gave wrong boundary values in
        // batches.  Cause, from the ISA (tools/isa_check.py): the last
        // group's prefetch - dead here, no lane passes the guard - became a
        // live load of row ld, still in flight when the compiler reused its
        // destination VGPRs for the last group's rows; it landed over them.
        // The last group now issues no prefetch.)
        auto fetch = [&](uint32_t r0) __attribute__((always_inline)) {
            if (!kFirst && lane < (int)kG && r0 + (uint32_t)lane <= ld)
                asm volatile("global_load_dwordx2 %0, %1, off sc1"
                             : "=v"(nv) : "v"(scr_in + r0 + kRowsOff + lane) : "memory");
        };
        fetch(1);
        if constexpr (!kFirst) asm volatile("s_waitcnt vmcnt(0)" : "+v"(nv) : : "memory");
        int32_t bh[kG], bi[kG];  // the boundary of rows r .. r+kG-1
        // kNext: prefetch the next group's rows.  The last group issues no
        // prefetch at all: an asm load still in flight when its registers are
        // reused corrupts whatever the compiler put there (the
        // hand-off rules; tests/test_isa_handoff.py checks the ISA)
        auto group = [&](uint32_t r, auto next_c) __attribute__((always_inline)) {
            constexpr bool kNext = decltype(next_c)::value;
            pub_base = scr_out + r;
            pub_voff = lane == 63 ? 0u : (ld + 1u - r) * 8u;
            if constexpr (kFirst) {
#pragma unroll
                for (uint32_t q = 0; q < kG; ++q) {
                    bi[q] = is4_col1(sc, r + q) + alpha * (int32_t)(r + q) + beta;
                    bh[q] = hs4_col0(sc, r + q) + alpha * (int32_t)(r + q);
                }
            } else {
                // kG mask stores and kG boundary stores followed the prefetch:
                // with that many younger VMEM ops outstanding it has landed
                // (GFX9 vmcnt retires in issue order)
                if constexpr (kCodes == kCodesNone) {  // no mask stores
                    if constexpr (kG == 8) asm volatile("s_waitcnt vmcnt(8)" : "+v"(nv) : : "memory");
                    else asm volatile("s_waitcnt vmcnt(4)" : "+v"(nv) : : "memory");
                } else {
                    if constexpr (kG == 8) asm volatile("s_waitcnt vmcnt(16)" : "+v"(nv) : : "memory");
                    else asm volatile("s_waitcnt vmcnt(8)" : "+v"(nv) : : "memory");
                }
                int32_t cH = (int32_t)(uint32_t)nv, cI = (int32_t)(uint32_t)(nv >> 32);
                const bool mine = lane < (int)kG && r + (uint32_t)lane <= ld;
                bool ok = !mine || (uint32_t)cH != kColEmpty;
                if (__builtin_expect(__builtin_amdgcn_ballot_w64(!ok) != 0, 0) && !failed) {
                    uint32_t spins = 0;  // not yet published: poll (rare)
                    do {
                        __builtin_amdgcn_s_sleep(1);
                        if (mine) {
                            const uint64_t v = __hip_atomic_load((const uint64_t *)(scr_in + r + kRowsOff + lane),
                                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            cH = (int32_t)(uint32_t)v;
                            cI = (int32_t)(uint32_t)(v >> 32);
                            ok = (uint32_t)cH != kColEmpty;
                        }
                        if (++spins > err[1]) failed = true;
                    } while (__builtin_amdgcn_ballot_w64(!ok) && !failed);
                }
                if constexpr (kNext) fetch(r + kG);
                cH_prev_v = cH_v;
                cH_v = cH;
#pragma unroll
                for (uint32_t q = 0; q < kG; ++q) {
                    bh[q] = 0;  // (rows take H~ from cH_v)
                    bi[q] = __builtin_amdgcn_readlane(cI, q);
                }
            }
        };
        // four rows r .. r+3 of a group (their boundary at bh/bi[o .. o+3])
        // K = 2: fill0 runs inside row r's prefix chain (the previous quad's
        // last code word); kFlush = false leaves rows r+2, r+3's code word to
        // the caller (the next quad's fill0)
        auto quad = [&](uint32_t r, auto o_c, auto m_c, auto &&fill0, auto flush_c)
                        __attribute__((always_inline)) {
            constexpr int o = decltype(o_c)::value;
            constexpr bool kFlush = decltype(flush_c)::value;
            const std::integral_constant<int, o> q0;  // rows of the boundary group
            const std::integral_constant<int, o + 1> q1;
            const std::integral_constant<int, o + 2> q2;
            const std::integral_constant<int, o + 3> q3;
            const uint32_t w = doff ? (dcur >> doff) | (dnxt << (32u - doff)) : dcur;
            dcur = dnxt;
            dnidx = min(dnidx + 1, last_dw);
            dnxt = dw[dnidx];
            if constexpr (K == 2) {
                // rows r, r+1's code word is built inside row r+2's prefix chain
                row(r, (w & 0xFFu) << 8, bh[o], bi[o], u0, q0, m_c, fill0, VB, PL);
                row(r + 1, ((w >> 8) & 0xFFu) << 8, bh[o + 1], bi[o + 1], u1, q1, m_c, nofill, VB, PL);
                row(r + 2, ((w >> 16) & 0xFFu) << 8, bh[o + 2], bi[o + 2], u0, q2, m_c,
                    [&]() __attribute__((always_inline)) { put(r, 2, m_c); }, VB, PL);
                row(r + 3, (w >> 24) << 8, bh[o + 3], bi[o + 3], u1, q3, m_c, nofill, VB, PL);
                if constexpr (kFlush) put(r + 2, 2, m_c);
            } else {
                row(r, (w & 0xFFu) << 8, bh[o], bi[o], u0, q0, m_c, fill0, VB, PL);
                row(r + 1, ((w >> 8) & 0xFFu) << 8, bh[o + 1], bi[o + 1], u1, q1, m_c, nofill, VB, PL);
                row(r + 2, ((w >> 16) & 0xFFu) << 8, bh[o + 2], bi[o + 2], u2, q2, m_c, nofill, VB, PL);
                row(r + 3, (w >> 24) << 8, bh[o + 3], bi[o + 3], u3, q3, m_c, nofill, VB, PL);
                if constexpr (kFlush) put(r, 4, m_c);
            }
        };
        // the last 1-3 rows (boundary at bh/bi[o ..])
        auto tail = [&](uint32_t r, auto o_c, auto m_c) __attribute__((always_inline)) {
            constexpr int o = decltype(o_c)::value;
            const std::integral_constant<int, o> q0;
            const std::integral_constant<int, o + 1> q1;
            const std::integral_constant<int, o + 2> q2;
            const uint32_t w = doff ? (dcur >> doff) | (dnxt << (32u - doff)) : dcur;
            const uint32_t n = ld - r + 1;
            if constexpr (K == 2) {
                row(r, (w & 0xFFu) << 8, bh[o], bi[o], u0, q0, m_c, nofill, VB, PL);
                if (n > 1) row(r + 1, ((w >> 8) & 0xFFu) << 8, bh[o + 1], bi[o + 1], u1, q1, m_c, nofill, VB, PL);
                put(r, min(n, 2u), m_c);
                if (n > 2) { row(r + 2, ((w >> 16) & 0xFFu) << 8, bh[o + 2], bi[o + 2], u0, q2, m_c, nofill, VB, PL); put(r + 2, 1, m_c); }
            } else {
                row(r, (w & 0xFFu) << 8, bh[o], bi[o], u0, q0, m_c, nofill, VB, PL);
                if (n > 1) row(r + 1, ((w >> 8) & 0xFFu) << 8, bh[o + 1], bi[o + 1], u1, q1, m_c, nofill, VB, PL);
                if (n > 2) row(r + 2, ((w >> 16) & 0xFFu) << 8, bh[o + 2], bi[o + 2], u2, q2, m_c, nofill, VB, PL);
                put(r, n, m_c);
            }
        };
        const std::integral_constant<int, 0> o0;
        const std::integral_constant<int, 4> o4;
        const std::false_type M0;  // rows that cannot be the last one
        const std::true_type M1;   // the last group (holds row ld)
        static_assert(kG == 4 || kG == 8, "four or eight rows per boundary group");
        uint32_t r = 1;
        for (; r + kG - 1 < ld; r += kG) {  // full groups before the one holding row ld
            group(r, std::true_type{});
            if constexpr (kG == 8 && K <= 2) {
                // the first quad's last code word goes into row r+4's prefix chain
                quad(r, o0, M0, nofill, std::false_type{});
                quad(r + 4, o4, M0,
                     [&]() __attribute__((always_inline)) {
                         if constexpr (K == 2) put(r + 2, 2, M0);
                         else put(r, 4, M0);
                     },
                     std::true_type{});
            } else {
                quad(r, o0, M0, nofill, std::true_type{});
                if constexpr (kG == 8) quad(r + 4, o4, M0, nofill, std::true_type{});
            }
        }
        // the last group: 1 .. kG rows, row ld among them
        group(r, std::false_type{});
        const uint32_t nq = (ld - r + 1) / 4;  // full quads
        const bool t = (ld - r + 1) % 4 != 0;
        if (nq == 0) {
            tail(r, o0, M1);
        } else if constexpr (kG == 8) {
            if (nq == 1) {
                quad(r, o0, M1, nofill, std::true_type{});
                if (t) tail(r + 4, o4, M1);
            } else {
                quad(r, o0, M1, nofill, std::true_type{});
                quad(r + 4, o4, M1, nofill, std::true_type{});
            }
        } else {
            quad(r, o0, M1, nofill, std::true_type{});
        }
    };
    if constexpr (kPlace == kPlaceXcd) {
        if (plain_pub) {
            if (g == 0) rows(std::true_type{}, std::true_type{});
            else rows(std::false_type{}, std::true_type{});
        } else {
            if (g == 0) rows(std::true_type{}, std::false_type{});
            else rows(std::false_type{}, std::false_type{});
        }
    } else {
        if (g == 0) rows(std::true_type{}, std::false_type{});
        else rows(std::false_type{}, std::false_type{});
    }
    if (end_lane) {
        int32_t e = 0;
#pragma unroll
        for (int k = 0; k < K; ++k)
            if ((uint32_t)k == k_end) e = Hp[k];
        end_h[wk.x] = x4_to_x2(e - alpha * (int32_t)ld - beta * (int32_t)lq);
    }
    if (failed && lane == 0) atomicOr(err, 1u);
}

// ------------------------------------------------------------ i32 lanes
// Pairs the packed fills cannot hold (long dbs, wide penalties): one pair per
// group of G lanes, K columns per lane, i32 with the transformed recurrence
// and sign-bit parent codes of the stripe fill (X~ = X' + alpha*r + beta*c;
// the literal -32768 sentinel stays exact since the offsets are linear).
// kStaged: the group's db row is staged in LDS (bytes, padded by G on both
// sides) and a previous chunk's boundary column is read in G-row blocks with
// the wait on the block step only: otherwise every step waits (vmcnt) for its
// own char / boundary load and with it for every mask store.
template <int G, int K, int kCodes, bool kMinPen, bool kStaged>
__global__ __launch_bounds__(256) void nw_fill_lanes_kernel(
    const NwPairDesc *__restrict__ pairs, uint32_t first, uint32_t count,
    const uint8_t *__restrict__ qs, const uint8_t *__restrict__ ds, uint8_t *__restrict__ mask,
    int2 *__restrict__ scratch, int32_t *__restrict__ end_h, Scoring sc, uint32_t ld_max) {
    constexpr int GPB = 256 / G;
    constexpr int KD = (K + 3) / 4;
    constexpr Geom geo{G, K};
    const int lane = threadIdx.x % G;
    const uint32_t gi = pack_block(blocks_per_pack(GPB)) * GPB + threadIdx.x / G;
    if (gi >= count) return;  // whole group (DPP never crosses groups)
    const NwPairDesc p = pairs[first + gi];
    const uint32_t lq = p.len_q, ld = p.len_db;
    const uint8_t *__restrict__ q = qs + p.q_off;
    const uint8_t *__restrict__ d = ds + p.db_off;
    uint8_t *__restrict__ mk = mask + p.mask_off;
    int2 *__restrict__ scr = scratch + p.scratch_off;
    const uint32_t nch = geo.n_chunks(lq);
    // V'' = 4V + 2a + p (nw_common.hpp); tie masks as in the stripe fill
    const int32_t beta = -4 * sc.gap_extend;
    const int32_t alpha = -4 * sc.match - beta;
    const int32_t pen_max = 4 * (sc.match - sc.mismatch);
    const int32_t kOpen = 4 * sc.gap_open;
    const int32_t kDstep = 4 * sc.gap_extend + alpha;
    constexpr int32_t kTieOr = kCodes == kCodesFull ? 3 : 1;
    const uint32_t jend = lq - 1;
    const uint32_t c_end = jend / geo.W(), l_end = (jend % geo.W()) / K, k_end = jend % K;
    extern __shared__ uint8_t drow8[];  // kStaged: [GPB][G + ld_max + G] db chars
    const uint8_t *myrow = drow8 + (threadIdx.x / G) * (ld_max + 2 * G) + G;
    if constexpr (kStaged) {
        uint8_t *row = drow8 + (threadIdx.x / G) * (ld_max + 2 * G) + G;
        for (int i = lane; i < (int)ld; i += G) row[i] = d[i];
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        __builtin_amdgcn_wave_barrier();
    }
    const int bsrc = (int)((threadIdx.x & 63u) & ~(uint32_t)(G - 1));  // my group's lane 0 in the wave

    for (uint32_t c = 0; c < nch; ++c) {
        const uint32_t col0 = c * geo.W() + (uint32_t)lane * K;  // my columns: col0+1 .. col0+K
        uint32_t qc[K];
        int32_t Hp[K], Dn[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t j = col0 + k + 1;
            qc[k] = j <= lq ? (uint32_t)q[j - 1] << 8 : 0xFFFFFF00u;
            Hp[k] = hs4_row0(sc, j) + beta * (int32_t)j;
            Dn[k] = ds4_row1(sc, j) + alpha + beta * (int32_t)j;
        }
        int32_t hd = hs4_row0(sc, col0) + beta * (int32_t)col0;
        int32_t pubF = 0, pubH = 0;
        int32_t dnext = (!kStaged && lane == 0) ? (int32_t)d[0] : 0;
        int2 bnext = make_int2(0, 0);
        if (!kStaged && c > 0 && lane == 0) bnext = scr[1];
        int32_t blkH = 0, blkF = 0;  // kStaged: lane i holds boundary row (block start + i)
        uint8_t *mseg = mk + (uint64_t)(c * G + (uint32_t)lane) * p.mask_bs;
        const int T = (int)geo.steps(ld);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the query chars
        for (int t = 0; t < T; ++t) {
            const int r = t - lane + 1;
            uint32_t dch;
            if constexpr (kStaged) {
                dch = (uint32_t)myrow[t - lane] << 8;  // d[r-1]; the pads cover r outside the db
            } else {
                dch = (uint32_t)dnext << 8;
                if (r >= 0 && r < (int)ld) dnext = (int32_t)d[r];
            }
            int32_t bF, bH;
            const int32_t rr = t + 1;  // lane 0's row
            if (c == 0) {
                bF = is4_col1(sc, (uint32_t)rr) + alpha * rr + beta;
                bH = hs4_col0(sc, (uint32_t)rr) + alpha * rr;
            } else if constexpr (kStaged) {
                if (t % G == 0 && rr <= (int)ld) {  // wave-uniform: every group is at step t
                    const int row = rr + lane;
                    if (row <= (int)ld) {
                        const int2 v = scr[row];
                        blkH = v.x;
                        blkF = v.y;
                    }
                    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), on the block step only
                }
                const int src = (bsrc + t % G) * 4;
                bH = __builtin_amdgcn_ds_bpermute(src, blkH);
                bF = __builtin_amdgcn_ds_bpermute(src, blkF);
            } else {
                bH = bnext.x;
                bF = bnext.y;
                if (lane == 0 && t + 2 <= (int)ld) bnext = scr[t + 2];
            }
            const int32_t inF = shr1<G>(bF, pubF);  // I~(r, col0+1)
            const int32_t inH = shr1<G>(bH, pubH);  // H~(r, col0)
            if (r >= 1 && r <= (int)ld) {
                int32_t F = inF;
                const int32_t hm = kCodes == kCodesFull || r == (int)ld ? ~3 : ~1;
                uint32_t sg[8][4 * KD];
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const uint32_t x = qc[k] ^ dch;
                    const int32_t pen = kMinPen ? (int32_t)min(x, (uint32_t)pen_max) : (x ? pen_max : 0);
                    const int32_t M = hd - pen;
                    const int32_t I = F, D = Dn[k];
                    const int32_t H = max(M, max(I, D));
                    const int32_t tO = M + kOpen;
                    if constexpr (kCodes != kCodesNone) {
                        const int32_t Hc = H & hm;
                        const int32_t tOr = tO | kTieOr;
                        sg[0][k] = (uint32_t)(M - Hc);
                        sg[1][k] = (uint32_t)(I - Hc);
                        sg[2][k] = (uint32_t)(D - Hc);
                        sg[4][k] = (uint32_t)(tOr - I);
                        sg[6][k] = (uint32_t)(tOr - D);
                        sg[7][k] = x - 1u;  // sign <=> q == d
                        if constexpr (kCodes == kCodesFull) {
                            const int32_t tOc = tO & ~3;
                            sg[3][k] = (uint32_t)(I - tOc);
                            sg[5][k] = (uint32_t)(D - tOc);
                        } else {
                            sg[3][k] = sg[5][k] = 0u;
                        }
                    }
                    F = max(tO, I);
                    Dn[k] = max(tO, D) + kDstep;
                    hd = Hp[k];
                    Hp[k] = H;
                }
                hd = inH;
                pubF = F;
                pubH = Hp[K - 1];
                if constexpr (kCodes != kCodesNone) {
#pragma unroll
                    for (int k = K; k < 4 * KD; ++k)
#pragma unroll
                        for (int u = 0; u < 8; ++u) sg[u][k] = 0u;  // pad columns: never read
                    MaskWords<K> mw;
#pragma unroll
                    for (int w = 0; w < KD; ++w) {
                        uint32_t s4[8][4];
#pragma unroll
                        for (int u = 0; u < 8; ++u)
#pragma unroll
                            for (int k = 0; k < 4; ++k) s4[u][k] = sg[u][4 * w + k];
                        mw.w[w] = stripe_code_word<kCodes>(s4);
                    }
                    // walk codes: lanes wholly past the query store nothing (as the packed fill)
                    if (kCodes != kCodesWalk || col0 < lq)
                        *reinterpret_cast<MaskWords<K> *>(mseg + (uint64_t)(r - 1) * p.mask_rs) = mw;
                }
                if (lane == G - 1 && c + 1 < nch) scr[r] = make_int2(pubH, pubF);
                if (c == c_end && (uint32_t)lane == l_end && r == (int)ld) {
                    int32_t e = 0;
#pragma unroll
                    for (int k = 0; k < K; ++k)
                        if ((uint32_t)k == k_end) e = Hp[k];
                    end_h[first + gi] = x4_to_x2(e - alpha * (int32_t)ld - beta * (int32_t)lq);
                }
            }
        }
        if (c + 1 < nch) {
            __builtin_amdgcn_s_waitcnt(0x0F70);  // the boundary column is stored
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        }
    }
}

// ------------------------------------------- long pairs: packed stripe fill
// The column-stripe protocol of nw_fill_stripe_kernel with int16 pairs.  A
// stripe's 256 columns are 128 virtual lanes of 2 columns: lane l holds
// virtual lane l in its low halves and virtual lane 64 + l in its high
// halves.  A row's chain runs lanes 0..63 in the low halves and then, one
// step later, lanes 0..63 in the high halves (wave_ror: lane 0's high half
// takes lane 63's low half), so at step t lane l works on row t - l + 1 low
// and row t - l - 63 high.  Every value of row r is held relative to the
// row's frame B(r) = H~(r, c0) & ~1 (even: the panic flags survive), the
// stripe's left input: a row's values lie within 256 * (2|m| + 4|ge|) of it
// whatever the pair's length (packed_stripe_ok).  The frame step
// dB(r) = B(r) - B(r-1) travels down the chain with the row (0 for rows
// outside the db), and a lane moves its carried state (previous-row H, D,
// the diagonal) into the new frame with one v_pk_sub each.  Halves outside
// the db keep their state (bit selects, first 128 and last steps only).
// The last lane tracks B of its high-half row to publish absolute values.
// Mask layout (nw_common.hpp, bs == 0): line t of a stripe's region holds
// the lanes' code dwords of step t, lane l's dword [lo k0, hi k0, lo k1, hi k1].
template <int kCodes>
__global__ __launch_bounds__(64) void nw_fill_stripe_pk_kernel(
    const NwPairDesc *__restrict__ pairs, const uint2 *__restrict__ work,
    const uint8_t *__restrict__ qs, const uint8_t *__restrict__ ds, uint8_t *__restrict__ mask,
    int2 *__restrict__ scratch, uint32_t *__restrict__ prog, uint32_t *__restrict__ err,
    int32_t *__restrict__ end_h, Scoring sc) {
    constexpr int G = 64, K = 2, W = 256;
    const int lane = threadIdx.x;
    const uint2 wk = work[blockIdx.x];
    const NwPairDesc p = pairs[wk.x];
    const uint32_t c = wk.y;
    const uint32_t lq = p.len_q, ld = p.len_db;
    const uint8_t *__restrict__ q = qs + p.q_off;
    const uint8_t *__restrict__ d = ds + p.db_off;
    const uint32_t nch = (lq + W - 1) / W;
    const int2 *__restrict__ scr_in = c > 0 ? scratch + p.scratch_off + (uint64_t)(c - 1) * scratch_col(ld) : nullptr;
    int2 *__restrict__ scr_out = c + 1 < nch ? scratch + p.scratch_off + (uint64_t)c * scratch_col(ld) : nullptr;
    const int32_t beta = -2 * sc.gap_extend;
    const int32_t alpha = -2 * sc.match - beta;
    const uint32_t kPen = cst2(2 * (sc.match - sc.mismatch));  // 2 <= pen <= 32
    const uint32_t kOpen = cst2(2 * sc.gap_open);
    const uint32_t kDstep = cst2(2 * sc.gap_extend + alpha);
    auto psub = [](uint32_t a, uint32_t b) { return as_u(as_s2(a) - as_s2(b)); };

    const int c0 = (int)(c * W);
    const int col_lo = c0 + 2 * lane, col_hi = c0 + 128 + 2 * lane;  // my columns: +1, +2
    const int32_t B0 = c == 0 ? 0 : ((hs_row0(sc, (uint32_t)c0) + beta * c0) & ~1);
    uint32_t qc[K], Hp[K], HpB[K], Dn[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int jl = col_lo + k + 1, jh = col_hi + k + 1;
        const uint32_t ca = jl <= (int)lq ? (uint32_t)q[jl - 1] << 5 : 0xE000u;
        const uint32_t cb = jh <= (int)lq ? (uint32_t)q[jh - 1] << 5 : 0xE000u;
        qc[k] = ca | (cb << 16);
        Hp[k] = pkb(hs_row0(sc, (uint32_t)jl) + beta * jl - B0, hs_row0(sc, (uint32_t)jh) + beta * jh - B0);
        Dn[k] = pkb(ds_row1(sc, (uint32_t)jl) + alpha + beta * jl - B0,
                    ds_row1(sc, (uint32_t)jh) + alpha + beta * jh - B0);
    }
    uint32_t hd = pkb(hs_row0(sc, (uint32_t)col_lo) + beta * col_lo - B0,
                      hs_row0(sc, (uint32_t)col_hi) + beta * col_hi - B0);
    uint32_t pubH = Hp[K - 1], pubF = 0x80008000u, dch = 0, dBc = 0;
    int32_t Bprev = B0;   // lane 0's frame of the previous row (wave-uniform)
    int32_t B63 = B0;     // frame of my high-half row (read in the last lane)
    typedef const __attribute__((address_space(4))) uint32_t cu32;  // constant: scalar loads
    cu32 *dw = (cu32 *)((uintptr_t)d & ~(uintptr_t)3);
    const uint32_t doff = 8u * (uint32_t)((uintptr_t)d & 3);
    const uint32_t last_dw = ((uint32_t)ld - 1 + (uint32_t)((uintptr_t)d & 3)) >> 2;
    uint32_t dnidx = min(1u, last_dw);
    uint32_t dcur = dw[0], dnxt = dw[dnidx];
    auto group_chars = [&]() __attribute__((always_inline)) {
        const uint32_t w = doff ? (dcur >> doff) | (dnxt << (32u - doff)) : dcur;
        dcur = dnxt;
        dnidx = min(dnidx + 1, last_dw);
        dnxt = dw[dnidx];
        return w;
    };
    int32_t blkH = 0, blkF = 0;
    bool failed = false;
    uint8_t *mseg = mask + p.mask_off + (uint64_t)c * p.mask_cs + (uint32_t)lane * 4u;
    const int T = (int)ld + 2 * G - 1;
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the query chars
    // lane 0 <- boundary (low half); others <- lane-1 of the previous step;
    // lane 0's high half <- lane 63's low half (the row continues)
    auto chain = [&](uint32_t v, uint32_t bnd16) __attribute__((always_inline)) {
        const uint32_t rot = __builtin_amdgcn_update_dpp(0u, v, 0x13C /*wave_ror:1*/, 0xf, 0xf, false);
        const uint32_t fix = __builtin_amdgcn_perm(rot, bnd16, 0x05040100u);
        return lane == 0 ? fix : rot;
    };
    int32_t gH0 = 0, gH1 = 0, gH2 = 0, gH3 = 0, gF0 = 0, gF1 = 0, gF2 = 0, gF3 = 0;
    auto step = [&](int t, uint32_t(&Hin)[K], uint32_t(&Hout)[K], uint32_t dt, auto pos_c,
                    auto sel_c) __attribute__((always_inline)) {
        constexpr int kPos = decltype(pos_c)::value;
        constexpr bool kSel = decltype(sel_c)::value;  // some half outside the db
        const uint32_t rr = (uint32_t)t + 1;  // lane 0's low-half row
        int32_t inH0 = 0, inF0 = 0, dB0 = 0;
        if (rr <= ld) {
            int32_t bF, bH;
            if (c == 0) {
                bF = is_col1(sc, rr) + alpha * (int32_t)rr + beta;
                bH = hs_col0(sc, rr) + alpha * (int32_t)rr;
            } else {
                if (kPos == 0 && (rr - 1) % kPub == 0) {  // new 32-row block of the left column
                    // rows are published by replacing the kColEmpty preset
                    // (nw_fill_stripe_kernel)
                    const uint32_t row = rr + (uint32_t)lane;
                    uint32_t spins = 0;
                    for (;;) {
                        bool ok = true;
                        if (lane < (int)kPub && row <= ld) {
                            const uint64_t v = __hip_atomic_load((const uint64_t *)(scr_in + row),
                                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            blkH = (int32_t)(uint32_t)v;
                            blkF = (int32_t)(uint32_t)(v >> 32);
                            ok = (uint32_t)blkH != kColEmpty;
                        }
                        if (__builtin_amdgcn_ballot_w64(!ok) == 0 || failed) break;
                        __builtin_amdgcn_s_sleep(2);
                        if (++spins > err[1]) failed = true;
                    }
                }
                const uint32_t sl = (rr - 1) % kPub;
                bH = __builtin_amdgcn_readlane(blkH, sl);
                bF = __builtin_amdgcn_readlane(blkF, sl);
            }
            const int32_t Bn = bH & ~1;
            dB0 = Bn - Bprev;
            Bprev = Bn;
            inH0 = bH - Bn;
            inF0 = bF - Bn;
        }
        dch = chain(dch, dt << 5);
        const uint32_t dB = chain(dBc, (uint32_t)dB0 & 0xFFFFu);
        const uint32_t inF = chain(pubF, (uint32_t)(inF0 + 32768) & 0xFFFFu);
        const uint32_t inH = chain(pubH, (uint32_t)(inH0 + 32768) & 0xFFFFu);
        dBc = dB;
        B63 += (int32_t)dB >> 16;  // the high half's frame step
        // carried state into this row's frame (dB is 0 for a half outside the db)
#pragma unroll
        for (int k = 0; k < K; ++k) {
            Hin[k] = psub(Hin[k], dB);
            Dn[k] = psub(Dn[k], dB);
        }
        hd = psub(hd, dB);
        uint32_t F = inF;
        uint32_t diag = hd;
        uint32_t prv[8];
        uint32_t cw = 0;
        uint32_t Dnew[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t hdk = diag;
            diag = Hin[k];
            const uint32_t pen = umin2(qc[k] ^ dch, kPen);
            const uint32_t M = hdk - pen;
            const uint32_t I = F, D = Dn[k];
            const uint32_t H = umax2(M, umax2(I, D));
            const uint32_t tO = M + kOpen;
            if constexpr (kCodes != kCodesNone) {
                const uint32_t Hc = H & 0xFFFEFFFEu;
                const uint32_t tOr = tO | 0x00010001u;
                uint32_t sg[8];
                sg[0] = psub(M, Hc);
                sg[1] = psub(I, Hc);
                sg[2] = psub(D, Hc);
                sg[4] = psub(tOr, I);
                sg[6] = psub(tOr, D);
                sg[7] = pen - 0x00010001u;
                if constexpr (kCodes == kCodesFull) {
                    const uint32_t tOc = tO & 0xFFFEFFFEu;
                    sg[3] = psub(I, tOc);
                    sg[5] = psub(D, tOc);
                } else {
                    sg[3] = sg[5] = 0u;
                }
                if (k == 0) {
#pragma unroll
                    for (int u = 0; u < 8; ++u) prv[u] = sg[u];
                } else {
                    uint32_t pw[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) pw[u] = col_pair_signs(sg[u], prv[u]);
                    cw = kCodes == kCodesFull ? merge_full(pw) : merge_walk<true>(pw);
                }
            }
            F = umax2(tO, I);
            Dnew[k] = umax2(tO, D) + kDstep;
            Hout[k] = H;
        }
        if constexpr (kSel) {  // keep the state of a half outside the db
            const int rlo = t - lane + 1, rhi = rlo - G;
            const uint32_t vm = ((rlo >= 1 && rlo <= (int)ld) ? 0x0000FFFFu : 0u) |
                                ((rhi >= 1 && rhi <= (int)ld) ? 0xFFFF0000u : 0u);
#pragma unroll
            for (int k = 0; k < K; ++k) {
                Hout[k] = bfi(vm, Hout[k], Hin[k]);
                Dn[k] = bfi(vm, Dnew[k], Dn[k]);
            }
            hd = bfi(vm, inH, hd);
            pubF = bfi(vm, F, pubF);
            pubH = bfi(vm, Hout[K - 1], pubH);
        } else {
#pragma unroll
            for (int k = 0; k < K; ++k) Dn[k] = Dnew[k];
            hd = inH;
            pubF = F;
            pubH = Hout[K - 1];
        }
        if constexpr (kCodes != kCodesNone) *reinterpret_cast<uint32_t *>(mseg) = cw;
        mseg += kCoopLine;
        // the last lane's high-half row t - 126 as absolute values
        const int32_t aH = (int32_t)(pubH >> 16) - 32768 + B63;
        const int32_t aF = (int32_t)(pubF >> 16) - 32768 + B63;
        if constexpr (kPos == 0) gH0 = aH, gF0 = aF;
        if constexpr (kPos == 1) gH1 = aH, gF1 = aF;
        if constexpr (kPos == 2) gH2 = aH, gF2 = aF;
        if constexpr (kPos == 3) gH3 = aH, gF3 = aF;
    };
    auto publish = [&](int t0, int n) __attribute__((always_inline)) {
        if (lane == G - 1 && scr_out) {
            const int lo = max(t0 - (2 * G - 2), 1), hi = min(t0 + n - 1 - (2 * G - 2), (int)ld);
            if (hi >= lo) {
                auto put = [&](int qq, int32_t h, int32_t f) __attribute__((always_inline)) {
                    const int r = t0 + qq - (2 * G - 2);
                    if (qq < n && r >= lo && r <= hi)
                        __hip_atomic_store((uint64_t *)(scr_out + r),
                                           (uint64_t)(uint32_t)h | ((uint64_t)(uint32_t)f << 32),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                };
                put(0, gH0, gF0);
                put(1, gH1, gF1);
                put(2, gH2, gF2);
                put(3, gH3, gF3);
            }
        }
    };
    const std::integral_constant<int, 0> p0;
    const std::integral_constant<int, 1> p1;
    const std::integral_constant<int, 2> p2;
    const std::integral_constant<int, 3> p3;
    const std::true_type slow;
    const std::false_type fast;
    int t = 0;
    for (; t + 3 < T; t += 4) {
        const uint32_t w = group_chars();
        if (t >= 2 * G && t + 3 <= (int)ld - 1) {  // every half of every lane inside the db
            step(t, Hp, HpB, w & 0xFFu, p0, fast);
            step(t + 1, HpB, Hp, (w >> 8) & 0xFFu, p1, fast);
            step(t + 2, Hp, HpB, (w >> 16) & 0xFFu, p2, fast);
            step(t + 3, HpB, Hp, w >> 24, p3, fast);
        } else {
            step(t, Hp, HpB, w & 0xFFu, p0, slow);
            step(t + 1, HpB, Hp, (w >> 8) & 0xFFu, p1, slow);
            step(t + 2, Hp, HpB, (w >> 16) & 0xFFu, p2, slow);
            step(t + 3, HpB, Hp, w >> 24, p3, slow);
        }
        publish(t, 4);
    }
    const int ntail = T - t;
    if (ntail > 0) {
        const uint32_t w = group_chars();
        step(t, Hp, HpB, w & 0xFFu, p0, slow);
        if (ntail > 1) step(t + 1, HpB, Hp, (w >> 8) & 0xFFu, p1, slow);
        if (ntail > 2) step(t + 2, Hp, HpB, (w >> 16) & 0xFFu, p2, slow);
        publish(t, ntail);
    }
    // end cell: every half ends on row ld in the array the last step wrote
    const uint32_t jend = lq - 1;
    if (jend / W == c) {
        const uint32_t o = jend % W, v = o / 2;
        if ((uint32_t)lane == v % 64) {
            const uint32_t hv = v / 64, ke = o % 2;
            uint32_t wv = 0;
#pragma unroll
            for (int k = 0; k < K; ++k)
                if ((uint32_t)k == ke) wv = (ntail & 1) ? HpB[k] : Hp[k];
            const int32_t rel = (int32_t)(hv ? wv >> 16 : wv & 0xFFFFu) - 32768;
            const int32_t Bld = c == 0 ? (hs_col0(sc, ld) + alpha * (int32_t)ld) & ~1
                                       : (int32_t)(uint32_t)__hip_atomic_load(
                                             (const uint64_t *)(scr_in + ld), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT) & ~1;
            end_h[wk.x] = rel + Bld - alpha * (int32_t)ld - beta * (int32_t)lq;
        }
    }
    if (failed && lane == 0) atomicOr(err, 1u);
}

// Score-only results (saln_nw_plan_set_score_only): score and panic status
// from the end value; no traceback fields (flags bit 3).
__global__ __launch_bounds__(256) void nw_score_results_kernel(const NwPairDesc *__restrict__ pairs,
                                                               uint32_t first, uint32_t n,
                                                               const int32_t *__restrict__ end_h,
                                                               saln_nw_result *__restrict__ results,
                                                               Scoring sc) {
    const uint32_t idx = first + blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= first + n) return;
    const NwPairDesc p = pairs[idx];
    const int32_t h = p.len_q && p.len_db ? end_h[idx] : hs_boundary_end(sc, p.len_q, p.len_db);
    saln_nw_result r;
    r.score = h >> 1;
    r.status = (h & 1) ? SALN_REF_PANIC_BOUNDARY : SALN_OK;
    r.cigar_len = 0;
    r.end_states = 0;
    r.printed = 0;
    r.flags = 8;
    r.reserved = 0;
    results[p.pair_id] = r;
}

hipError_t launch_score_results(const NwPairDesc *pairs, uint32_t first, uint32_t n,
                                const int32_t *end_h, saln_nw_result *results, Scoring sc,
                                hipStream_t stream) {
    if (!n) return hipSuccess;
    nw_score_results_kernel<<<dim3((n + 255) / 256), dim3(256), 0, stream>>>(pairs, first, n, end_h,
                                                                            results, sc);
    return hipGetLastError();
}

// ----------------------------------------------------------------- launchers
// variants 0-3: i32 lanes; 4-6: packed i16 (two pairs per lane)
constexpr Geom kVariants[kNumVariants] = {{16, 10}, {16, 16}, {64, 8}, {64, 4},
                                          {8, 19},  {16, 16}, {32, 16}, {16, 10}, {64, 16}};
constexpr bool kPacked[kNumVariants] = {false, false, false, false, true, true, true, true, true};
// Lanes per pair of each variant's fill kernel.  (8-lane groups of 20
// columns writing variant 7's layout measured equal in round 1: 202 VGPRs
// halve the occupancy.)
constexpr uint32_t kFillG[kNumVariants] = {16, 16, 64, 64, 8, 16, 32, 16, 64};


// Dynamic LDS cap of the packed fill's staged db rows: two workgroups per CU.
constexpr size_t kPackedLdsMax = 80 * 1024;
constexpr size_t kLdsPerCu = 160 * 1024;  // MI355X_MICROARCH.md
static bool packed_ok(uint32_t lq, uint32_t ld, const Scoring &sc);

template <int G, int K>
static void fill_i32(dim3 grid, hipStream_t s, const NwPairDesc *pairs, uint32_t first,
                     uint32_t count, const uint8_t *qs, const uint8_t *ds, uint8_t *mask,
                     int2 *scratch, int32_t *end_h, saln_nw_result *, uint32_t *, Scoring sc,
                     int codes, uint32_t ld_max) {
    const size_t lds = (size_t)(256 / G) * (ld_max + 2 * G);
    const int32_t pen_max = 4 * (sc.match - sc.mismatch);  // the i32 fills' V'' scale
    auto go = [&](auto codes_c, auto minpen_c, auto staged_c) {
        nw_fill_lanes_kernel<G, K, decltype(codes_c)::value, decltype(minpen_c)::value,
                             decltype(staged_c)::value>
            <<<grid, dim3(256), decltype(staged_c)::value ? lds : 0, s>>>(
                pairs, first, count, qs, ds, mask, scratch, end_h, sc, ld_max);
    };
    auto by_staged = [&](auto codes_c, auto minpen_c) {
        if (lds <= 65536) go(codes_c, minpen_c, std::true_type{});
        else go(codes_c, minpen_c, std::false_type{});
    };
    auto by_pen = [&](auto codes_c) {
        if (pen_max >= 0 && pen_max <= 256) by_staged(codes_c, std::true_type{});
        else by_staged(codes_c, std::false_type{});
    };
    if (codes == kCodesFull) by_pen(std::integral_constant<int, kCodesFull>{});
    else if (codes == kCodesNone) by_pen(std::integral_constant<int, kCodesNone>{});
    else by_pen(std::integral_constant<int, kCodesWalk>{});
}

// The table-penalty fill's bonuses fit a byte (fill_pk_body, kTab) and its
// frame's floor, a few opens below zero, stays far inside int16.
static bool pk_tab_ok(const Scoring &sc) {
    const int64_t cm = 2ll * sc.match - 4ll * sc.gap_extend, cmm = 2ll * sc.mismatch - 4ll * sc.gap_extend;
    return cmm >= 0 && cm <= 255 && cmm < cm && -(int64_t)sc.gap_open <= 2000;
}
// ... and its values, biased by kFreeBias, stay positive normal halves for
// W-column lanes groups over `rows` rows: X~ = X' + 2|ge|(r + c) is at least
// the all-gap path's 4go + 4ge less an open and a mismatch for M / I / D, at
// most rows (2|m| + 2|ge|) + 2|ge| W plus the boundary flag.
// scale: 2 (V = 2x + p) or 4 (the scale-4 table body, kTabMode 4): every
// bound scales with it, and its bonuses must still fit a byte.
static bool pk_free_ok(const Scoring &sc, uint32_t W, uint32_t rows, int scale = 2) {
    if (!pk_tab_ok(sc)) return false;
    const int64_t m = std::abs(sc.match), mm = std::abs(sc.mismatch), ge = std::abs(sc.gap_extend),
                  go = std::abs(sc.gap_open);
    const int64_t f = scale / 2;
    if (f * (2ll * sc.match - 4ll * sc.gap_extend) > 255) return false;
    const int64_t lo = f * (6 * go + 6 * ge + 2 * mm + 64);
    const int64_t hi = f * ((int64_t)rows * (2 * m + 2 * ge) + 2 * ge * (int64_t)W + 2 * go + 64);
    return lo <= kFreeBias - 0x400 && hi <= 0x7BFF - kFreeBias;
}

template <int G, int K, int KS = K>
static hipError_t fill_pk(dim3 grid, hipStream_t s, const NwPairDesc *pairs, uint32_t first,
                          uint32_t count, const uint8_t *qs, const uint8_t *ds, uint8_t *mask,
                          int32_t *end_h, saln_nw_result *, uint32_t *, Scoring sc,
                          int codes, uint32_t ld_max, bool rebase, const FillExtras &fx) {
    const Options &o = *fx.o;
    const size_t lds = (size_t)(256 / G) * (ld_max + 2 * G) * (rebase ? 2 : 4);
    if (lds > kPackedLdsMax) return hipErrorInvalidValue;  // choose_variant keeps ld below this
    const PlanSrc src{pairs, first, end_h};
    auto big_lds = [](std::initializer_list<const void *> fs, size_t n) -> hipError_t {
        if (n <= 65536) return hipSuccess;
        for (const void *f : fs) {
            const hipError_t e =
                hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPackedLdsMax);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    };
    auto go = [&](auto codes_c, auto rebase_c) -> hipError_t {
        const auto kern = nw_fill_pk_kernel<G, K, decltype(codes_c)::value, PlanSrc, KS,
                                            decltype(rebase_c)::value>;
        if constexpr (decltype(codes_c)::value == kCodesNib && KS == K) {
            // (the table body stages 32-bit row words; a rebasing fallback 16-bit ones)
            // (and keeps four workgroups per CU where the rebasing fill had them)
            const size_t lds_tab = (size_t)(256 / G) * (ld_max + 2 * G) * 4;
            if (o[Opt::PkTab] && fx.bail && pk_free_ok(sc, G * K, ld_max) &&
                lds_tab <= std::max(lds, kLdsPerCu / 4)) {
                constexpr bool kRb = decltype(rebase_c)::value;
                // nw.pk_tab 1: scale 2; 2: the scale-4 body where its window
                // holds the launch, else scale 2; 3: row profiles (scale 2)
                const size_t lds_prof = lds_tab;
                const int sel = o[Opt::PkTab] == 2 && pk_free_ok(sc, G * K, ld_max, 4) ? 4
                                : o[Opt::PkTab] == 3 ? 3 : 2;
                const void *tk = sel == 4 ? (const void *)nw_fill_pk_tab_kernel<G, K, PlanSrc, 4>
                                 : sel == 3 ? (const void *)nw_fill_pk_tab_kernel<G, K, PlanSrc, 3>
                                            : (const void *)nw_fill_pk_tab_kernel<G, K, PlanSrc, 2>;
                const size_t lds_k = sel == 3 ? lds_prof : lds_tab;
                hipError_t e = big_lds({tk}, lds_k);
                if (e == hipSuccess)
                    e = big_lds({(const void *)nw_fill_pk_tabfb_kernel<G, K, PlanSrc, kRb>}, lds_tab);
                if (e != hipSuccess) return e;
                if (sel == 4)
                    nw_fill_pk_tab_kernel<G, K, PlanSrc, 4><<<grid, dim3(256), lds_k, s>>>(
                        src, count, qs, ds, mask, sc, ld_max, fx.bail, fx.epoch);
                else if (sel == 3)
                    nw_fill_pk_tab_kernel<G, K, PlanSrc, 3><<<grid, dim3(256), lds_k, s>>>(
                        src, count, qs, ds, mask, sc, ld_max, fx.bail, fx.epoch);
                else
                    nw_fill_pk_tab_kernel<G, K, PlanSrc, 2><<<grid, dim3(256), lds_k, s>>>(
                        src, count, qs, ds, mask, sc, ld_max, fx.bail, fx.epoch);
                auto fb = [=, bail = fx.bail, epoch = fx.epoch](hipStream_t fs) {
                    nw_fill_pk_tabfb_kernel<G, K, PlanSrc, kRb>
                        <<<dim3(std::min(grid.x, kTabFbBlocks)), dim3(256), lds_tab, fs>>>(
                            src, count, qs, ds, mask, sc, ld_max, bail, epoch, grid.x);
                    return hipGetLastError();
                };
                if (fx.deferred) fx.deferred->push_back(fb);
                else return fb(s);
                return hipSuccess;
            }
        }
        // full parent sets (round 6): the table body with row profiles for the
        // 16-lane geometries (queries of up to 256 columns), nw.pk_tab != 0
        if constexpr (decltype(codes_c)::value == kCodesFull && KS == K && G == 16) {
            const size_t lds_tab = (size_t)(256 / G) * (ld_max + 2 * G) * 4;
            if (o[Opt::PkTab] && fx.bail && pk_free_ok(sc, G * K, ld_max) &&
                lds_tab <= std::max(lds, kLdsPerCu / 4)) {
                constexpr bool kRb = decltype(rebase_c)::value;
                const void *tk = (const void *)nw_fill_pk_tab_kernel<G, K, PlanSrc, 3, kCodesFull>;
                const void *fk = (const void *)nw_fill_pk_tabfb_kernel<G, K, PlanSrc, kRb, kCodesFull>;
                hipError_t e = big_lds({tk, fk}, lds_tab);
                if (e != hipSuccess) return e;
                nw_fill_pk_tab_kernel<G, K, PlanSrc, 3, kCodesFull><<<grid, dim3(256), lds_tab, s>>>(
                    src, count, qs, ds, mask, sc, ld_max, fx.bail, fx.epoch);
                auto fb = [=, bail = fx.bail, epoch = fx.epoch](hipStream_t fs) {
                    nw_fill_pk_tabfb_kernel<G, K, PlanSrc, kRb, kCodesFull>
                        <<<dim3(std::min(grid.x, kTabFbBlocks)), dim3(256), lds_tab, fs>>>(
                            src, count, qs, ds, mask, sc, ld_max, bail, epoch, grid.x);
                    return hipGetLastError();
                };
                if (fx.deferred) fx.deferred->push_back(fb);
                else return fb(s);
                return hipSuccess;
            }
        }
        const hipError_t e = big_lds({(const void *)kern}, lds);
        if (e != hipSuccess) return e;
        kern<<<grid, dim3(256), lds, s>>>(src, count, qs, ds, mask, sc, ld_max, true);
        return hipSuccess;
    };
    auto by_codes = [&](auto rebase_c) {
        if (codes == kCodesFull) return go(std::integral_constant<int, kCodesFull>{}, rebase_c);
        if (codes == kCodesNone) return go(std::integral_constant<int, kCodesNone>{}, rebase_c);
        // the short-query variants (7: 16 x 10, 4: 8 x 19) store 4-bit walk
        // codes, the wider ones bytes
        if constexpr (G * K <= 160) {
            if (codes == kCodesNib) return go(std::integral_constant<int, kCodesNib>{}, rebase_c);
            return hipErrorInvalidValue;
        } else {
            if (codes == kCodesWalk) return go(std::integral_constant<int, kCodesWalk>{}, rebase_c);
            return hipErrorInvalidValue;
        }
    };
    return rebase ? by_codes(std::true_type{}) : by_codes(std::false_type{});
}

// Blocks of a score-only all-vs-all launch of `count` pairs with G-lane
// groups: two pairs per group, 256 / G groups per block, rounded up to whole
// XCD super-blocks of 8 * blocks_per_pack blocks (pack_block).
static uint64_t avsa_blocks(uint32_t G, uint64_t count) {
    const uint64_t gpb = 256 / G, sup = 8 * blocks_per_pack(2 * (uint32_t)gpb);
    const uint64_t groups = (count + 1) / 2;
    return ((groups + gpb - 1) / gpb + sup - 1) / sup * sup;
}

static uint32_t avsa_lanes(int variant) {
    switch (variant) {
        case 4: return 8;
        case 5: case 7: return 16;
        case 6: return 32;
        case 8: return 64;
        default: return 0;
    }
}

// The most pairs one launch of a packed class may take: the dispatch packet's
// grid size is a 32-bit count of work-items (blocks * 256 <= 2^32 - 1), so
// the largest whole number of super-blocks below that, two pairs per group.
uint64_t avsa_chunk_pairs(int variant) {
    const uint32_t G = avsa_lanes(variant);
    if (!G) return 0;
    const uint64_t gpb = 256 / G, sup = 8 * blocks_per_pack(2 * (uint32_t)gpb);
    const uint64_t blocks = (0xFFFFFFFFull / 256) / sup * sup;
    return std::min<uint64_t>(blocks * gpb * 2, 0x80000000ull);  // count is a uint32
}

uint64_t avsa_launch_blocks(int variant, uint64_t count) {
    const uint32_t G = avsa_lanes(variant);
    return G ? avsa_blocks(G, count) : 0;
}

template <int G, int K>
static hipError_t avsa_pk(const AvsaSrc &src, uint32_t count, const uint8_t *qs, const uint8_t *ds,
                          Scoring sc, uint32_t ld_max, hipStream_t s, const uint32_t *generic,
                          const Options &o) {
    constexpr uint32_t gpb = 256 / G;
    const uint64_t blocks = avsa_blocks(G, count);
    if (blocks * 256 > 0xFFFFFFFFull) return hipErrorInvalidConfiguration;  // 32-bit grid
    const dim3 grid((uint32_t)blocks);
    const bool rebase = !packed_ok(G * K, ld_max, sc);
    const size_t lds = (size_t)gpb * (ld_max + 2 * G) * (rebase ? 2 : 4);
    if (lds > kPackedLdsMax) return hipErrorInvalidValue;
    // the table body stages 32-bit row words, the rebasing xor body 16-bit ones
    const size_t lds_tab = (size_t)gpb * (ld_max + 2 * G) * 4;
    const bool tab = generic && o[Opt::PkTab] && pk_free_ok(sc, G * K, ld_max) &&
                     lds_tab <= std::max(lds, kLdsPerCu / 4);
    auto go = [&](auto rebase_c) -> hipError_t {
        if (tab) {
            const auto kern = nw_fill_avsa_tab_kernel<G, K, decltype(rebase_c)::value>;
            if (lds_tab > 65536) {
                const hipError_t e = hipFuncSetAttribute(
                    (const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                    (int)kPackedLdsMax);
                if (e != hipSuccess) return e;
            }
            kern<<<grid, dim3(256), lds_tab, s>>>(src, count, qs, ds, sc, ld_max, true, generic);
            return hipSuccess;
        }
        const auto kern = nw_fill_pk_kernel<G, K, kCodesNone, AvsaSrc, K, decltype(rebase_c)::value>;
        if (lds > 65536) {
            const hipError_t e = hipFuncSetAttribute((const void *)kern,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     (int)kPackedLdsMax);
            if (e != hipSuccess) return e;
        }
        kern<<<grid, dim3(256), lds, s>>>(src, count, qs, ds, nullptr, sc, ld_max, true);
        return hipSuccess;
    };
    return rebase ? go(std::true_type{}) : go(std::false_type{});
}

// The 8 x 19 class with query profiles (AvsaSrcP: count even, pairs
// [base, base + count) of its index space over whole db pairs).  Returns
// hipErrorInvalidValue where the profile kernel does not apply (a db too long
// for one int16 frame): the caller runs launch_avsa instead.
hipError_t launch_avsa_prof(const uint64_t *q_off, const uint64_t *d_off, const uint32_t *q_ids,
                            uint32_t nq, const uint32_t *d_ids, uint32_t nq_total, uint64_t base,
                            uint32_t count, const uint8_t *qs, const uint8_t *ds, int2 *out,
                            Scoring sc, uint32_t ld_max, const uint32_t *generic,
                            hipStream_t stream, const Options &o) {
    constexpr int G = 8, K = 19;
    if (!count) return hipSuccess;
    if ((count | base) & 1u || !packed_ok(G * K, ld_max, sc)) return hipErrorInvalidValue;
    AvsaSrcP src;
    static_cast<AvsaSrc &>(src) = AvsaSrc{q_off, d_off, q_ids, d_ids, nq, nq_total, base, out};
    const uint64_t blocks = avsa_blocks(G, count);
    if (blocks * 256 > 0xFFFFFFFFull) return hipErrorInvalidConfiguration;
    const size_t lds = (size_t)(256 / G) * (ld_max + 2 * G) * 4;
    if (lds > kPackedLdsMax) return hipErrorInvalidValue;
    const auto kern = o[Opt::PkTab] && pk_free_ok(sc, G * K, ld_max) ? nw_fill_avsa_prof_kernel<G, K, true>
                                                       : nw_fill_avsa_prof_kernel<G, K, false>;
    if (lds > 65536) {
        const hipError_t e = hipFuncSetAttribute((const void *)kern,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 (int)kPackedLdsMax);
        if (e != hipSuccess) return e;
    }
    kern<<<dim3((uint32_t)blocks), dim3(256), lds, stream>>>(src, count, qs, ds, sc, ld_max,
                                                              true, generic);
    return hipGetLastError();
}

hipError_t launch_acgt_check(const uint8_t *seq, uint64_t n, uint32_t *flag, hipStream_t stream) {
    if (!n) return hipSuccess;
    const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 2048);
    nw_acgt_check_kernel<<<dim3((uint32_t)blocks), dim3(256), 0, stream>>>(seq, n, flag);
    return hipGetLastError();
}

// Score-only all-vs-all over one packed query class (variant 4-7): pairs
// [base, base + count) of the class's (query, db) index space.
hipError_t launch_avsa(int variant, const uint64_t *q_off, const uint64_t *d_off,
                       const uint32_t *q_ids, uint32_t nq, const uint32_t *d_ids,
                       uint32_t nq_total, uint64_t base, uint32_t count, const uint8_t *qs,
                       const uint8_t *ds, int2 *out, Scoring sc, uint32_t ld_max,
                       hipStream_t stream, const Options &o, const uint32_t *generic) {
    if (!count) return hipSuccess;
    const AvsaSrc src{q_off, d_off, q_ids, d_ids, nq, nq_total, base, out};
    hipError_t e;
    switch (variant) {
        case 4: e = avsa_pk<8, 19>(src, count, qs, ds, sc, ld_max, stream, generic, o); break;
        case 5: e = avsa_pk<16, 16>(src, count, qs, ds, sc, ld_max, stream, generic, o); break;
        case 6: e = avsa_pk<32, 16>(src, count, qs, ds, sc, ld_max, stream, generic, o); break;
        case 7: e = avsa_pk<16, 10>(src, count, qs, ds, sc, ld_max, stream, generic, o); break;
        case 8: e = avsa_pk<64, 16>(src, count, qs, ds, sc, ld_max, stream, generic, o); break;
        default: return hipErrorInvalidValue;
    }
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

// Pairs with an empty side (no fill): out[d * nq_total + q] from the
// boundary formulas.  Index space: (q_ids[i % nq], d_ids[i / nq]).
__global__ __launch_bounds__(256) void nw_avsa_boundary_kernel(
    const uint64_t *__restrict__ q_off, const uint64_t *__restrict__ d_off,
    const uint32_t *__restrict__ q_ids, uint32_t nq, const uint32_t *__restrict__ d_ids,
    uint64_t n, uint32_t nq_total, int2 *__restrict__ out, Scoring sc) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t qi = q_ids ? q_ids[k % nq] : (uint32_t)(k % nq);
    const uint32_t di = d_ids ? d_ids[k / nq] : (uint32_t)(k / nq);
    const int32_t h = hs_boundary_end(sc, (uint32_t)(q_off[qi + 1] - q_off[qi]),
                                      (uint32_t)(d_off[di + 1] - d_off[di]));
    out[(uint64_t)di * nq_total + qi] = make_int2(h >> 1, (h & 1) ? SALN_REF_PANIC_BOUNDARY : SALN_OK);
}

hipError_t launch_avsa_boundary(const uint64_t *q_off, const uint64_t *d_off,
                                const uint32_t *q_ids, uint32_t nq, const uint32_t *d_ids,
                                uint64_t n, uint32_t nq_total, int2 *out, Scoring sc,
                                hipStream_t stream) {
    if (!n) return hipSuccess;
    nw_avsa_boundary_kernel<<<dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream>>>(
        q_off, d_off, q_ids, nq, d_ids, n, nq_total, out, sc);
    return hipGetLastError();
}

// Fallback queries run through an ordinary score-only plan whose pair k is
// (q_ids[k % nq], d_ids[k / nq]); scatter its 16-byte results into out.
__global__ __launch_bounds__(256) void nw_avsa_scatter_kernel(
    const saln_nw_result *__restrict__ res, const uint32_t *__restrict__ q_ids, uint32_t nq,
    const uint32_t *__restrict__ d_ids, uint64_t n, uint32_t nq_total, int2 *__restrict__ out) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const saln_nw_result r = res[k];
    out[(uint64_t)d_ids[k / nq] * nq_total + q_ids[k % nq]] = make_int2(r.score, r.status);
}

hipError_t launch_avsa_scatter(const saln_nw_result *res, const uint32_t *q_ids, uint32_t nq,
                               const uint32_t *d_ids, uint64_t n, uint32_t nq_total, int2 *out,
                               hipStream_t stream) {
    if (!n) return hipSuccess;
    nw_avsa_scatter_kernel<<<dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream>>>(
        res, q_ids, nq, d_ids, n, nq_total, out);
    return hipGetLastError();
}

hipError_t launch_fill(int variant, const NwPairDesc *pairs, uint32_t first, uint32_t count,
                       const uint8_t *qs, const uint8_t *ds, uint8_t *mask, int2 *scratch,
                       int32_t *end_h, saln_nw_result *res, uint32_t *cig, Scoring sc,
                       int codes, uint32_t ld_max, hipStream_t stream, const FillExtras &fx) {
    if (count == 0) return hipSuccess;
    const uint32_t gpb = 256 / kFillG[variant];  // lane groups per block
    const uint32_t groups = kPacked[variant] ? (count + 1) / 2 : count;
    const uint32_t sup = 8 * blocks_per_pack(kPacked[variant] ? 2 * gpb : gpb);
    const dim3 grid(((groups + gpb - 1) / gpb + sup - 1) / sup * sup);
    // packed pairs beyond one int16 frame (packed_ok_rebase) take the rebasing fill
    const bool rebase = kPacked[variant] && !packed_ok(kVariants[variant].W(), ld_max, sc);
    hipError_t e = hipSuccess;
    switch (variant) {
        case 0: fill_i32<16, 10>(grid, stream, pairs, first, count, qs, ds, mask, scratch, end_h, res, cig, sc, codes, ld_max); break;
        case 1: fill_i32<16, 16>(grid, stream, pairs, first, count, qs, ds, mask, scratch, end_h, res, cig, sc, codes, ld_max); break;
        case 2: fill_i32<64, 8>(grid, stream, pairs, first, count, qs, ds, mask, scratch, end_h, res, cig, sc, codes, ld_max); break;
        case 3: return hipErrorInvalidValue;  // stripes: launch_fill_stripes
        case 4: e = fill_pk<8, 19>(grid, stream, pairs, first, count, qs, ds, mask, end_h, res, cig, sc, codes, ld_max, rebase, fx); break;
        case 5: e = fill_pk<16, 16>(grid, stream, pairs, first, count, qs, ds, mask, end_h, res, cig, sc, codes, ld_max, rebase, fx); break;
        case 7: e = fill_pk<16, 10>(grid, stream, pairs, first, count, qs, ds, mask, end_h, res, cig, sc, codes, ld_max, rebase, fx); break;
        case 8: e = fill_pk<64, 16>(grid, stream, pairs, first, count, qs, ds, mask, end_h, res, cig, sc, codes, ld_max, rebase, fx); break;
        default: e = fill_pk<32, 16>(grid, stream, pairs, first, count, qs, ds, mask, end_h, res, cig, sc, codes, ld_max, rebase, fx); break;
    }
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

template <int G, int K, bool kNib = false>
static void tb_lds(hipStream_t s, const NwPairDesc *pairs, uint32_t first, uint32_t n,
                   const uint8_t *mask, const int32_t *end_h, uint32_t *ops, saln_nw_result *res,
                   uint32_t *cig, Scoring sc, const uint8_t *qs, uint32_t waves = 0) {
    constexpr uint32_t nt = tb_lds_threads<G, K, kNib>();
    uint32_t blocks = (n + nt - 1) / nt;
    if (waves) blocks = std::min(blocks, std::max(1u, waves / (nt / 64u)));
    nw_traceback_lds_kernel<G, K, kNib><<<dim3(blocks), dim3(nt), 0, s>>>(
        pairs, first, n, mask, end_h, ops, res, cig, sc, qs);
}

// Traceback of plan range [first, first+n).  variant >= 0: all pairs of that
// fill variant (LDS walker where the segments fit); variant < 0: generic
// walker (pairs with an empty side, or any variant).
hipError_t launch_traceback(int variant, const NwPairDesc *pairs, uint32_t first, uint32_t n,
                            const uint8_t *qs, const uint8_t *ds, const uint8_t *mask,
                            const int32_t *end_h, uint32_t *ops, saln_nw_result *results,
                            uint32_t *cigar, Scoring sc, int stripe_layout, hipStream_t stream,
                            const uint32_t *spec_done, bool nib, uint32_t walk_waves) {
    if (n == 0) return hipSuccess;
    const dim3 grid((n + 255) / 256);
    if (nib && variant != 4 && variant != 7) return hipErrorInvalidValue;
    switch (variant) {
        case 0: tb_lds<16, 10>(stream, pairs, first, n, mask, end_h, ops, results, cigar, sc, qs); break;
        case 1: tb_lds<16, 16>(stream, pairs, first, n, mask, end_h, ops, results, cigar, sc, qs); break;
        case 2: tb_lds<64, 8>(stream, pairs, first, n, mask, end_h, ops, results, cigar, sc, qs); break;
        case 3: {  // column-stripe pairs: one cooperative wave per pair
            // a few pairs: the whole 160 KB (fewer window reloads); batches:
            // 48 KB windows, three waves per CU
            constexpr int kLoaders = 4;  // waves per pair: one walks, all load its windows
            auto go = [&](auto lay_c) -> hipError_t {
                constexpr int kLay = decltype(lay_c)::value;
                constexpr int32_t kSkew = kLay == 1 ? 127 : kLay == 2 ? 0 : 63;
                static const hipError_t attr = hipFuncSetAttribute(
                    (const void *)nw_traceback_coop_kernel<kLoaders, kLay>,
                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                if (attr != hipSuccess) return attr;
                // kLay 2: the window's sequence bytes (272 + rows + 8) beside it
                const int32_t rows = n <= 256 ? (kLay == 2 ? 628 : 632 - (kSkew + 1)) : 128;
                const size_t seq = kLay == 2 ? 272 + (size_t)rows + 16 : 0;
                nw_traceback_coop_kernel<kLoaders, kLay>
                    <<<dim3(n), dim3(64 * kLoaders),
                       (size_t)(rows + kSkew + 1) * kCoopLine + 16 + seq, stream>>>(
                        pairs, first, mask, end_h, results, cigar, sc, rows, qs, ds,
                        SpecArgs{nullptr, nullptr, nullptr, nullptr, spec_done, 0});
                return hipSuccess;
            };
            const hipError_t e = stripe_layout == 1   ? go(std::integral_constant<int, 1>{})
                                 : stripe_layout == 2 ? go(std::integral_constant<int, 2>{})
                                                      : hipErrorInvalidValue;
            if (e != hipSuccess) return e;
            break;
        }
        case 4:  // 8 x 19 groups: 4-bit codes only (byte segments would not fit a slot)
            if (!nib) return hipErrorInvalidValue;
            tb_lds<8, 19, true>(stream, pairs, first, n, mask, end_h, ops, results, cigar, sc, qs,
                                walk_waves);
            break;
        case 5: tb_lds<16, 16>(stream, pairs, first, n, mask, end_h, ops, results, cigar, sc, qs); break;
        case 6: tb_lds<32, 16>(stream, pairs, first, n, mask, end_h, ops, results, cigar, sc, qs); break;
        case 7:
            // (a lane per pair: two per lane made both 16 x 10 walks slower
            // beside the next fill - the 4-bit one in round 5, the full-code
            // one 1.367-1.384 -> 1.429-1.433 ms per step in round 6,
            // profiles/r06_full_walk_ab.jsonl)
            if (nib) tb_lds<16, 10, true>(stream, pairs, first, n, mask, end_h, ops, results, cigar, sc, qs);
            else tb_lds<16, 10>(stream, pairs, first, n, mask, end_h, ops, results, cigar, sc, qs);
            break;
        case 8: tb_lds<64, 16>(stream, pairs, first, n, mask, end_h, ops, results, cigar, sc, qs); break;
        default: {  // empty-side pairs
            GeomTable gt;
            for (int v = 0; v < kNumVariants; ++v) gt.g[v] = kVariants[v];
            nw_traceback_kernel<<<grid, dim3(256), 0, stream>>>(pairs, first, n, qs, ds, mask,
                                                                end_h, results, cigar, sc, gt);
        }
    }
    return hipGetLastError();
}

hipError_t launch_traceback_spec(const NwPairDesc *pairs, SpecArgs sa, uint32_t n_blocks,
                                 uint32_t n_spec_pairs, uint32_t *done, int passes,
                                 const uint8_t *qs, const uint8_t *ds, const uint8_t *mask,
                                 const int32_t *end_h, saln_nw_result *results, uint32_t *cigar,
                                 Scoring sc, int stripe_layout, uint32_t *strict_err,
                                 hipStream_t stream) {
    if (n_blocks == 0 || passes < 1) return hipSuccess;
    constexpr int kLoaders = 4;
    // a stripe walk from its right edge needs ~256 + kCoopSlack rows: two
    // blocks per CU
    constexpr int32_t rows = 296;
    auto go = [&](auto lay_c) -> hipError_t {
        constexpr int kLay = decltype(lay_c)::value;
        constexpr int32_t kSkew = kLay == 1 ? 127 : kLay == 2 ? 0 : 63;
        const size_t lds = (size_t)(rows + kSkew + 1) * kCoopLine + 16 +
                           (kLay == 2 ? 272 + (size_t)rows + 16 : 0);
        static const hipError_t attr = hipFuncSetAttribute(
            (const void *)nw_traceback_coop_kernel<kLoaders, kLay, true>,
            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (attr != hipSuccess) return attr;
        for (int k = 1; k <= passes; ++k) {
            sa.pass = k;
            nw_traceback_coop_kernel<kLoaders, kLay, true>
                <<<dim3(n_blocks), dim3(64 * kLoaders), lds, stream>>>(
                    pairs, 0, mask, end_h, results, cigar, sc, rows, qs, ds, sa);
        }
        return hipGetLastError();
    };
    const hipError_t e = stripe_layout == 1   ? go(std::integral_constant<int, 1>{})
                         : stripe_layout == 2 ? go(std::integral_constant<int, 2>{})
                                              : hipErrorInvalidValue;
    if (e != hipSuccess) return e;
    sa.pass = passes;
    nw_spec_link_kernel<<<dim3(n_spec_pairs), dim3(256), 0, stream>>>(pairs, sa, done, end_h,
                                                                       results, strict_err);
    if (cigar) {
        sa.done = done;
        nw_spec_copy_kernel<<<dim3(n_blocks), dim3(64), 0, stream>>>(pairs, sa, results, cigar);
    }
    return hipGetLastError();
}

// Column spans (nw_span.cpp): one walk from the entry in sa.stripes[1]
// (pass 2 reads the previous pass's exit slot) to where it leaves the span.
hipError_t launch_span_walk(const NwPairDesc *pairs, SpecArgs sa, const uint8_t *qs,
                            const uint8_t *ds, const uint8_t *mask, const int32_t *end_h,
                            Scoring sc, hipStream_t stream) {
    constexpr int kLoaders = 4;
    constexpr int32_t rows = 296;
    const size_t lds = (size_t)(rows + 1) * kCoopLine + 16 + 272 + (size_t)rows + 16;
    static const hipError_t attr = hipFuncSetAttribute(
        (const void *)nw_traceback_coop_kernel<kLoaders, 2, true>,
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (attr != hipSuccess) return attr;
    sa.pass = 2;
    sa.span = 1;
    nw_traceback_coop_kernel<kLoaders, 2, true><<<dim3(1), dim3(64 * kLoaders), lds, stream>>>(
        pairs, 0, mask, end_h, nullptr, nullptr, sc, rows, qs, ds, sa);
    return hipGetLastError();
}

// Column spans: `passes` speculative passes over the span's walker stripes
// (one block each, sa.blocks), the rightmost entered at sa.entry_s1's given
// entry; the host links the stored walks (nw_span.cpp).
hipError_t launch_span_spec(const NwPairDesc *pairs, SpecArgs sa, uint32_t n_blocks, int passes,
                            const uint8_t *qs, const uint8_t *ds, const uint8_t *mask,
                            const int32_t *end_h, Scoring sc, hipStream_t stream, int pass_lo) {
    constexpr int kLoaders = 4;
    constexpr int32_t rows = 296;
    const size_t lds = (size_t)(rows + 1) * kCoopLine + 16 + 272 + (size_t)rows + 16;
    static const hipError_t attr = hipFuncSetAttribute(
        (const void *)nw_traceback_coop_kernel<kLoaders, 2, true>,
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (attr != hipSuccess) return attr;
    sa.span = 0;  // every stripe stops at its own left edge
    for (int k = pass_lo; k <= passes; ++k) {
        sa.pass = k;
        nw_traceback_coop_kernel<kLoaders, 2, true><<<dim3(n_blocks), dim3(64 * kLoaders), lds, stream>>>(
            pairs, 0, mask, end_h, nullptr, nullptr, sc, rows, qs, ds, sa);
    }
    return hipGetLastError();
}

// Returns once rows r0 .. r1 of a boundary column are published (the row
// fill's 8-byte (H~, I~) elements, preset to kColEmpty), so that work queued
// behind it (an RCCL send of those rows) reads them.  Bounded like the fill's
// own waits: each row's wait gets err[1] polls (the count restarts per row),
// then err[0] bit 0.
__global__ __launch_bounds__(64) void nw_span_watch_kernel(const int2 *__restrict__ col,
                                                           uint32_t r0, uint32_t r1,
                                                           uint32_t *__restrict__ err) {
    const uint32_t lim = err[1];
    bool failed = false;
    for (uint32_t r = r0 + threadIdx.x; r <= r1 && !failed; r += 64) {
        uint32_t spins = 0;
        for (;;) {
            const uint64_t v = __hip_atomic_load((const uint64_t *)(col + r), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
            if ((uint32_t)v != kColEmpty) break;
            if (++spins > lim) {
                failed = true;
                break;
            }
            __builtin_amdgcn_s_sleep(8);
        }
    }
    if (__builtin_amdgcn_ballot_w64(failed) && threadIdx.x == 0) atomicOr(err, 1u);
}

// One device, two spans: forwards rows r0 .. r1 of src's outbox into dst's
// inbox as they are published, 64 rows per round (one wave; each row one
// 8-byte sc1 load once published and one sc1 store, the form of the fill's
// own publication), so dst's first stripe sees them row by row.  Each row's
// wait gets err[1] polls (the count restarts per row, as in the fill), so the
// limit bounds one wait, not the upstream span's whole fill.
__global__ __launch_bounds__(64) void nw_span_relay_kernel(const int2 *__restrict__ src,
                                                           int2 *__restrict__ dst, uint32_t r0,
                                                           uint32_t r1, uint32_t *__restrict__ err) {
    const uint32_t lim = err[1];
    bool failed = false;
    for (uint32_t base = r0; base <= r1 && !failed; base += 64) {
        const uint32_t r = base + threadIdx.x;
        if (r <= r1) {
            uint64_t v;
            uint32_t spins = 0;
            for (;;) {
                v = __hip_atomic_load((const uint64_t *)(src + r), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
                if ((uint32_t)v != kColEmpty) break;
                if (++spins > lim) {
                    failed = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            if (!failed)
                __hip_atomic_store((uint64_t *)(dst + r), v, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        failed = __builtin_amdgcn_ballot_w64(failed) != 0;
    }
    if (failed && threadIdx.x == 0) atomicOr(err, 1u);
}

// Diagnostic (saln_device_cu_probe): where the waves of a launch run.  One
// wave per workgroup records its HW_ID (gfx9 layout: wave 3:0, SIMD 5:4,
// CU 11:8, SH 12, SE 15:13) and XCC_ID registers; vector stores only.
__global__ __launch_bounds__(64) void nw_cu_probe_kernel(uint32_t *__restrict__ hw,
                                                         uint32_t *__restrict__ xcc) {
    const uint32_t h = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
    const uint32_t x = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    // keep the wave resident a while so a launch spreads over the CUs it may use
    for (int k = 0; k < 64; ++k) __builtin_amdgcn_s_sleep(8);
    if (threadIdx.x == 0) {
        hw[blockIdx.x] = h;
        xcc[blockIdx.x] = x;
    }
}

hipError_t launch_cu_probe(uint32_t n_blocks, uint32_t *hw, uint32_t *xcc, hipStream_t stream) {
    if (!n_blocks) return hipSuccess;
    nw_cu_probe_kernel<<<dim3(n_blocks), dim3(64), 0, stream>>>(hw, xcc);
    return hipGetLastError();
}

hipError_t launch_span_relay(const int2 *src, int2 *dst, uint32_t r0, uint32_t r1, uint32_t *err,
                             hipStream_t stream) {
    if (r1 < r0) return hipSuccess;
    nw_span_relay_kernel<<<dim3(1), dim3(64), 0, stream>>>(src, dst, r0, r1, err);
    return hipGetLastError();
}

hipError_t launch_span_watch(const int2 *col, uint32_t r0, uint32_t r1, uint32_t *err,
                             hipStream_t stream) {
    if (r1 < r0) return hipSuccess;
    nw_span_watch_kernel<<<dim3(1), dim3(64), 0, stream>>>(col, r0, r1, err);
    return hipGetLastError();
}

// one stripe per SIMD (kPlaceLone) when a launch's stripes fit the device's
// SIMDs (option nw.rows_lone); XCD-local neighbours (kPlaceXcd) on top when
// the caller's stream may use every CU (option nw.rows_xcd)
static uint32_t device_simds() {
    static const uint32_t simds = [] {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return 0u;
        return 4u * (uint32_t)cus;
    }();
    return simds;
}

// XCD runs of a lone launch (kPlaceXcd: workgroup b on XCD b % 8, also on a
// CU-masked stream - tests/test_span_gpu.py) need every run resident at
// once: a run's first stripe waits for the previous XCD's last one, a later
// workgroup.  The stream's mask holds per XCD (bit c: a CU of XCD c mod 8,
// profiles/r04_cu_map.json; an XCD without a bit runs unmasked) CUs whose
// SIMDs must cover the run, one stripe per SIMD.
static bool xcd_fit(hipStream_t s, uint32_t run, uint32_t nw) {
    if (nw > kXcdSlots) return false;  // one slot per wave in the err buffer
    int dev = 0, cus = 0, xcds = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipDeviceGetAttribute(&xcds, hipDeviceAttributeNumberOfXccs, dev) != hipSuccess)
        return false;
    if (xcds != 8 || cus % 8) return false;  // the kernel's b % 8 mapping
    uint32_t m[32] = {};
    const uint32_t words = std::min<uint32_t>(32, ((uint32_t)cus + 31) / 32);
    if (hipExtStreamGetCUMask(s, words, m) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    uint32_t per[8] = {};
    for (uint32_t c = 0; c < (uint32_t)cus; ++c)
        if (m[c / 32] >> (c % 32) & 1u) ++per[c % 8];
    for (uint32_t x = 0; x < 8; ++x)
        if (4u * (per[x] ? per[x] : (uint32_t)cus / 8) < run) return false;
    return true;
}

hipError_t launch_fill_stripes(const NwPairDesc *pairs, const uint2 *work, uint32_t n_work,
                               const uint8_t *qs, const uint8_t *ds, uint8_t *mask,
                               int2 *scratch, uint32_t *prog, uint32_t *err, int32_t *end_h,
                               Scoring sc, int codes, int layout, int rows_k, hipStream_t stream,
                               const Options &o, uint32_t epoch) {
    if (!n_work) return hipSuccess;
    const dim3 grid(n_work), block(64);
    const bool pk = layout == 1;
    if (layout == 2) {  // row-synchronous stripes of 64 * rows_k columns
        const int32_t pm = 4 * (sc.match - sc.mismatch);
        auto go = [&](auto k_c, auto codes_c, auto minpen_c) {
            constexpr int kK = decltype(k_c)::value;
            constexpr int kC = decltype(codes_c)::value;
            constexpr bool kP = decltype(minpen_c)::value;
            const uint32_t nw = n_work * (4 / kK);
            const bool lone = o[Opt::RowsLone] && nw <= device_simds();
            const uint32_t run = (nw + 7) / 8;
            if (lone && o[Opt::RowsXcd] && nw >= 16 && xcd_fit(stream, run, nw)) {
                nw_fill_rows_kernel<kK, kC, kP, kPlaceXcd><<<dim3(8 * run), block, 0, stream>>>(
                    pairs, work, qs, ds, mask, scratch, err, end_h, sc, nw, run, epoch);
            } else if (lone) {
                nw_fill_rows_kernel<kK, kC, kP, kPlaceLone><<<dim3(nw), block, 0, stream>>>(
                    pairs, work, qs, ds, mask, scratch, err, end_h, sc, nw, 0, 0);
            } else {
                nw_fill_rows_kernel<kK, kC, kP, kPlaceShared><<<dim3(nw), block, 0, stream>>>(
                    pairs, work, qs, ds, mask, scratch, err, end_h, sc, nw, 0, 0);
            }
        };
        auto by_k = [&](auto codes_c, auto minpen_c) {
            if (rows_k == 2) go(std::integral_constant<int, 2>{}, codes_c, minpen_c);
            else go(std::integral_constant<int, 1>{}, codes_c, minpen_c);
        };
        auto by_codes = [&](auto minpen_c) {
            if (codes == kCodesFull) by_k(std::integral_constant<int, kCodesFull>{}, minpen_c);
            else if (codes == kCodesNone) by_k(std::integral_constant<int, kCodesNone>{}, minpen_c);
            else by_k(std::integral_constant<int, kCodesWalk>{}, minpen_c);
        };
        if (pm >= 0 && pm <= 256) by_codes(std::true_type{});
        else by_codes(std::false_type{});
        return hipGetLastError();
    }
    if (!pk) return hipErrorInvalidValue;  // (round 1's skewed i32 stripes are retired)
    if (codes == kCodesFull)
        nw_fill_stripe_pk_kernel<kCodesFull><<<grid, block, 0, stream>>>(pairs, work, qs, ds, mask, scratch, prog, err, end_h, sc);
    else if (codes == kCodesNone)
        nw_fill_stripe_pk_kernel<kCodesNone><<<grid, block, 0, stream>>>(pairs, work, qs, ds, mask, scratch, prog, err, end_h, sc);
    else
        nw_fill_stripe_pk_kernel<kCodesWalk><<<grid, block, 0, stream>>>(pairs, work, qs, ds, mask, scratch, prog, err, end_h, sc);
    return hipGetLastError();
}

// Host path: pack each pair's CIGAR words (capacity-spaced at src_off) densely
// at dst_off, so only the used words cross PCIe.  One wave per pair.
__global__ __launch_bounds__(256) void nw_cigar_compact_kernel(
    const saln_nw_result *__restrict__ res, const uint64_t *__restrict__ src_off,
    const uint64_t *__restrict__ dst_off, const uint32_t *__restrict__ src,
    uint32_t *__restrict__ dst, uint64_t n) {
    const uint64_t k = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
    if (k >= n) return;
    const uint32_t len = res[k].cigar_len;
    const uint32_t *s = src + src_off[k];
    uint32_t *d = dst + dst_off[k];
    for (uint32_t i = threadIdx.x % 64; i < len; i += 64) d[i] = s[i];
}

hipError_t launch_cigar_compact(const saln_nw_result *res, const uint64_t *src_off,
                                const uint64_t *dst_off, const uint32_t *src, uint32_t *dst,
                                uint64_t n, hipStream_t stream) {
    if (!n) return hipSuccess;
    nw_cigar_compact_kernel<<<dim3((uint32_t)((n + 3) / 4)), dim3(256), 0, stream>>>(
        res, src_off, dst_off, src, dst, n);
    return hipGetLastError();
}

Geom variant_geom(int v) { return kVariants[v]; }

// The packed stripe fill holds a row relative to the stripe's left input:
// within 256 columns of it values span 256 * (2|m| + 4|ge|) plus the gap
// and penalty offsets of M / I / D (see nw_fill_stripe_pk_kernel).
// The packed stripe fill: its 128-virtual-lane chain doubles a stripe's skew,
// so one long pair (C4, 391 waves alone on their SIMDs) fills slower (45.4 vs
// 40.1 ms) although the step is cheaper; once the stripe waves fill the chip
// it wins (400 x 5 kbp pairs: 8.0 vs 9.2 ms end to end).  Chosen per plan
// from the stripe-wave count; option nw.stripe_pk = 0 / 1 forces it.
// Row-fill columns per lane: K = 1 (64-column stripes) while every stripe
// wave of the plan has a SIMD to itself (a shorter row step: C1 0.197 ->
// 0.188 ms, 5 kbp 0.75 -> 0.70 ms), else K = 2 (C4: 1,564 K = 1 waves share
// SIMDs, 19.5 vs 14.5 ms).  Option nw.rows_k = 1, 2 or 4 forces it (read per
// plan).
int stripe_rows_k(uint64_t waves_k1, const Options &o) {
    if (const int64_t v = o[Opt::RowsK]) return v == 1 ? 1 : 2;
    return waves_k1 <= 1024 ? 1 : 2;
}

bool stripe_packed(const Scoring &sc, uint64_t n_waves, bool wide, const Options &o) {
    const int64_t force = o[Opt::StripePk];  // -1 auto
    if (force == 0) return false;
    if (force != 1 && (n_waves < kStripePkMinWaves || !wide)) return false;
    const int64_t pen = 2ll * (sc.match - sc.mismatch);
    if (pen < 2 || pen > 32 || sc.gap_extend > 0 || sc.gap_open > 0) return false;
    const int64_t m = std::abs(sc.match), ge = std::abs(sc.gap_extend), go = std::abs(sc.gap_open);
    return 256 * (2 * m + 4 * ge) + 4 * (go + ge) + 2 * pen + 512 < 30000;
}
bool variant_packed(int v) { return kPacked[v]; }

// Packed i16 is exact while every value and every same-cell difference stays
// inside int16 with the position offsets of nw_fill_pk_kernel (see there):
// `rows` rows of growth a and lq columns of growth b from the frame's origin.
static bool packed_range_ok(uint32_t lq, uint32_t rows, const Scoring &sc) {
    const int64_t pen = 2ll * (sc.match - sc.mismatch);
    // pen >= 2: the q==d bit comes from the penalty (0 or pen in each half)
    if (pen < 2 || pen > 32 || sc.gap_extend > 0 || sc.gap_open > 0) return false;
    const int64_t span = std::max<int64_t>(
        {std::abs(sc.match), std::abs(sc.mismatch), std::abs(sc.gap_open) + std::abs(sc.gap_extend)});
    const int64_t a = 2 * (std::abs(sc.match) + std::abs(sc.gap_extend)) + 2 * span;
    return (int64_t)rows * a + (int64_t)lq * (2 * std::abs(sc.gap_extend) + 2 * span) + 256 < 30000;
}
static bool packed_ok(uint32_t lq, uint32_t ld, const Scoring &sc) {
    return packed_range_ok(lq, ld, sc);
}
// The rebasing fill (kRebase).  At step t a lane's value is
// X~(r,c) - drift * r0 with r in [r0 - G, r0 + kRebaseSteps) and
//   X~(r,c) - drift*r0 = [X~(r,c) - X~(r,0)] + [X~(r,0) - drift*r] + drift*(r - r0):
// the first term lies in [2*go, c*(2|m| + 4|ge|)] (a row's H exceeds its
// column-0 value by at most c*(m - ge), the c columns' diagonal gain over the
// gap it replaces, and falls below it by at most a gap; beta*c on top), the
// second is the constant 2*(go + ge) + 1 while hs_col0 is linear (ld <= 4096
// and |go| + 4097*|ge| < 2^15: the sentinel floor is not reached), the third
// is at most |drift| * (period + G).  M / I / D sit within an open + extend +
// penalty of H.  The db length is also bounded by the staged rows
// (kPackedLdsMax).
static bool packed_ok_rebase(uint32_t lq, uint32_t ld, const Scoring &sc, uint32_t G, uint32_t W) {
    const int64_t pen = 2ll * (sc.match - sc.mismatch);
    if (pen < 2 || pen > 32 || sc.gap_extend > 0 || sc.gap_open > 0 || lq > W) return false;
    const uint32_t gpb = 256 / G;
    if ((size_t)gpb * (ld + 2 * G) * 2 > kPackedLdsMax || ld > 4096) return false;  // 16-bit rows
    const int64_t m = std::abs(sc.match), ge = std::abs(sc.gap_extend), go = std::abs(sc.gap_open);
    if (go + 4097 * ge >= 32768) return false;
    const int64_t drift = std::abs(2 * sc.gap_extend - 2 * sc.match + 2 * sc.gap_extend);
    // column term [-(2go + 1), W*(2m + 4ge) + 2(go + ge)] centred by rebase_center
    const int64_t col = (int64_t)W * (2 * m + 4 * ge);
    const int64_t half = std::max<int64_t>(col - rebase_center(sc, (int32_t)W), rebase_center(sc, (int32_t)W));
    const int64_t bound = half + (kRebaseSteps + (int64_t)G) * drift + 4 * (go + ge) + 2 * pen + 512;
    return bound < 30000;
}

int choose_variant(uint32_t len_q, uint32_t len_db, const Scoring &sc, bool narrow) {
    // the packed fills carry V' = 2V + p (no alive flag): sentinel-free pairs only
    const bool free = sentinel_free(sc, len_q, len_db);
    if (!free) return len_q <= 160 ? 0 : len_q <= 256 ? 1 : len_q <= 512 ? 2 : 3;
    // 8 x 19 groups (4-bit walk codes): queries of <= 152 columns, one
    // int16 frame or the rebasing one (launch_fill decides from the widest)
    if (narrow && len_q <= 152) {
        const Geom g = kVariants[4];
        if (packed_ok(g.W(), len_db, sc) || packed_ok_rebase(len_q, len_db, sc, g.G, g.W())) return 4;
    }
    if (packed_ok(len_q, len_db, sc)) {
        if (len_q <= 160) return 7;
        if (len_q <= 256) return 5;
        if (len_q <= 512) return 6;
    }
    // longer db: the same packed variants with a rebasing int16 frame; 513 to
    // 1,024 query columns in 64-lane groups (narrower queries would leave
    // most of those lanes idle: the i32 lanes are faster for them)
    for (const int v : {7, 5, 6}) {
        const Geom g = kVariants[v];
        if (len_q <= g.W() && packed_ok_rebase(len_q, len_db, sc, g.G, g.W())) return v;
    }
    if (len_q > 512 && packed_ok_rebase(len_q, len_db, sc, 64, 1024)) return 8;
    if (len_q <= 160) return 0;
    if (len_q <= 256) return 1;
    if (len_q <= 512) return 2;
    return 3;  // column stripes, one wave each (nw_fill_stripe_kernel)
}

}  // namespace saln

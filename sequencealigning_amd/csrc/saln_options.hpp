// Process-wide tuning options of the engine (include/saln.h saln_option_set).
//
// Every knob that selects a kernel geometry or an A/B variant lives here and
// is set through one explicit C-ABI call; nothing is read from the process
// environment, so an inherited variable cannot change what a benchmark
// times.  All options have the product's defaults; tools/ and tests set them
// for A/Bs and parity sweeps.
#pragma once
#include <atomic>
#include <cstdint>

namespace saln {

enum class Opt : int {
    PkSteady = 0,       // "nw.pk_steady": packed fill steady-step loop (1) or generic steps (0)
    WideMinPairs,       // "nw.wide_min_pairs": 513-1,024-column pairs a plan needs for the 64-lane packed fill
    TbChunks,           // "nw.tb_chunks": fill/traceback sub-batches per execute
    FillLdsMin,         // "nw.fill_lds_min": LDS floor per packed-fill workgroup (occupancy A/B)
    RowsK,              // "nw.rows_k": row-fill columns per lane (0 auto, 1, 2, 4)
    StripePk,           // "nw.stripe_pk": packed column stripes (-1 auto, 0 off, 1 forced)
    Spec,               // "nw.spec": speculative stripe walks (1) or the sequential walker only (0)
    SpecPasses,         // "nw.spec_passes": speculative walk passes
    SpecStrict,         // "nw.spec_strict": a walk that does not link raises SALN_FLAG_SPEC_UNLINKED
    AvsaNarrow,         // "nw.avsa_narrow": 8 x 19 lane groups for the score-only all-vs-all
    NibCodes,           // "nw.nib_codes": 4-bit walk codes for the short-query packed fills
    NarrowWalk,         // "nw.narrow_walk": 8 x 19 lane groups for queries of <= 152 columns
    RowsWpg,            // "nw.rows_wpg": row-fill stripes (waves) per workgroup, 1-4
    RowsLone,           // "nw.rows_lone": a row fill that fits the SIMDs gets one stripe per SIMD
    WalkPrio,           // "nw.walk_prio": issue priority (s_setprio) of the LDS walker's waves
    AvsaProfile,        // "nw.avsa_profile": query-profile penalties in the 8 x 19 all-vs-all fill
    PkTab,              // "nw.pk_tab": table penalties + extension-free frame in the 4-bit-code fills
    Wfa2SeqLds,         // "wfa2.seq_lds": LDS bytes for staged sequences (corrected WFA)
    Wfa2W1,             // "wfa2.w1": first-pass ring width (0 auto)
    Wfa2W2,             // "wfa2.w2": second-pass ring width (0 auto)
    HostTiming,         // "host.timing": stage times of the host paths on stderr
    Count
};

struct OptDesc {
    const char *name;
    int64_t def, lo, hi;
};

const OptDesc &opt_desc(Opt o);
int64_t opt(Opt o);  // current value (relaxed atomic load)

}  // namespace saln

// Tuning options of the engine (include/saln.h saln_option_set,
// saln_context_option_set).
//
// Every knob that selects a kernel geometry or an A/B variant lives here and
// is set through an explicit C-ABI call; nothing is read from the process
// environment, so an inherited variable cannot change what a benchmark
// times.  Two levels:
//   - the process registry (saln_option_set): the defaults of every context;
//   - a context's overrides (saln_context_option_set): that context only.
// A plan, an all-vs-all handle or a span takes a snapshot of its context's
// effective values when it is created (Options) and its launches read only
// that snapshot: two contexts on two threads can run different kernel
// choices at once, and a later option change never reaches a live plan.
#pragma once
#include <atomic>
#include <cstdint>

namespace saln {

enum class Opt : int {
    WideMinPairs = 0,   // "nw.wide_min_pairs": 513-1,024-column pairs a plan needs for the 64-lane packed fill
    RowsK,              // "nw.rows_k": row-fill columns per lane (0 auto, 1, 2)
    StripePk,           // "nw.stripe_pk": packed column stripes (-1 auto, 0 off, 1 forced)
    Spec,               // "nw.spec": speculative stripe walks (1) or the sequential walker only (0)
    SpecPasses,         // "nw.spec_passes": speculative walk passes
    SpecStrict,         // "nw.spec_strict": a walk that does not link raises SALN_FLAG_SPEC_UNLINKED
    AvsaNarrow,         // "nw.avsa_narrow": 8 x 19 lane groups for the score-only all-vs-all
    RowsLone,           // "nw.rows_lone": a row fill that fits the SIMDs gets one stripe per SIMD
    RowsXcd,            // "nw.rows_xcd": XCD-local neighbours for row fills whose stripes fit the SIMDs
    AvsaProfile,        // "nw.avsa_profile": query-profile penalties in the 8 x 19 all-vs-all fill
    PkTab,              // "nw.pk_tab": table penalties + extension-free frame in the 4-bit-code fills (1: scale 2, 2: scale 4 where it fits, 3: scale 2 with row profiles, the default); != 0: the full-code 16-lane fills' row-profile body
    WalkWaves,          // "nw.walk_waves": waves of an LDS walk launch (-1 auto, 0 a lane per pair)
    Wfa2SeqLds,         // "wfa2.seq_lds": LDS bytes for staged sequences (corrected WFA)
    Wfa2W1,             // "wfa2.w1": first-pass ring width (0 auto)
    Wfa2W2,             // "wfa2.w2": second-pass ring width (0 auto)
    HostTiming,         // "host.timing": stage times of the host paths on stderr
    HostPrefaultMb,     // "host.prefault_mb": host buffer a new context faults in while HIP starts
    Count
};
constexpr int kNumOpts = (int)Opt::Count;

struct OptDesc {
    const char *name;
    int64_t def, lo, hi;
};

// A snapshot of effective option values (a context's at the time its plan,
// handle or span was created).
struct Options {
    int64_t v[kNumOpts];
    int64_t operator[](Opt o) const { return v[(int)o]; }
};

const OptDesc &opt_desc(Opt o);
int opt_find(const char *name);         // index, or -1
int64_t opt(Opt o);                     // the process registry's current value
Options opt_registry();                 // the whole registry (relaxed loads)

// A context's overrides on top of the registry (saln_context_option_set).
struct OptOverrides {
    std::atomic<uint64_t> set{0};       // bit i: option i overridden
    std::atomic<int64_t> v[kNumOpts] = {};
    Options effective() const;          // registry with the overrides applied
};

}  // namespace saln

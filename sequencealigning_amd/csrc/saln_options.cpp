// saln_option_* / saln_context_option_* (include/saln.h): the engine's
// tuning knobs in one table (saln_options.hpp).
#include "saln_options.hpp"

#include <cstring>
#include <string>

#include "nw_host.hpp"
#include "saln.h"

namespace saln {

namespace {
// name, default, min, max
const OptDesc kDesc[kNumOpts] = {
    {"nw.wide_min_pairs", 1536, 0, int64_t(1) << 40},
    {"nw.rows_k", 0, 0, 2},
    {"nw.stripe_pk", -1, -1, 1},
    {"nw.spec", 1, 0, 1},
    {"nw.spec_passes", 3, 0, 16},
    {"nw.spec_strict", 0, 0, 1},
    {"nw.avsa_narrow", 1, 0, 1},
    {"nw.rows_lone", 1, 0, 1},
    {"nw.rows_xcd", 1, 0, 1},
    {"nw.avsa_profile", 1, 0, 1},
    {"nw.pk_tab", 3, 0, 3},
    {"nw.walk_waves", -1, -1, 1 << 20},
    {"wfa2.seq_lds", 24 * 1024, 0, 64 * 1024},
    {"wfa2.w1", 0, 0, 4096},
    {"wfa2.w2", 0, 0, 4096},
    {"host.timing", 0, 0, 1},
    {"host.prefault_mb", 0, 0, 1 << 16},
};
struct Values {
    std::atomic<int64_t> v[kNumOpts];
    Values() {
        for (int i = 0; i < kNumOpts; ++i) v[i].store(kDesc[i].def, std::memory_order_relaxed);
    }
};
Values g_vals;  // kDesc is constant-initialized, so it is ready before this runs
std::atomic<int64_t> *const g_val = g_vals.v;

// index of a known option whose value is in range, else -1 (error set)
int checked(const char *name, int64_t value, bool check_value) {
    const int i = opt_find(name);
    if (i < 0) {
        set_error(std::string("unknown option ") + (name ? name : "(null)"));
        return -1;
    }
    const OptDesc &d = kDesc[i];
    if (check_value && (value < d.lo || value > d.hi)) {
        set_error(std::string("option ") + name + " out of range [" + std::to_string(d.lo) + ", " +
                  std::to_string(d.hi) + "]");
        return -1;
    }
    return i;
}
}  // namespace

const OptDesc &opt_desc(Opt o) { return kDesc[(int)o]; }
int64_t opt(Opt o) { return g_val[(int)o].load(std::memory_order_relaxed); }

int opt_find(const char *name) {
    if (!name) return -1;
    for (int i = 0; i < kNumOpts; ++i)
        if (std::strcmp(kDesc[i].name, name) == 0) return i;
    return -1;
}

Options opt_registry() {
    Options o;
    for (int i = 0; i < kNumOpts; ++i) o.v[i] = g_val[i].load(std::memory_order_relaxed);
    return o;
}

Options OptOverrides::effective() const {
    Options o = opt_registry();
    const uint64_t m = set.load(std::memory_order_acquire);
    for (int i = 0; i < kNumOpts; ++i)
        if (m >> i & 1u) o.v[i] = v[i].load(std::memory_order_relaxed);
    return o;
}

}  // namespace saln

extern "C" {

int saln_option_set(const char *name, int64_t value) {
    const int i = saln::checked(name, value, true);
    if (i < 0) return SALN_E_INVALID;
    saln::g_val[i].store(value, std::memory_order_relaxed);
    return SALN_OK;
}

int saln_option_get(const char *name, int64_t *value, int64_t *default_value) {
    const int i = saln::checked(name, 0, false);
    if (i < 0) return SALN_E_INVALID;
    if (value) *value = saln::g_val[i].load(std::memory_order_relaxed);
    if (default_value) *default_value = saln::kDesc[i].def;
    return SALN_OK;
}

int saln_option_name(uint32_t index, const char **name) {
    if (!name || index >= (uint32_t)saln::kNumOpts) return SALN_E_INVALID;
    *name = saln::kDesc[index].name;
    return SALN_OK;
}

int saln_options_reset(void) {
    for (int i = 0; i < saln::kNumOpts; ++i)
        saln::g_val[i].store(saln::kDesc[i].def, std::memory_order_relaxed);
    return SALN_OK;
}

int saln_context_option_set(saln_context *ctx, const char *name, int64_t value) {
    if (!ctx) return SALN_E_INVALID;
    const int i = saln::checked(name, value, true);
    if (i < 0) return SALN_E_INVALID;
    ctx->opts.v[i].store(value, std::memory_order_relaxed);
    ctx->opts.set.fetch_or(1ull << i, std::memory_order_release);
    return SALN_OK;
}

int saln_context_option_get(saln_context *ctx, const char *name, int64_t *value) {
    if (!ctx) return SALN_E_INVALID;
    const int i = saln::checked(name, 0, false);
    if (i < 0) return SALN_E_INVALID;
    if (value) *value = ctx->opts.effective().v[i];
    return SALN_OK;
}

int saln_context_option_clear(saln_context *ctx, const char *name) {
    if (!ctx) return SALN_E_INVALID;
    if (!name) {
        ctx->opts.set.store(0, std::memory_order_release);
        return SALN_OK;
    }
    const int i = saln::checked(name, 0, false);
    if (i < 0) return SALN_E_INVALID;
    ctx->opts.set.fetch_and(~(1ull << i), std::memory_order_release);
    return SALN_OK;
}

}  // extern "C"

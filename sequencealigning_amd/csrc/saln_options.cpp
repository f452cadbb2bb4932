// saln_option_set / saln_option_get (include/saln.h): the engine's tuning
// knobs in one table (saln_options.hpp).
#include "saln_options.hpp"

#include <cstring>
#include <string>

#include "saln.h"

namespace saln {
void set_error(const std::string &msg);

namespace {
constexpr int kN = (int)Opt::Count;
// name, default, min, max
const OptDesc kDesc[kN] = {
    {"nw.pk_steady", 1, 0, 1},
    {"nw.wide_min_pairs", 1536, 0, int64_t(1) << 40},
    {"nw.tb_chunks", 1, 1, 64},
    {"nw.fill_lds_min", 0, 0, 160 * 1024},
    {"nw.rows_k", 0, 0, 4},
    {"nw.stripe_pk", -1, -1, 1},
    {"nw.spec", 1, 0, 1},
    {"nw.spec_passes", 3, 0, 16},
    {"nw.spec_strict", 0, 0, 1},
    {"nw.avsa_narrow", 1, 0, 1},
    {"nw.nib_codes", 1, 0, 1},
    {"nw.narrow_walk", 1, 0, 1},
    {"nw.rows_wpg", 1, 1, 4},
    {"nw.rows_lone", 1, 0, 1},
    {"nw.walk_prio", 3, 0, 3},
    {"nw.avsa_profile", 1, 0, 1},
    {"nw.pk_tab", 1, 0, 1},
    {"wfa2.seq_lds", 24 * 1024, 0, 64 * 1024},
    {"wfa2.w1", 0, 0, 4096},
    {"wfa2.w2", 0, 0, 4096},
    {"host.timing", 0, 0, 1},
};
struct Values {
    std::atomic<int64_t> v[kN];
    Values() {
        for (int i = 0; i < kN; ++i) v[i].store(kDesc[i].def, std::memory_order_relaxed);
    }
};
Values g_vals;  // kDesc is constant-initialized, so it is ready before this runs
std::atomic<int64_t> *const g_val = g_vals.v;

int find(const char *name) {
    if (!name) return -1;
    for (int i = 0; i < kN; ++i)
        if (std::strcmp(kDesc[i].name, name) == 0) return i;
    return -1;
}
}  // namespace

const OptDesc &opt_desc(Opt o) { return kDesc[(int)o]; }
int64_t opt(Opt o) { return g_val[(int)o].load(std::memory_order_relaxed); }

}  // namespace saln

extern "C" {

int saln_option_set(const char *name, int64_t value) {
    const int i = saln::find(name);
    if (i < 0) {
        saln::set_error(std::string("unknown option ") + (name ? name : "(null)"));
        return SALN_E_INVALID;
    }
    const saln::OptDesc &d = saln::kDesc[i];
    if (value < d.lo || value > d.hi) {
        saln::set_error(std::string("option ") + name + " out of range [" + std::to_string(d.lo) +
                        ", " + std::to_string(d.hi) + "]");
        return SALN_E_INVALID;
    }
    saln::g_val[i].store(value, std::memory_order_relaxed);
    return SALN_OK;
}

int saln_option_get(const char *name, int64_t *value, int64_t *default_value) {
    const int i = saln::find(name);
    if (i < 0) {
        saln::set_error(std::string("unknown option ") + (name ? name : "(null)"));
        return SALN_E_INVALID;
    }
    if (value) *value = saln::g_val[i].load(std::memory_order_relaxed);
    if (default_value) *default_value = saln::kDesc[i].def;
    return SALN_OK;
}

int saln_option_name(uint32_t index, const char **name) {
    if (!name || index >= (uint32_t)saln::kN) return SALN_E_INVALID;
    *name = saln::kDesc[index].name;
    return SALN_OK;
}

int saln_options_reset(void) {
    for (int i = 0; i < saln::kN; ++i) saln::g_val[i].store(saln::kDesc[i].def, std::memory_order_relaxed);
    return SALN_OK;
}

}  // extern "C"

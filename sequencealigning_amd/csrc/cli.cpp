// saln — command-line drop-in for the reference binary (src/main.rs:19-80,
// src/parse.rs:8-50): same short/long flags (-q -d -o -v -m -a), same value
// names, same db-outer / query-inner pair order and the same stdout/stderr
// text.  NW alignments are computed by libsaln on the GPU in batches of
// pairs (saln_nw_render_batch: one plan per chunk of the pair loop, each pair
// filled and walked once); the reference's exhaustive block printing is
// replayed on the host from the GPU's parent codes.  The `{:#?}` timing line
// after each NW pair (needleman_wunsch_affine.rs:431) prints that pair's
// share of the batch's device time plus its own host DFS time.
//
// Differences by design: `-a a-star` (the reference default) is not part of
// this engine and is rejected; `-a wfa` caps the score loop (--wfa-steps),
// where the reference would not terminate; a reference panic (boundary index panic of the
// NW traceback) aborts with exit code 101 after the blocks printed before it,
// like the reference, unless --no-abort is given.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <thread>
#include <vector>

#include <sys/stat.h>
#include <sys/uio.h>
#include <unistd.h>

#include <cerrno>

#include "saln.h"

namespace {

struct Args {
    std::string query, db, out = "./results";
    bool verbose = false;
    int mode = SALN_MODE_GLOBAL;
    int algo = 0;  // 0 a-star (reference default), 1 needleman-wunsch, 2 wfa
    int device = 0;
    bool timing = true, abort_on_panic = true;
    uint32_t wfa_steps = 64;  // cap on WFA score steps (the reference loops without one)
    uint64_t max_blocks = 0;
    uint64_t chunk_pairs = 1u << 14;  // pairs per render batch (the first one: a quarter)
    bool stage_times = false;
    bool teardown = false;
    std::vector<std::pair<std::string, int64_t>> options;  // --option NAME=VALUE, in order
};

const char *kUsage =
    "Usage: saln [OPTIONS] --query-file <QUERY_FILE> --db-file <DB_FILE>\n"
    "\n"
    "Options:\n"
    "  -q, --query-file <QUERY_FILE>  Path to query sequence\n"
    "  -d, --db-file <DB_FILE>        path to db sequence\n"
    "  -o, --out-path <OUT_PATH>      out path [default: ./results]\n"
    "  -v, --verbose                  verbose\n"
    "  -m, --mode <MODE>              modus [default: global] [possible values: global, local, "
    "semi-global]\n"
    "  -a, --algo <ALGO>              algo [default: a-star] [possible values: a-star, "
    "needleman-wunsch, wfa]\n"
    "      --device <N>               HIP device [default: 0]\n"
    "      --no-timing                omit the per-pair timing line\n"
    "      --no-abort                 report reference panics and continue\n"
    "      --wfa-steps <N>            cap on WFA score steps [default: 64]\n"
    "      --max-blocks <N>           cap on printed alignments per pair [default: 0 = none]\n"
    "      --chunk-pairs <N>          pairs per GPU batch [default: 16384]\n"
    "      --stage-times              stage times of this run on stderr\n"
    "      --teardown                 the HIP runtime's full tear-down at exit (for profilers)\n"
    "      --option <NAME=VALUE>      set an engine option (saln_option_set; repeatable)\n"
    "  -h, --help                     Print help\n";

[[noreturn]] void usage_error(const std::string &msg) {
    std::fprintf(stderr, "error: %s\n\n%s", msg.c_str(), kUsage);
    std::exit(2);
}

Args parse_args(int argc, char **argv) {
    Args a;
    bool have_q = false, have_d = false;
    for (int k = 1; k < argc; ++k) {
        std::string s = argv[k];
        std::string val;
        auto need = [&](const char *name) -> std::string {
            const size_t eq = s.find('=');
            if (s.rfind("--", 0) == 0 && eq != std::string::npos) return s.substr(eq + 1);
            if (k + 1 >= argc) usage_error(std::string("a value is required for '") + name + "'");
            return argv[++k];
        };
        auto is = [&](const char *sh, const char *lg) {
            return s == sh || s == lg || (s.rfind(std::string(lg) + "=", 0) == 0);
        };
        if (s == "-h" || s == "--help") {
            std::fputs(kUsage, stdout);
            std::exit(0);
        } else if (is("-q", "--query-file")) {
            a.query = need("--query-file <QUERY_FILE>");
            have_q = true;
        } else if (is("-d", "--db-file")) {
            a.db = need("--db-file <DB_FILE>");
            have_d = true;
        } else if (is("-o", "--out-path")) {
            a.out = need("--out-path <OUT_PATH>");
        } else if (s == "-v" || s == "--verbose") {
            a.verbose = true;
        } else if (is("-m", "--mode")) {
            val = need("--mode <MODE>");
            if (val == "global") a.mode = SALN_MODE_GLOBAL;
            else if (val == "local") a.mode = SALN_MODE_LOCAL;
            else if (val == "semi-global") a.mode = SALN_MODE_SEMI_GLOBAL;
            else usage_error("invalid value '" + val + "' for '--mode <MODE>'");
        } else if (is("-a", "--algo")) {
            val = need("--algo <ALGO>");
            if (val == "a-star") a.algo = 0;
            else if (val == "needleman-wunsch") a.algo = 1;
            else if (val == "wfa") a.algo = 2;
            else usage_error("invalid value '" + val + "' for '--algo <ALGO>'");
        } else if (is("--device", "--device")) {
            a.device = std::atoi(need("--device <N>").c_str());
        } else if (s == "--no-timing") {
            a.timing = false;
        } else if (s == "--no-abort") {
            a.abort_on_panic = false;
        } else if (is("--wfa-steps", "--wfa-steps")) {
            a.wfa_steps = (uint32_t)std::strtoul(need("--wfa-steps <N>").c_str(), nullptr, 10);
        } else if (s == "--stage-times") {
            a.stage_times = true;
        } else if (s == "--teardown") {
            a.teardown = true;
        } else if (is("--max-blocks", "--max-blocks")) {
            a.max_blocks = std::strtoull(need("--max-blocks <N>").c_str(), nullptr, 10);
        } else if (is("--option", "--option")) {
            val = need("--option <NAME=VALUE>");
            const size_t eq = val.find('=');
            char *end = nullptr;
            const long long v = eq == std::string::npos ? 0 : std::strtoll(val.c_str() + eq + 1, &end, 10);
            if (eq == std::string::npos || eq == 0 || end == val.c_str() + eq + 1 || *end != '\0')
                usage_error("invalid value '" + val + "' for '--option <NAME=VALUE>'");
            a.options.emplace_back(val.substr(0, eq), (int64_t)v);
        } else if (is("--chunk-pairs", "--chunk-pairs")) {
            a.chunk_pairs = std::max<uint64_t>(1, std::strtoull(need("--chunk-pairs <N>").c_str(), nullptr, 10));
        } else {
            usage_error("unexpected argument '" + s + "' found");
        }
    }
    if (!have_q || !have_d)
        usage_error("the following required arguments were not provided:\n  --query-file "
                    "<QUERY_FILE>\n  --db-file <DB_FILE>");
    return a;
}

// Rust `{:?}` of a char (used for the CharError vector, main.rs:29-35).
std::string rust_char_debug(uint8_t c) {
    switch (c) {
        case '\t': return "'\\t'";
        case '\r': return "'\\r'";
        case '\n': return "'\\n'";
        case '\'': return "'\\''";
        case '\\': return "'\\\\'";
        case 0: return "'\\0'";
        default: break;
    }
    char buf[16];
    if (c < 0x20 || (c >= 0x7F && c < 0xA0) || c == 0xAD) {
        std::snprintf(buf, sizeof(buf), "'\\u{%x}'", c);
        return buf;
    }
    if (c < 0x80) {
        std::snprintf(buf, sizeof(buf), "'%c'", c);
        return buf;
    }
    // Latin-1 code point as UTF-8
    buf[0] = '\'';
    buf[1] = (char)(0xC0 | (c >> 6));
    buf[2] = (char)(0x80 | (c & 0x3F));
    buf[3] = '\'';
    buf[4] = 0;
    return buf;
}

// `{:#?}` of a Vec<char>
std::string vec_char_pretty(const std::vector<uint8_t> &v) {
    if (v.empty()) return "[]";
    std::string s = "[\n";
    for (uint8_t c : v) s += "    " + rust_char_debug(c) + ",\n";
    return s + "]";
}

// `{:#?}` of a std::time::Duration (Debug: integer part + trimmed fraction)
std::string duration_debug(uint64_t ns) {
    const char *unit;
    uint64_t integer, frac, frac_digits;
    if (ns >= 1000000000ull) {
        unit = "s";
        integer = ns / 1000000000ull;
        frac = ns % 1000000000ull;
        frac_digits = 9;
    } else if (ns >= 1000000ull) {
        unit = "ms";
        integer = ns / 1000000ull;
        frac = ns % 1000000ull;
        frac_digits = 6;
    } else if (ns >= 1000ull) {
        unit = "\xC2\xB5s";
        integer = ns / 1000ull;
        frac = ns % 1000ull;
        frac_digits = 3;
    } else {
        return std::to_string(ns) + "ns";
    }
    std::string s = std::to_string(integer);
    if (frac) {
        std::string f = std::to_string(frac);
        f = std::string(frac_digits - f.size(), '0') + f;
        while (!f.empty() && f.back() == '0') f.pop_back();
        s += "." + f;
    }
    return s + unit;
}

struct Rec {
    std::vector<uint8_t> name, seq;
};

// parse_fasta + the match in main.rs:22-60.  Returns false to stop (`return`).
bool load(const std::string &path, const char *which, std::vector<Rec> *out) {
    saln_records *r = nullptr;
    std::vector<uint8_t> bad(1 << 16);
    uint64_t nbad = 0;
    const int rc = saln_parse_fasta(path.c_str(), &r, bad.data(), bad.size(), &nbad);
    if (rc == SALN_E_FASTA) {
        std::string e = saln_last_error();
        const std::string pre = "Fasta could not be opened with err: ";
        if (e.rfind(pre, 0) == 0) e = e.substr(pre.size());
        std::fprintf(stderr, "%s fasta could not be opened: %s\naborting\n", which, e.c_str());
        return false;
    }
    if (rc != SALN_OK && rc != SALN_E_FASTA_CHARS) {
        std::fprintf(stderr, "Unexpected error in %s fasta: %s\n", which, saln_last_error());
        return false;
    }
    if (rc == SALN_E_FASTA_CHARS) {
        if (nbad > bad.size()) {  // re-read with room for every dropped byte
            saln_records_free(r);
            bad.resize(nbad);
            saln_parse_fasta(path.c_str(), &r, bad.data(), bad.size(), &nbad);
        }
        bad.resize(nbad);
        std::fprintf(stderr, "Invalid character '%s' detected in %s fasta; continuing by ignoring it\n",
                     vec_char_pretty(bad).c_str(), which[0] == 'D' ? "db" : "query");
    }
    const uint64_t n = saln_records_count(r);
    out->resize(n);
    for (uint64_t k = 0; k < n; ++k) {
        const uint8_t *nm, *sq;
        uint64_t nl, sl;
        saln_records_get(r, k, &nm, &nl, &sq, &sl);
        (*out)[k].name.assign(nm, nm + nl);
        (*out)[k].seq.assign(sq, sq + sl);
    }
    saln_records_free(r);
    return true;
}

std::string as_str(const std::vector<uint8_t> &v) { return std::string(v.begin(), v.end()); }

// The end of a finished run: the output is flushed and every GPU result has
// been read, so the process leaves without the HIP runtime's tear-down (its
// queues, code objects and GB-sized device and pinned blocks; after main
// 4-108 ms against 58-114 ms on MI355X, profiles/r05_cli_exit_ab.jsonl),
// which the kernel driver reclaims at exit anyway.  --teardown keeps the
// normal exit (e.g. under a profiler whose exit handlers write its results).
int leave(int code, bool teardown) {
    std::fflush(stdout);
    std::fflush(stderr);
    if (teardown) return code;
    std::_Exit(code);
}

}  // namespace

int main(int argc, char **argv) {
    const Args a = parse_args(argc, argv);
    auto t_mark = std::chrono::steady_clock::now();
    auto mark = [&](const char *what) {
        if (!a.stage_times) return;
        const auto n = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[saln cli] %-16s %8.3f ms\n", what,
                     std::chrono::duration<double, std::milli>(n - t_mark).count());
        t_mark = n;
    };
    // wall-clock stamps, so a caller can split its own process time into
    // start-up before main, main, and tear-down after it
    auto clock_stamp = [&](const char *what) {
        if (!a.stage_times) return;
        timespec ts{};
        clock_gettime(CLOCK_REALTIME, &ts);
        std::fprintf(stderr, "[saln-clock] %s %lld\n", what,
                     static_cast<long long>(ts.tv_sec) * 1000000000LL + ts.tv_nsec);
    };
    clock_stamp("main-entry");
    if (a.stage_times) saln_option_set("host.timing", 1);
    // stdout to a file or pipe: large writes (the default 4 KB buffer makes
    // ~10^4 write calls per 45 MB of text); a terminal keeps line buffering
    // (stderr too: --max-blocks prints a line per capped pair)
    if (!isatty(STDOUT_FILENO)) std::setvbuf(stdout, nullptr, _IOFBF, 4u << 20);
    if (!isatty(STDERR_FILENO)) std::setvbuf(stderr, nullptr, _IOFBF, 1u << 20);
    if (a.algo == 0) {
        std::vector<Rec> db, query;  // the reference parses both files first
        if (!load(a.db, "DB", &db) || !load(a.query, "Query", &query)) return 0;
        std::fprintf(stderr,
                     "saln: -a a-star (the reference's A* aligner) is not part of this engine; "
                     "use -a needleman-wunsch or -a wfa\n");
        return 2;
    }
    // The reference's default NW output (every block) runs the host DFS over
    // parent codes downloaded per chunk: the context faults their host buffer
    // in while the HIP runtime starts (host.prefault_mb), sized from the files
    // (~1.3 B of codes per cell, a chunk of at most 2^31 cells; 512 MB at most)
    if (a.algo == 1 && a.max_blocks != 1) {
        struct stat sq{}, sd{};
        if (::stat(a.query.c_str(), &sq) == 0 && ::stat(a.db.c_str(), &sd) == 0) {
            const double cells = std::min((double)sq.st_size * (double)sd.st_size, double(1u << 31));
            const int64_t mb = std::min<int64_t>(512, (int64_t)(cells * 1.3 / (1 << 20)) + 1);
            if (mb >= 16) saln_option_set("host.prefault_mb", mb);
        }
    }
    for (const auto &o : a.options) {
        if (saln_option_set(o.first.c_str(), o.second) != SALN_OK) {
            std::fprintf(stderr, "saln: --option %s=%lld: %s\n", o.first.c_str(), (long long)o.second,
                         saln_last_error());
            return 2;
        }
    }
    // the HIP runtime starts (~0.2 s) while the FASTA files are read
    saln_context *ctx = nullptr;
    int ctx_rc = SALN_OK;
    std::string ctx_err;  // (saln_last_error is per thread)
    std::thread ctx_thread([&] {
        ctx_rc = saln_context_create(a.device, &ctx);
        if (ctx_rc != SALN_OK) ctx_err = saln_last_error();
    });
    std::vector<Rec> db, query;
    const bool loaded = load(a.db, "DB", &db) && load(a.query, "Query", &query);
    mark("load fasta");
    ctx_thread.join();
    if (!loaded) {
        if (ctx) saln_context_destroy(ctx);
        return 0;
    }
    if (ctx_rc != SALN_OK) {
        std::fprintf(stderr, "saln: %s\n", ctx_err.c_str());
        return 1;
    }
    mark("context");
    // Both engines run the pair loop main.rs:61-74 in chunks of pairs in the
    // reference's order (db outer, query inner); each chunk is one batched
    // render call (every pair computed once on the GPU), then printed pair by
    // pair.
    std::vector<uint8_t> qs, ds;
    std::vector<uint64_t> qo{0}, dof{0};
    for (const Rec &q : query) {
        qs.insert(qs.end(), q.seq.begin(), q.seq.end());
        qo.push_back(qs.size());
    }
    for (const Rec &d : db) {
        ds.insert(ds.end(), d.seq.begin(), d.seq.end());
        dof.push_back(ds.size());
    }
    const uint64_t nq = query.size(), nd = db.size(), total = nq * nd;
    std::vector<uint32_t> pq, pd;
    if (a.algo == 2) {  // Algo::Wfa => wfa_align(q, d, mode)  (main.rs:66)
        // A chunk's alignment rows are sized for its longest pair
        // (2 * (len_q + len_db) + 64 bytes per row, two rows per pair); keep
        // them under kWfaRowBytes.
        constexpr uint64_t kWfaPairs = 1u << 16, kWfaRowBytes = 1ull << 30;
        for (uint64_t p0 = 0; p0 < total;) {
            pq.clear();
            pd.clear();
            uint64_t cap = 64;
            for (uint64_t p = p0; p < total && pq.size() < kWfaPairs; ++p) {
                const uint64_t qi = p % nq, di = p / nq;
                const uint64_t c =
                    std::max<uint64_t>(cap, 2 * (query[qi].seq.size() + db[di].seq.size()) + 64);
                if (!pq.empty() && (pq.size() + 1) * 2 * c > kWfaRowBytes) break;
                cap = c;
                pq.push_back((uint32_t)qi);
                pd.push_back((uint32_t)di);
            }
            saln_wfa_text *t = nullptr;
            int rc = saln_wfa_render_batch(ctx, qs.data(), qo.data(), nq, ds.data(), dof.data(),
                                           nd, pq.data(), pd.data(), pq.size(), a.mode,
                                           a.wfa_steps, 0, &t);
            if (rc != SALN_OK) {
                std::fprintf(stderr, "saln: %s\n", saln_last_error());
                saln_context_destroy(ctx);
                return 1;
            }
            for (uint64_t k = 0; k < pq.size(); ++k) {
                const Rec &q = query[pq[k]], &d = db[pd[k]];
                const char *txt = nullptr;
                uint64_t len = 0;
                saln_wfa_result r;
                saln_wfa_text_get(t, k, &txt, &len, &r);
                if (r.status == SALN_NOT_IMPLEMENTED) {
                    std::fprintf(stderr,
                                 "An error occured during alignment of %s and %s\nError in "
                                 "alignment: not implemented\n",
                                 as_str(q.name).c_str(), as_str(d.name).c_str());
                    continue;
                }
                std::fwrite(txt, 1, len, stdout);
                if (r.status == SALN_REF_PANIC_TRIM || r.status == SALN_REF_PANIC_SLICE) {
                    std::fflush(stdout);
                    const char *where = r.status == SALN_REF_PANIC_TRIM
                                            ? "src/wfa.rs: mid > len (Ocean::trim rotate_left)"
                                            : "src/wfa.rs: slice index out of range (rec_tr)";
                    if (a.abort_on_panic) {
                        std::fprintf(stderr,
                                     "thread 'main' panicked at %s\nnote: run with "
                                     "`RUST_BACKTRACE=1` environment variable to display a "
                                     "backtrace\n",
                                     where);
                        saln_wfa_text_free(t);
                        saln_context_destroy(ctx);
                        return 101;
                    }
                    std::fprintf(stderr, "saln: reference panic (%s) for %s vs %s\n",
                                 r.status == SALN_REF_PANIC_TRIM ? "REF_PANIC_TRIM"
                                                                 : "REF_PANIC_SLICE",
                                 as_str(q.name).c_str(), as_str(d.name).c_str());
                    continue;
                }
                if (r.status == SALN_NONCONVERGED)
                    std::fprintf(stderr,
                                 "saln: %s vs %s did not converge within %u score steps (the "
                                 "reference would not terminate)\n",
                                 as_str(q.name).c_str(), as_str(d.name).c_str(), a.wfa_steps);
            }
            saln_wfa_text_free(t);
            p0 += pq.size();
        }
        saln_context_destroy(ctx);
        return 0;
    }
    // Needleman-Wunsch: each chunk is one saln_nw_render_batch (one plan,
    // fill + walk on the GPU).  A chunk holds up to kChunkPairs pairs or
    // ~kChunkCells cells (its full-code mask and the host copy of it stay
    // bounded).  A chunk's text is printed on a thread while the next chunk
    // renders, unless the chunk ends the run (a panic under the reference's
    // abort), which is printed before anything else happens.  The first
    // chunk is a quarter of the others, so printing starts early; the last
    // chunk's print is the part that overlaps nothing.
    const uint64_t kChunkPairs = a.chunk_pairs;
    constexpr uint64_t kChunkCells = 2ull << 30;
    // pair k of a rendered chunk: its text and what the reference does next;
    // returns the process exit code when the run ends here, else -1
    auto print_pair = [&](const Rec &q, const Rec &d, const char *txt, uint64_t len,
                          int32_t status, uint64_t ns) -> int {
        if (status == SALN_NOT_IMPLEMENTED) {  // main.rs:68-74
            std::fprintf(stderr,
                         "An error occured during alignment of %s and %s\nError in alignment: "
                         "not implemented\n",
                         as_str(q.name).c_str(), as_str(d.name).c_str());
            return -1;
        }
        std::fwrite(txt, 1, len, stdout);
        if (status == SALN_REF_PANIC_BOUNDARY) {
            std::fflush(stdout);
            if (a.abort_on_panic) {
                std::fprintf(stderr,
                             "thread 'main' panicked at src/needleman_wunsch_affine.rs: index "
                             "out of bounds (traceback reached a boundary cell other than the "
                             "origin)\nnote: run with `RUST_BACKTRACE=1` environment variable "
                             "to display a backtrace\n");
                return 101;
            }
            std::fprintf(stderr, "saln: reference panic (REF_PANIC_BOUNDARY) for %s vs %s\n",
                         as_str(q.name).c_str(), as_str(d.name).c_str());
            return -1;
        }
        if (status == SALN_ENUM_CAP)
            std::fprintf(stderr, "saln: enumeration capped at %llu blocks for %s vs %s\n",
                         (unsigned long long)a.max_blocks, as_str(q.name).c_str(),
                         as_str(d.name).c_str());
        if (a.timing) std::printf("%s\n", duration_debug(ns).c_str());
        return -1;
    };
    // A chunk's text goes to stdout with writev straight from the render
    // handle's buffers (no copy through the stdio buffer: the all-blocks text
    // of 10^5 G-mut pairs is 1.6 GB, and its copy was the printer's time).
    // Pairs whose status prints anything else go through print_pair, after
    // the gathered text before them.
    auto print_chunk = [&](saln_nw_text *t, const std::vector<uint32_t> &cq,
                           const std::vector<uint32_t> &cd) -> int {
        const uint64_t n = saln_nw_text_count(t);
        std::vector<iovec> iov;
        std::vector<std::string> lines;  // timing lines, alive until written
        iov.reserve(1024);
        lines.reserve(512);
        bool ok = true;
        auto drain = [&]() {
            if (iov.empty()) return;
            std::fflush(stdout);  // whatever stdio holds goes first
            size_t i = 0;
            while (ok && i < iov.size()) {
                const int cnt = (int)std::min<size_t>(iov.size() - i, 1024);
                ssize_t w = ::writev(STDOUT_FILENO, iov.data() + i, cnt);
                if (w < 0) {
                    if (errno == EINTR) continue;
                    ok = false;
                    break;
                }
                // skip the fully written entries, trim a partial one
                while (i < iov.size() && w >= (ssize_t)iov[i].iov_len) w -= (ssize_t)iov[i++].iov_len;
                if (i < iov.size() && w > 0) {
                    iov[i].iov_base = (char *)iov[i].iov_base + w;
                    iov[i].iov_len -= (size_t)w;
                }
            }
            iov.clear();
            lines.clear();
        };
        for (uint64_t k = 0; k < n; ++k) {
            const char *txt = nullptr;
            uint64_t len = 0, blocks = 0, ns = 0;
            int32_t status = SALN_OK;
            saln_nw_text_get(t, k, &txt, &len, &blocks, &status, nullptr, &ns);
            if (status != SALN_OK) {  // stderr lines, a flush or the abort: the stdio path
                drain();
                const int e = print_pair(query[cq[k]], db[cd[k]], txt, len, status, ns);
                if (e >= 0) return e;
                continue;
            }
            if (len) iov.push_back(iovec{(void *)txt, (size_t)len});
            if (a.timing) {
                lines.push_back(duration_debug(ns) + "\n");
                iov.push_back(iovec{(void *)lines.back().data(), lines.back().size()});
            }
            if (iov.size() >= 1022 || lines.size() >= 511) drain();
        }
        drain();
        if (!ok) {
            std::fprintf(stderr, "saln: writing the output failed\n");
            return 1;
        }
        return -1;
    };
    std::thread printer;
    double print_ms = 0;  // the printer thread's time for its chunk
    auto join_printer = [&]() {
        if (!printer.joinable()) return;
        printer.join();
        if (a.stage_times) std::fprintf(stderr, "[saln cli] %-16s %8.3f ms\n", "print (beside)", print_ms);
    };
    auto finish = [&](int code) {
        join_printer();
        std::fflush(stdout);
        if (code != 0) saln_context_destroy(ctx);
        return code == 0 ? leave(code, a.teardown) : code;
    };
    for (uint64_t p0 = 0; p0 < total;) {
        pq.clear();
        pd.clear();
        uint64_t cells = 0;
        const uint64_t cap = p0 == 0 ? std::max<uint64_t>(1, kChunkPairs / 4) : kChunkPairs;
        for (uint64_t p = p0; p < total && pq.size() < cap; ++p) {
            const uint64_t qi = p % nq, di = p / nq;
            const uint64_t c = (uint64_t)query[qi].seq.size() * db[di].seq.size();
            if (!pq.empty() && cells + c > kChunkCells) break;
            cells += c;
            pq.push_back((uint32_t)qi);
            pd.push_back((uint32_t)di);
        }
        p0 += pq.size();
        saln_nw_text *t = nullptr;
        mark("chunk plan");
        const int rc = saln_nw_render_batch(ctx, qs.data(), qo.data(), nq, ds.data(), dof.data(), nd,
                                            pq.data(), pd.data(), pq.size(), a.mode, a.max_blocks,
                                            a.abort_on_panic ? 1 : 0, &t);
        mark("render batch");
        join_printer();  // the previous chunk's text comes first
        if (rc != SALN_OK) {
            // a chunk that fails as a whole (one pair whose scores leave the
            // engine's int32 range, an allocation) is rendered pair by pair,
            // so every pair before the failing one is printed first, in the
            // reference's streaming order (main.rs:61-74)
            if (t) saln_nw_text_free(t);
            for (uint64_t k = 0; k < pq.size(); ++k) {
                const Rec &q = query[pq[k]], &d = db[pd[k]];
                saln_nw_text *one = nullptr;
                if (saln_nw_render_text(ctx, q.seq.data(), q.seq.size(), d.seq.data(), d.seq.size(),
                                        a.mode, a.max_blocks, &one) != SALN_OK) {
                    std::fflush(stdout);
                    std::fprintf(stderr, "saln: %s\n", saln_last_error());
                    return finish(1);
                }
                const char *txt = nullptr;
                uint64_t len = 0, blocks = 0, ns = 0;
                int32_t status = SALN_OK;
                saln_nw_text_get(one, 0, &txt, &len, &blocks, &status, nullptr, &ns);
                const int e = print_pair(q, d, txt, len, status, ns);
                saln_nw_text_free(one);
                if (e >= 0) return finish(e);
            }
            mark("print");
            continue;
        }
        bool ends = false;  // a panic the reference aborts at
        if (a.abort_on_panic)
            for (uint64_t k = 0, n = saln_nw_text_count(t); k < n && !ends; ++k) {
                int32_t status = SALN_OK;
                saln_nw_text_get(t, k, nullptr, nullptr, nullptr, &status, nullptr, nullptr);
                ends = status == SALN_REF_PANIC_BOUNDARY;
            }
        if (ends || p0 >= total) {  // the last chunk: nothing to overlap
            const int e = print_chunk(t, pq, pd);
            saln_nw_text_free(t);
            mark("print");
            if (e >= 0) return finish(e);
            continue;
        }
        printer = std::thread([&, t, cq = pq, cd = pd]() {
            const auto s0 = std::chrono::steady_clock::now();
            print_chunk(t, cq, cd);  // (no exit code: the chunk has no abort)
            saln_nw_text_free(t);
            print_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - s0).count();
        });
    }
    join_printer();
    // The context is left to the process exit: destroying it frees the GB-sized
    // device and host blocks one by one (measured 0.26 s at the end of a 10^5-pair
    // run), which the exit's teardown does anyway.
    mark("exit");
    clock_stamp("main-exit");
    return leave(0, a.teardown);
}

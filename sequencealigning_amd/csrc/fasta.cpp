// FASTA reader of the C ABI — replaces parse_fasta (src/parse.rs:54-99).
// Behaviour kept from the reference: extension must be exactly fa|fasta|fna
// (:55-60, has_extension :101-106); '>' opens a record whose name keeps the
// '>' (:67-74); a newline ends the name (:76-81); newlines in sequence lines
// are skipped; every byte outside {A,G,C,T,N} is dropped and reported
// (:82-88), so lowercase and '\r' are dropped too; the implicit record that
// collects bytes before the first '>' is discarded (:91).
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "saln.h"

namespace saln {
void set_error(const std::string &msg);
}

struct saln_records {
    std::vector<std::vector<uint8_t>> names, seqs;
};

namespace {

bool valid_extension(const char *path) {
    // Path::extension(): text after the last '.' of the file name, provided
    // the name does not start with that dot and the dot is not the last char.
    const char *base = std::strrchr(path, '/');
    base = base ? base + 1 : path;
    const char *dot = std::strrchr(base, '.');
    if (!dot || dot == base) return false;
    const char *ext = dot + 1;
    return !std::strcmp(ext, "fa") || !std::strcmp(ext, "fasta") || !std::strcmp(ext, "fna");
}

inline bool allowed(uint8_t c) { return c == 'A' || c == 'G' || c == 'C' || c == 'T' || c == 'N'; }

}  // namespace

extern "C" {

int saln_parse_fasta_buffer(const uint8_t *buf, uint64_t len, saln_records **out,
                            uint8_t *bad_chars, uint64_t bad_cap, uint64_t *n_bad) {
    if (!out || (len && !buf)) return SALN_E_INVALID;
    auto *r = new saln_records;
    std::vector<uint8_t> name, seq;
    bool in_name = false, started = false;  // `started`: a '>' has been seen
    uint64_t nbad = 0;
    for (uint64_t k = 0; k < len; ++k) {
        const uint8_t c = buf[k];
        if (c == '>') {
            if (started) {
                r->names.push_back(std::move(name));
                r->seqs.push_back(std::move(seq));
            }
            name.assign(1, c);
            seq.clear();
            started = true;
            in_name = true;
            continue;
        }
        if (in_name) {
            if (c == '\n') {
                in_name = false;
                continue;
            }
            name.push_back(c);
        } else if (c == '\n') {
            continue;
        } else if (!allowed(c)) {
            if (bad_chars && nbad < bad_cap) bad_chars[nbad] = c;
            ++nbad;
        } else if (started) {
            seq.push_back(c);
        }
    }
    if (started) {
        r->names.push_back(std::move(name));
        r->seqs.push_back(std::move(seq));
    }
    *out = r;
    if (n_bad) *n_bad = nbad;
    return nbad ? SALN_E_FASTA_CHARS : SALN_OK;
}

int saln_parse_fasta(const char *path, saln_records **out, uint8_t *bad_chars, uint64_t bad_cap,
                     uint64_t *n_bad) {
    if (!path || !out) return SALN_E_INVALID;
    *out = nullptr;
    if (n_bad) *n_bad = 0;
    if (!valid_extension(path)) {
        saln::set_error("Fasta could not be opened with err: invalid input parameter");
        return SALN_E_FASTA;
    }
    FILE *f = std::fopen(path, "rb");
    const int err_no = errno;
    if (!f) {
        // io::Error Display: "<strerror> (os error N)"
        saln::set_error(std::string("Fasta could not be opened with err: ") + std::strerror(err_no) +
                        " (os error " + std::to_string(err_no) + ")");
        return SALN_E_FASTA;
    }
    std::vector<uint8_t> data;
    uint8_t chunk[1 << 16];
    size_t n;
    while ((n = std::fread(chunk, 1, sizeof(chunk), f)) > 0) data.insert(data.end(), chunk, chunk + n);
    const bool err = std::ferror(f) != 0;
    std::fclose(f);
    if (err) {
        saln::set_error("Fasta could not be opened with err: read error");
        return SALN_E_FASTA;
    }
    return saln_parse_fasta_buffer(data.data(), data.size(), out, bad_chars, bad_cap, n_bad);
}

uint64_t saln_records_count(const saln_records *r) { return r ? r->names.size() : 0; }

int saln_records_get(const saln_records *r, uint64_t i, const uint8_t **name, uint64_t *name_len,
                     const uint8_t **seq, uint64_t *seq_len) {
    if (!r || i >= r->names.size()) return SALN_E_INVALID;
    if (name) *name = r->names[i].data();
    if (name_len) *name_len = r->names[i].size();
    if (seq) *seq = r->seqs[i].data();
    if (seq_len) *seq_len = r->seqs[i].size();
    return SALN_OK;
}

void saln_records_free(saln_records *r) { delete r; }

}  // extern "C"

// CPU test (tests/test_host_dfs.py): the host DFS renderer saln::render_blocks
// (nw_host.cpp, the text of render batches and the CLI) against the oracle's
// literal DFS (oracle/refcpu.c ref_nw_traceback_dfs_blocks, needleman_wunsch_affine.rs:242-334)
// on 4,000 random short pairs: two- to five-letter alphabets with N, empty
// sides, near-identical pairs, block caps 0 (all) and 1-4; the parent codes laid out
// as the device stores them (I parents of I(i, j+1) at (i, j), D parents of D(i+1, j)
// at (i, j), bits inverted).
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <random>
#include "nw_host.hpp"
extern "C" {
typedef struct { int32_t *M,*I,*D; uint8_t *pM,*pI,*pD; size_t lq, ld; } ref_nw_mats;
int ref_nw_fill(const uint8_t *q, size_t lq, const uint8_t *d, size_t ld, ref_nw_mats *o);
void ref_nw_free(ref_nw_mats *m);
void ref_nw_dense_mask(const ref_nw_mats *m, uint8_t *out);
int ref_nw_traceback_dfs_blocks(const uint8_t *q, const uint8_t *d, const ref_nw_mats *m, char *out,
                                size_t out_cap, size_t *out_len, uint64_t max_pops, uint64_t max_blocks, uint64_t *n_blocks);
}
int main() {
    std::mt19937_64 r(11); const char *A = "ACGTN";
    int bad = 0, n = 0;
    for (int it = 0; it < 4000; ++it) {
        int lq = r() % 40, ld = r() % 40; int alpha = 2 + r() % 3;
        std::string q, d; for (int i = 0; i < lq; ++i) q.push_back(A[r() % alpha]); for (int i = 0; i < ld; ++i) d.push_back(A[r() % alpha]);
        if (it % 3 == 0) { d = q; if (!d.empty() && r()%2) d.erase(r() % d.size(), 1); ld = d.size(); }
        ref_nw_mats m; ref_nw_fill((const uint8_t*)q.data(), lq, (const uint8_t*)d.data(), ld, &m);
        std::vector<uint8_t> dense((lq+1)*(ld+1)); ref_nw_dense_mask(&m, dense.data());
        uint64_t mb = it % 4 == 0 ? 0 : 1 + r() % 4;
        std::vector<char> buf(1 << 22); size_t olen = 0; uint64_t nb = 0;
        int rc = ref_nw_traceback_dfs_blocks((const uint8_t*)q.data(), (const uint8_t*)d.data(), &m, buf.data(), buf.size(), &olen, 10000000, mb, &nb);
        ref_nw_free(&m);
        if (rc == 2 || olen > buf.size()) continue;
        std::vector<uint8_t> mm(std::max(1, lq*ld));
        // device layout: the I parents of I(i, j+1) at (i, j), the D parents of D(i+1, j) at (i, j)
        for (int i = 1; i <= ld; ++i) for (int j = 1; j <= lq; ++j) {
            uint8_t b = dense[i*(lq+1)+j] & 7;
            if (j + 1 <= lq) b |= dense[i*(lq+1)+j+1] & 0x18;
            if (i + 1 <= ld) b |= dense[(i+1)*(lq+1)+j] & 0x60;
            mm[(i-1)*lq+(j-1)] = b ^ 0x7F;
        }
        saln::HostMask hm; hm.m = mm.data(); hm.g = saln::Geom{1, (uint32_t)std::max(1, lq)};
        hm.rs = lq; hm.bs = 1; hm.cs = 0; hm.lq = lq; hm.ld = ld;
        std::string out;
        auto o = saln::render_blocks(hm, (const uint8_t*)q.data(), (const uint8_t*)d.data(), mb, &out);
        const int want_st = rc == 1 ? SALN_REF_PANIC_BOUNDARY : rc == 3 ? SALN_ENUM_CAP : SALN_OK;
        ++n;
        if (out != std::string(buf.data(), olen) || o.blocks != nb || o.status != want_st) {
            if (bad++ < 5) printf("mismatch it=%d q=%s d=%s mb=%llu rc=%d st=%d blocks %llu/%llu\n", it, q.c_str(), d.c_str(), (unsigned long long)mb, rc, o.status, (unsigned long long)o.blocks, (unsigned long long)nb);
        }
    }
    printf("%d checked, %d mismatches\n", n, bad);
    return bad != 0;
}

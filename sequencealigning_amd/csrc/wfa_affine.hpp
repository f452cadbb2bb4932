// Shared host/device definitions of the corrected gap-affine WFA engine
// (wfa_affine_kernels.hip, wfa_affine_host.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace saln {

struct WfaAffPair {  // 32 bytes
    uint64_t q_off, d_off;
    uint32_t lq, ld;
    uint32_t out;  // index into scores
    uint32_t reserved;
};

struct WfaAffParams {
    int32_t x, o, e;     // mismatch, gap open, gap extend (gap of length L: o + L*e)
    int32_t g;           // gcd(x, o+e, e): scores step in units of g
    int32_t RM, RI;      // ring slots: M (max(x, o+e)/g + 1), I/D (e/g + 1)
    int32_t W;           // diagonals per wavefront slot (power of two)
    int32_t max_score;   // give up above this penalty (score -1)
    int32_t seqcap;      // LDS bytes for a pair's staged sequences (0: read them from HBM)
};

size_t wfa_affine_lds_bytes(const WfaAffParams &prm, bool wide);
// n_dev (optional): the pair count is read from device memory (n bounds it)
// next: a zeroed device counter the launch's waves take pair indices from
hipError_t launch_wfa_affine(const WfaAffPair *pairs, uint32_t n, const uint8_t *qs,
                             const uint8_t *ds, const WfaAffParams &prm, bool wide,
                             uint32_t grid, const uint32_t *n_dev, uint32_t *next, int32_t *scores,
                             hipStream_t stream);
hipError_t launch_wfa_affine_compact(const WfaAffPair *pairs, uint32_t n, const int32_t *scores,
                                     WfaAffPair *out, uint32_t *count, hipStream_t stream);

}  // namespace saln

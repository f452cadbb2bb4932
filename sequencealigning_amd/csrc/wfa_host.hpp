// WFA engine: device structures shared by wfa_kernels.hip and wfa_host.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "saln.h"

namespace saln {

// One pair as the WFA kernel sees it.
struct WfaPairDesc {
    uint64_t q_off, db_off;  // byte offsets into the query / db buffers
    uint64_t aln_off;        // byte offset of the pair's alignment rows (2 x aln_cap)
    uint32_t len_q, len_db;
    uint32_t pair_id;        // index into results (and the per-pair logs)
    int32_t mode;            // saln_mode
    uint32_t aln_cap;        // bytes per alignment row
    uint32_t reserved;
};

// Tensor-history arena of one launch (layout: wfa_kernels.hip header).
struct WfaArena {
    int32_t *hdr;
    int32_t *off;
    uint32_t *meta;
    uint8_t *tsome;
    uint32_t nl, S, W;
};

hipError_t launch_wfa(const WfaPairDesc *pairs, uint32_t first, uint32_t n, const uint8_t *qs,
                      const uint8_t *ds, const WfaArena &arena, uint32_t max_steps,
                      saln_wfa_result *results, uint8_t *aln, int32_t *lohi_log, uint8_t *ev_log,
                      uint32_t ev_cap, WfaPairDesc *rerun, uint32_t *rerun_cnt,
                      hipStream_t stream);

}  // namespace saln

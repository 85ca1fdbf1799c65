// nsg_host.h -- host-side context shared by the single-pass path (nsg_coder.hip) and the wide path
// (nsg_wide.hip).  Not part of the public ABI (include/nsg_coder.h only sees an opaque ns_ctx).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "nsg_common.h"

namespace nsg {

// per-stream statistics of the wide path's first pass
struct WideStat {
    float m;          // row max (valid ids)
    float m2;         // second largest value (>= 2 ids are always collected)
    float r;          // reference of the fast sum
    uint32_t active;  // 0: stream done/inactive this step
    double S_lo;      // proven interval of the canonical float64 row sum
    double S_hi;
    double S_fast;
    uint32_t exact;   // 1: the fast bound is unusable, the CDF kernel computes the exact sum
    uint32_t pad;
    double S_r, B_r, U_r;  // raw streaming sums against r (statistics: row_stats_from_stream)
    float xt;         // wide_stream_kernel: final collection threshold (segment entries below it are stale)
    uint32_t nraw;    // wide_stream_kernel: entries written to the stream's segment
};

}  // namespace nsg

struct NsgWide {
    int cap = 0;                    // keys per stream segment (= vocab)
    uint64_t* keys_in = nullptr;    // [max_batch * cap]
    uint64_t* keys_out = nullptr;   // [max_batch * cap]
    unsigned int* count = nullptr;  // [max_batch] collected ids per stream
    unsigned int* begin = nullptr;  // [max_batch] segment offsets for the sort
    unsigned int* end = nullptr;    // [max_batch]
    unsigned int* todo = nullptr;   // [1 + max_batch] streams left to wide_cdf_kernel: count, then ids
    nsg::WideStat* stat = nullptr;  // [max_batch]
    void* sort_tmp = nullptr;
    size_t sort_tmp_bytes = 0;
    uint32_t* vals_in = nullptr;    // NS_DTYPE_F64 rank rows: array positions sorted with the 64-bit keys
    uint32_t* vals_out = nullptr;   // [max_batch * cap]
};

struct ns_ctx {
    int device;
    int max_batch;
    int vocab;
    int max_k;
    int precision;
    int dtype;
    unsigned long long* d_counters;
    NsgWide wide;
    const uint8_t* sent_end;  // device table [vocab] for NS_STEP_FINISH_SENT (ns_set_sentence_end)
    double* stats;            // encode statistics sink [B][4] (ns_set_stats), nullable
    int32_t* ranked;          // decode rank export [B][ranked_stride] (ns_set_rank_export), nullable
    int ranked_stride;
    uint64_t* stamps;         // NSG_STAMPS diagnostic builds: per-stream phase stamps
    const int32_t* rk_count;  // NS_DTYPE_F64: entries per row [B] (ns_set_rank_rows), nullable = vocab
    const int32_t* rk_idmap;  // NS_DTYPE_F64: token id of each row entry [B][idmap_stride], nullable = position
    int64_t rk_idmap_stride;
    int rk_dict;              // NS_DTYPE_F64: rows are dict ProbDists (cap_bits universe, codec/quality.py:161-171)
    std::string err;
};

// wide (top-k beyond the single-pass limit) path, nsg_wide.hip
int nsg_wide_alloc(ns_ctx* ctx);  // NS_OK or NS_ERR_HIP
void nsg_wide_free(ns_ctx* ctx);
bool nsg_wide_launch(ns_ctx* ctx, const nsg::StepParams& p, bool decode, hipStream_t s);
bool nsg_rank_launch(ns_ctx* ctx, const nsg::StepParams& p, bool decode, hipStream_t s);  // src rank coder

// nsg_common.h -- device helpers shared by the single-pass coder kernel (nsg_coder.hip) and the
// wide (large top-k) path (nsg_wide.hip).  Canonical arithmetic here must stay bit-identical to
// oracle/nsg_oracle.c.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nsg_coder.h"

#pragma clang fp contract(off)

namespace nsg {

#ifndef NSG_WPB
#define NSG_WPB 4
#endif
#ifndef NSG_CAND
#define NSG_CAND 1024
#endif
#ifndef NSG_PREFETCH
#define NSG_PREFETCH 4
#endif
#ifndef NSG_LOAD_AUX
#define NSG_LOAD_AUX 2  // cache policy of the streamed logit loads: nt (read-once stream)
#endif
#ifndef NSG_MIN_WAVES_PER_EU
#define NSG_MIN_WAVES_PER_EU 4
#endif

constexpr int WAVE = 64;
#define NS_COUNTER_SHARDS 256
constexpr int WPB = NSG_WPB;            // waves (streams) per workgroup
constexpr int CAND = NSG_CAND;          // candidate keys per wave (8 B each, LDS)
constexpr int PREFETCH = NSG_PREFETCH;  // tiles in flight per wave

// ------------------------------------------------------------------------------------------------
// canonical float64 exp -- identical operation sequence to or_exp_canon (oracle/nsg_oracle.c)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ double exp_canon(double d) {
    if (!(d >= -700.0)) return 0.0;
    const double n = __builtin_rint(d * 1.44269504088896338700e+00);
    double r = __builtin_fma(-n, 6.93147180369123816490e-01, d);
    r = __builtin_fma(-n, 1.90821492927058770002e-10, r);
    double p = 1.60590438368216145994e-10;
    p = __builtin_fma(p, r, 2.08767569878680989792e-09);
    p = __builtin_fma(p, r, 2.50521083854417187751e-08);
    p = __builtin_fma(p, r, 2.75573192239858906526e-07);
    p = __builtin_fma(p, r, 2.75573192239858906526e-06);
    p = __builtin_fma(p, r, 2.48015873015873015873e-05);
    p = __builtin_fma(p, r, 1.98412698412698412698e-04);
    p = __builtin_fma(p, r, 1.38888888888888888889e-03);
    p = __builtin_fma(p, r, 8.33333333333333333333e-03);
    p = __builtin_fma(p, r, 4.16666666666666666667e-02);
    p = __builtin_fma(p, r, 1.66666666666666666667e-01);
    p = __builtin_fma(p, r, 0.5);
    p = __builtin_fma(p, r, 1.0);
    p = __builtin_fma(p, r, 1.0);
    return __builtin_ldexp(p, (int)n);
}

// ------------------------------------------------------------------------------------------------
// keys: (value desc, id asc) as one descending uint64
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ord32(float x) {
    x = x + 0.0f;  // -0 -> +0
    const uint32_t u = __float_as_uint(x);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord32(uint32_t o) {
    const uint32_t u = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
    return __uint_as_float(u);
}
__device__ __forceinline__ uint64_t make_key(float x, uint32_t j) {
    return ((uint64_t)ord32(x) << 32) | (uint64_t)(0xFFFFFFFFu - j);
}
__device__ __forceinline__ uint32_t key_id(uint64_t k) { return 0xFFFFFFFFu - (uint32_t)k; }
__device__ __forceinline__ float key_val(uint64_t k) { return unord32((uint32_t)(k >> 32)); }

// ------------------------------------------------------------------------------------------------
// wave helpers
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int popc64(uint64_t m) { return __popcll(m); }
__device__ __forceinline__ int lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ void lds_fence() { __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }


// DPP cross-lane steps (no LDS round trip, unlike ds_bpermute): row_shr:1,2,4,8 inside each 16-lane row,
// then row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) -- the wave64 inclusive scan of GFX9.  Lanes
// whose source is outside the row keep `old` (the identity).  Exact for integer add and for max.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v, uint32_t identity) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)identity, (int)v, CTRL, ROW_MASK, 0xF, false);
}
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
    v += dpp_u32<0x111, 0xF>(v, 0u);
    v += dpp_u32<0x112, 0xF>(v, 0u);
    v += dpp_u32<0x114, 0xF>(v, 0u);
    v += dpp_u32<0x118, 0xF>(v, 0u);
    v += dpp_u32<0x142, 0xA>(v, 0u);
    v += dpp_u32<0x143, 0xC>(v, 0u);
    return v;
}
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ int64_t dpp_add64(int64_t v) {
    const uint64_t u = (uint64_t)v;
    const uint32_t lo = dpp_u32<CTRL, ROW_MASK>((uint32_t)u, 0u);
    const uint32_t hi = dpp_u32<CTRL, ROW_MASK>((uint32_t)(u >> 32), 0u);
    return v + (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int64_t wave_incl_scan(int64_t v, int lane) {
    (void)lane;
    v = dpp_add64<0x111, 0xF>(v);
    v = dpp_add64<0x112, 0xF>(v);
    v = dpp_add64<0x114, 0xF>(v);
    v = dpp_add64<0x118, 0xF>(v);
    v = dpp_add64<0x142, 0xA>(v);
    v = dpp_add64<0x143, 0xC>(v);
    return v;
}
// value of lane (lane ^ OFF) without an LDS round trip: quad_perm for 1 and 2, row_shl/row_shr:4 selected by
// lane bit 2, row_ror:8, and the gfx950 v_permlane16/32_swap for 16 and 32 (they return {vdst', vsrc'}: the
// partner row sits in vsrc' for the lower row of each pair and in vdst' for the upper one)
template <int OFF>
__device__ __forceinline__ uint32_t xor_lane_u32(uint32_t v) {
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    if constexpr (OFF == 1) {
        return dpp_u32<0xB1, 0xF>(v, 0u);
    } else if constexpr (OFF == 2) {
        return dpp_u32<0x4E, 0xF>(v, 0u);
    } else if constexpr (OFF == 4) {
        const uint32_t up = dpp_u32<0x104, 0xF>(v, 0u), dn = dpp_u32<0x114, 0xF>(v, 0u);
        return (lane & 4u) ? dn : up;
    } else if constexpr (OFF == 8) {
        return dpp_u32<0x128, 0xF>(v, 0u);
    } else if constexpr (OFF == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (lane & 16u) ? r[0] : r[1];
    } else {
        static_assert(OFF == 32, "xor offsets 1..32");
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (lane & 32u) ? r[0] : r[1];
    }
}
template <int OFF>
__device__ __forceinline__ double xor_lane_f64(double v) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint64_t w = ((uint64_t)xor_lane_u32<OFF>((uint32_t)(u >> 32)) << 32) | xor_lane_u32<OFF>((uint32_t)u);
    return __builtin_bit_cast(double, w);
}
__device__ __forceinline__ double wave_sum_butterfly(double v) {
    // canonical xor butterfly 32,16,8,4,2,1 (commutative per pair => every lane ends identical)
    v = v + xor_lane_f64<32>(v);
    v = v + xor_lane_f64<16>(v);
    v = v + xor_lane_f64<8>(v);
    v = v + xor_lane_f64<4>(v);
    v = v + xor_lane_f64<2>(v);
    v = v + xor_lane_f64<1>(v);
    return v;
}
// ---- order-free kept mass E (canonical step 6, oracle or_kept_mass): e in [0,1] cut into four 36-bit limbs
// (truncated at 2^-120); limb sums are integers < 2^53, exact in float64 in ANY order, so no rank order is needed
struct Mass {
    double a, b, c, d;
};
__device__ __forceinline__ void mass_add(Mass& s, double e) {
    double t = e * 0x1p12;
    const double a = __builtin_floor(t);
    t = (t - a) * 0x1p36;
    const double b = __builtin_floor(t);
    t = (t - b) * 0x1p36;
    const double c = __builtin_floor(t);
    t = (t - c) * 0x1p36;
    s.a += a;
    s.b += b;
    s.c += c;
    s.d += __builtin_floor(t);
}
__device__ __forceinline__ void mass_wave_sum(Mass& s) {  // exact: every lane ends with the wave's sums
    s.a = wave_sum_butterfly(s.a);
    s.b = wave_sum_butterfly(s.b);
    s.c = wave_sum_butterfly(s.c);
    s.d = wave_sum_butterfly(s.d);
}
__device__ __forceinline__ double mass_value(Mass s) {  // normalise (carries), then the canonical roundings
    double q = __builtin_floor(s.d * 0x1p-36);
    s.d -= q * 0x1p36;
    s.c += q;
    q = __builtin_floor(s.c * 0x1p-36);
    s.c -= q * 0x1p36;
    s.b += q;
    q = __builtin_floor(s.b * 0x1p-36);
    s.b -= q * 0x1p36;
    s.a += q;
    double t = s.d * 0x1p-120;
    t = __builtin_fma(s.c, 0x1p-84, t);  // products by powers of two are exact: fma == mul + add here
    t = __builtin_fma(s.b, 0x1p-48, t);
    return __builtin_fma(s.a, 0x1p-12, t);
}

// value of lane `src` (wave-uniform) in every lane: two v_readlane, no LDS
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int src) {
    src = __builtin_amdgcn_readfirstlane(src);  // the callers' lane index is uniform (ballot-derived)
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, src);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ float wave_max(float v) {
    // max-scan with identity -inf, then lane 63 holds the wave max
    const uint32_t ninf = 0xFF800000u;
    auto step = [&](uint32_t o) { v = fmaxf(v, __uint_as_float(o)); };
    step(dpp_u32<0x111, 0xF>(__float_as_uint(v), ninf));
    step(dpp_u32<0x112, 0xF>(__float_as_uint(v), ninf));
    step(dpp_u32<0x114, 0xF>(__float_as_uint(v), ninf));
    step(dpp_u32<0x118, 0xF>(__float_as_uint(v), ninf));
    step(dpp_u32<0x142, 0xA>(__float_as_uint(v), ninf));
    step(dpp_u32<0x143, 0xC>(__float_as_uint(v), ninf));
    return __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(v), 63));
}

// ------------------------------------------------------------------------------------------------
// logit loads
// ------------------------------------------------------------------------------------------------
template <typename T>
struct Elem;
template <>
struct Elem<float> {
    static constexpr int W = 4;
    __device__ static __forceinline__ void unpack(const uint4& v, float (&x)[4]) {
        x[0] = __uint_as_float(v.x);
        x[1] = __uint_as_float(v.y);
        x[2] = __uint_as_float(v.z);
        x[3] = __uint_as_float(v.w);
    }
    __device__ static __forceinline__ float load1(const void* row, int j) { return ((const float*)row)[j]; }
};
template <>
struct Elem<_Float16> {
    static constexpr int W = 8;
    __device__ static __forceinline__ float h2f(uint32_t bits16) {
        const uint16_t b = (uint16_t)bits16;
        _Float16 h;
        __builtin_memcpy(&h, &b, 2);
        return (float)h;
    }
    __device__ static __forceinline__ void unpack(const uint4& v, float (&x)[8]) {
        x[0] = h2f(v.x & 0xFFFFu);
        x[1] = h2f(v.x >> 16);
        x[2] = h2f(v.y & 0xFFFFu);
        x[3] = h2f(v.y >> 16);
        x[4] = h2f(v.z & 0xFFFFu);
        x[5] = h2f(v.z >> 16);
        x[6] = h2f(v.w & 0xFFFFu);
        x[7] = h2f(v.w >> 16);
    }
    __device__ static __forceinline__ float load1(const void* row, int j) {
        return h2f(((const uint16_t*)row)[j]);
    }
};

// ------------------------------------------------------------------------------------------------
// step parameters (kernel argument, by value)
// ------------------------------------------------------------------------------------------------
struct StepParams {
    const void* logits;
    int64_t ld;
    int B, V, P, topk, K;  // K = min(topk, #valid ids)
    double inv_temp;
    float c32;  // (float)(inv_temp * log2(e))
    int nbanned;
    int banned[NS_MAX_BANNED];  // sorted ascending, unique, in [0, V)
    int spec_j;  // speculative threshold rank in the 4096-id sample (0: no sample)
    uint32_t flags;
    // encode
    const uint8_t* payload;
    int64_t payload_stride;
    const int64_t* nbits;
    int32_t* out_token;
    int32_t* hist;
    int64_t hist_stride;
    // decode
    const int32_t* in_token;
    const uint8_t* is_last;
    const uint8_t* active;
    uint8_t* out_bits;
    int64_t out_stride;
    // sampler (ns_sample_step): code_base/sample.py token loop
    int sample;              // 1: sampler step (no interval, no payload)
    uint64_t seed;           // counter-based draw: rand64(seed, stream_offset + b, ntokens)
    int64_t stream_offset;
    // statistics sink [B][4]: sum log p(sel), sum KL bits, sum entropy bits, steps (nullable)
    double* stats;
    // decode: ranked ids of a diverged stream (ranks < k', then -1), [B][ranked_stride] (nullable)
    int32_t* ranked;
    int ranked_stride;
    // src rank coder (ns_rank_encode_step / ns_rank_decode_step)
    int rank;                 // 1: rank-coder step on the wide path
    int rk_top_k, rk_cap;     // <= 0: off
    double rk_top_p;          // <= 0: off
    double rk_min_prob;       // < 0: off
    double rk_ptemp;          // crypto quality LM: temperature on the probabilities (<= 0: off)
    int32_t* rk_cons;         // encode: bits consumed per token, [B][hist_stride]
    const int32_t* rk_keep;   // decode: bits to keep this step, [B]
    int rk_crypto;            // crypto quality policy active (prob_temp > 0 given, isclose or not)
    const int32_t* rk_count;  // f64 provider rows: entries per row [B] (nullable: V)
    const int32_t* rk_idmap;  // f64 provider rows: token id per entry [B][rk_idmap_stride] (nullable: position)
    int64_t rk_idmap_stride;
    int rk_dict;              // f64 provider rows are dict ProbDists
    double* probs_out;        // ns_token_probs: filtered, renormalised p by id, [B][probs_stride]
    int64_t probs_stride;
    uint64_t* stamps;         // NSG_STAMPS diagnostic builds: s_memtime at phase boundaries, [B][16]
    // common
    ns_stream_state* state;
    ns_step_trace* trace;
    unsigned long long* counters;
};

// In-kernel phase stamps (diagnostic builds only: -DNSG_STAMPS=1, tools/stamp_phases.py)
#ifdef NSG_STAMPS
__device__ __forceinline__ uint64_t nsg_memtime() {
    uint64_t t;
    __asm__ volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ __forceinline__ uint64_t nsg_realtime() {
    uint64_t t;
    __asm__ volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
#define NSG_STAMP_RT(p, b, lane, k)                                                                   \
    do {                                                                                              \
        const uint64_t _t = nsg_realtime();                                                           \
        if ((p).stamps && (lane) == 0) (p).stamps[(int64_t)(b) * 16 + (k)] = _t;                     \
    } while (0)
#define NSG_STAMP(p, b, lane, k)                                                                      \
    do {                                                                                              \
        const uint64_t _t = nsg_memtime();                                                            \
        if ((p).stamps && (lane) == 0) (p).stamps[(int64_t)(b) * 16 + (k)] = _t;                     \
    } while (0)
#else
#define NSG_STAMP(p, b, lane, k) ((void)0)
#define NSG_STAMP_RT(p, b, lane, k) ((void)0)
#endif

// counter-based 64-bit draw, identical to or_rand64 (oracle/nsg_oracle.c): splitmix64 finaliser
__device__ __forceinline__ uint64_t rand64(uint64_t seed, int64_t gid, int64_t t) {
    uint64_t z = seed ^ ((uint64_t)gid * 0xD1B54A32D192ED03ull);
    z += (uint64_t)(t + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

constexpr float L2E_F = 1.44269504088896341f;   // log2(e), fp32 (untempered fast exps of the statistics)
constexpr double SAMPLE_SUPPORT = 0x1p-60;       // sampler support: e_i >= 2^-60 (oracle step S2)
constexpr double SAMPLE_SCALE = 0x1p48;          // sampler CDF resolution (oracle step S4)

// Fast statistics of one row relative to its max m (tolerance-checked, not part of the bit contract):
// lse1 = ln sum exp(x - m) (untempered), lst = ln sum exp((x - m)/T), a_over_s = sum p_T (x - m)/T.
struct RowStats {
    double lse1, lst, a_over_s;
};

// From the streaming accumulators taken against the reference r: S_r = sum 2^((x-r)c32), B_r = sum
// 2^((x-r)c32) (x-r), U_r = sum 2^((x-r) log2 e).  Returns false when they are unusable (overflow).
__device__ __forceinline__ bool row_stats_from_stream(double S_r, double B_r, double U_r, float r, double m,
                                                      double inv_temp, RowStats& rs) {
    if (!(S_r > 0.0 && S_r < 1.0e300 && U_r > 0.0 && U_r < 1.0e300 && B_r > -1.0e300 && B_r < 1.0e300))
        return false;
    const double rm = (double)r - m;
    rs.lse1 = log(U_r) + rm;
    rs.lst = log(S_r) + rm * inv_temp;
    rs.a_over_s = inv_temp * (B_r / S_r + rm);
    return true;
}

__device__ __forceinline__ bool is_banned(const StepParams& p, int j) {
    bool b = false;
#pragma unroll
    for (int i = 0; i < NS_MAX_BANNED; ++i) b |= (i < p.nbanned) && (p.banned[i] == j);
    return b;
}

// exact canonical row sum (oracle or_row_sum): id j -> lane (j>>2)&63, per-lane increasing, butterfly
template <typename T>
__device__ __forceinline__ double exact_row_sum(const StepParams& p, const void* row, double m, int lane) {
    double acc = 0.0;
    const int ngroups = (p.V + 3) >> 2;
    for (int g = lane; g < ngroups; g += WAVE) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int j = 4 * g + q;
            if (j < p.V && !is_banned(p, j)) {
                const float x = Elem<T>::load1(row, j) + 0.0f;
                acc += exp_canon(((double)x - m) * p.inv_temp);
            }
        }
    }
    return wave_sum_butterfly(acc);
}

// Statistics fallback (streaming accumulators unusable): re-read the row, float64 exps against the true max.
// Inlined (round 5): as a call it made the statistics builds of the coder keep a stack frame and spill around it
// -- 4.9 KB of scratch per lane in the fp16 one-wave form, 1.10 ms per step at B = 4,096 against 0.19 inlined.
template <typename T>
__device__ __forceinline__ RowStats wave_row_stats(const StepParams& p, const void* row, double m, int lane) {
    double s1 = 0.0, st = 0.0, at = 0.0;
    for (int j = lane; j < p.V; j += WAVE) {
        if (is_banned(p, j)) continue;
        const double d = (double)(Elem<T>::load1(row, j) + 0.0f) - m;
        const double et = exp(d * p.inv_temp);
        s1 += exp(d);
        st += et;
        at += et * (d * p.inv_temp);
    }
    s1 = wave_sum_butterfly(s1);
    st = wave_sum_butterfly(st);
    at = wave_sum_butterfly(at);
    RowStats rs;
    rs.lse1 = log(s1);
    rs.lst = log(st);
    rs.a_over_s = at / st;
    return rs;
}

__device__ __forceinline__ const void* uniform_ptr(const void* ptr) {
    const uint64_t a = (uint64_t)ptr;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return (const void*)(((uint64_t)hi << 32) | lo);
}

struct RowReader {
    __amdgpu_buffer_rsrc_t rs;
    __device__ __forceinline__ RowReader(const void* base, uint32_t bytes)
        : rs(__builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(uniform_ptr(base)), (short)0,
                                               (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000)) {}
    __device__ __forceinline__ uint4 vec(int v) const {
        const auto r = __builtin_amdgcn_raw_buffer_load_b128(rs, v * 16, 0, NSG_LOAD_AUX);
        return make_uint4(r[0], r[1], r[2], r[3]);
    }
    // default cache policy: bytes the same workgroup reads again soon (kept in L2 / the Infinity Cache)
    __device__ __forceinline__ uint4 vec_keep(int v) const {
        const auto r = __builtin_amdgcn_raw_buffer_load_b128(rs, v * 16, 0, 0);
        return make_uint4(r[0], r[1], r[2], r[3]);
    }
};

// Proven interval of the canonical float64 row sum S from the fast estimate S_r = sum 2^((x-r)*c32)
// accumulated in fp32 groups of at most `fp32_terms` terms.  Returns false when the
// bound is unusable (overflow/underflow of the estimate, reference too far from the max).
__device__ __forceinline__ bool fast_sum_interval(double S_r, float r, double m, float c32, double inv_temp,
                                                  int fp32_terms, double& Sf, double& S_lo, double& S_hi) {
    const double t_m = (m - (double)r) * (double)c32;
    if (!(S_r > 0.0 && S_r < 1.0e300) || !(t_m <= 100.0 && t_m >= -60.0)) return false;
    const double f = exp_canon(((double)r - m) * inv_temp);
    Sf = S_r * f;
    const double u24 = 5.9604644775390625e-08;  // 2^-24
    const double eb = 9.5367431640625e-07         // v_exp_f32 error (2^-20, generous)
                      + 3.0 * u24 * 0.6931471805599453 * (60.0 + fabs(t_m))  // argument rounding
                      + (double)(fp32_terms + 1) * u24                          // fp32 partials
                      + 1.0e-13;
    const double B2 = 2.0 * eb + 1.0e-12;
    S_lo = Sf * (1.0 - B2);
    S_hi = Sf * (1.0 + B2);
    return true;
}

// The same interval with a data-dependent argument term (round 3, the one-pass wide kernel).  The terms are
// e_i = 2^t_i with t_i = fl(x_i * c32 - fl(r * c32)) (one fma).  Against the exact t*_i = (x_i - r) * log2(e)/T:
// t_i = t*_i (1 + d_c) (1 + d_f) + D, where d_c is c32's rounding (<= u), d_f the fma's (<= u) and
// D = r*c32 - fl(r*c32) the rounding of the reference's product -- the SAME for every term, and exactly known
// (computed in double), so the sum is corrected by 2^-D.  What remains is a relative error of
// ln2 * 2u * |t_i| per term: summed with the terms as weights, 2u ln2 * A_r / S_r with A_r = sum e_i |t_i|.
// The kernel accumulates the signed B_t = sum e_i t_i (packed fmas; no abs in packed form), and
// A_r = -B_t + 2 sum_{t_i >= 0} e_i t_i <= -B_t + 2 max(t_m, 0) S_r  (t_m = the largest argument).
// A_r / S_r is the e-weighted mean |argument|, a few units for real rows, where the worst-case form above charges
// every term with 60 + |t_m|: about ten times narrower, so far fewer steps need the exact row sum.  Terms below
// 2^-200 of the largest add less than V * 2^-200 relative (the constant term).
__device__ __forceinline__ bool fast_sum_interval_dd(double S_r, double B_t, float r, double m, float c32,
                                                     double inv_temp, int fp32_terms, double& Sf, double& S_lo,
                                                     double& S_hi) {
    const double t_m = (m - (double)r) * (double)c32;
    if (!(S_r > 0.0 && S_r < 1.0e300) || !(B_t > -1.0e300 && B_t < 1.0e300) || !(t_m <= 100.0 && t_m >= -60.0))
        return false;
    const double rc = (double)r * (double)c32;                 // exact (float x float fits a double)
    const double D = rc - (double)(float)rc;                   // exact: the reference product's rounding
    const double S_c = S_r * exp_canon(-D * 0.6931471805599453);  // 2^-D
    const double A = fmax(0.0, -B_t) + 2.0 * fmax(t_m + 1.0e-6, 0.0) * S_r;
    const double f = exp_canon(((double)r - m) * inv_temp);
    Sf = S_c * f;
    const double u24 = 5.9604644775390625e-08;  // 2^-24
    const double eb = 9.5367431640625e-07                                // v_exp_f32 error (2^-20, generous)
                      + 2.0 * u24 * 0.6931471805599453 * 1.01 * (A / S_r)  // argument rounding, e-weighted
                      + (double)(fp32_terms + 1) * u24                     // fp32 partials
                      + 1.0e-13;
    const double B2 = 2.0 * eb + 1.0e-12;
    S_lo = Sf * (1.0 - B2);
    S_hi = Sf * (1.0 + B2);
    return true;
}

}  // namespace nsg

// Decode-step attention of the batched GPT-2 forward with the KV append fused in (include/nsg_attn.h).
//
// Reference semantics: Hugging Face GPT2Attention for one new token per stream over the unbounded cache the
// reference keeps (code_base/arithmetic.py:115-122): softmax(q k^T / sqrt(D)) v over positions 0..L0.
//
// Layout: a pair's rows are split over S = 1, 2, 4 or 8 waves by the KEY COUNT alone (att_split), so the
// summation order -- and every output bit -- is the same whatever the batch size; the S partials are merged in
// wave order through LDS.  Lane l holds dims 8*(l&7)..+7 of key row (l>>3) of an 8-row
// chunk, so an 8-lane group reads one 128-byte K (and V) row and the wave reads 1 KiB of contiguous cache per
// 16-byte load instruction.  Scores are reduced inside the 8-lane group; each group keeps its own online
// softmax (running max, sum, 8 accumulator dims) over the rows it saw, and the 8 groups are merged once at the
// end.  fp16 q.k products with fp32 accumulation (v_dot2_f32_f16), exp2 with log2(e) folded into the scale.
// HBM-bound: 2*(L0+1)*128 bytes per (stream, head) read once, non-temporal (the rows are not reused within
// the step).  The new token's k/v come from the qkv registers and are written to the cache by group 0.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "nsg_attn.h"
#include "nsg_coder.h"

namespace nsg {

#ifndef NSG_ATT_ROWS1
#define NSG_ATT_ROWS1 256  // keys per pair up to which one wave takes the whole pair (then 2, 4, 8 waves)
#endif
#ifndef NSG_ATT_HEAD_MAJOR
#define NSG_ATT_HEAD_MAJOR 1  // large batches: a workgroup's 8 pairs are 8 streams of ONE head (shared context rows
                              // then come from the CU's cache), not 8 consecutive (stream, head) pairs; round 5:
                              // 0.2-1.3 % faster at L = 300-1,000 (profiles/r05/attn_head_major_ab/)
#endif
#ifndef NSG_ATT_SMALL_PAIRS
#define NSG_ATT_SMALL_PAIRS 1024  // up to this many (stream, head) pairs: one pair per workgroup
#endif

constexpr int ATT_D = 64;

#ifndef NSG_ATT_LOAD
#define NSG_ATT_LOAD 0  // K/V row loads: 0 = non-temporal (the rows are not reused within the step), 1 = default policy
#endif

template <class R>
__device__ __forceinline__ R att_load(const R* p) {
#if NSG_ATT_LOAD == 1
    return *p;
#else
    return __builtin_nontemporal_load(p);
#endif
}


typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float dot8(f16x8 a, f16x8 b) {
    float s = 0.0f;
    s = __builtin_amdgcn_fdot2(__builtin_shufflevector(a, a, 0, 1), __builtin_shufflevector(b, b, 0, 1), s, false);
    s = __builtin_amdgcn_fdot2(__builtin_shufflevector(a, a, 2, 3), __builtin_shufflevector(b, b, 2, 3), s, false);
    s = __builtin_amdgcn_fdot2(__builtin_shufflevector(a, a, 4, 5), __builtin_shufflevector(b, b, 4, 5), s, false);
    s = __builtin_amdgcn_fdot2(__builtin_shufflevector(a, a, 6, 7), __builtin_shufflevector(b, b, 6, 7), s, false);
    return s;
}

__device__ __forceinline__ void unpack8(f16x8 v, float* f) {
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = (float)v[i];
}

// Split of one (stream, head) pair's rows over waves, a function of the key count ONLY (never of the batch):
// S waves take the 32-row chunks w, w + S, ... and their online-softmax partials are merged in wave order.
// Short caches keep one wave per pair (a short row list split eight ways is mostly idle waves); long caches
// use eight, so a lone stream still spreads its rows over a CU.
__device__ __forceinline__ int att_split(int Lk) {
    return Lk <= NSG_ATT_ROWS1 ? 1 : Lk <= 2 * NSG_ATT_ROWS1 ? 2 : Lk <= 4 * NSG_ATT_ROWS1 ? 4 : 8;
}

// K/V storage formats.  A lane holds DPL consecutive dims of one key row, LPR lanes a row, RPI rows per 16-byte
// wave-load, NI wave-loads per 32-row chunk.  The fp16 format is the reference configuration; the fp8 one
// (OCP e4m3fn, saturated to +-448, round to nearest even; opt-in) halves the cache bytes the HBM-bound decode
// reads.  q stays fp16 either way; scores and the softmax run in fp32.
struct FmtF16 {
    static constexpr int DPL = 8, LPR = 8, RPI = 8, NI = 4;
    typedef _Float16 Elem;
    typedef f16x8 Raw;
    struct Q {
        f16x8 v;
    };
    static __device__ __forceinline__ Q load_q(const _Float16* p) { return Q{*(const f16x8*)p}; }
    static __device__ __forceinline__ Raw from_qkv(const _Float16* p) { return *(const f16x8*)p; }
    static __device__ __forceinline__ float dot(const Q& q, Raw k) { return dot8(q.v, k); }
    static __device__ __forceinline__ void unpack(Raw v, float* f) { unpack8(v, f); }
};

__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d) {
    // saturate first: the conversion itself does not clamp, and e4m3fn has no infinity
    a = fminf(fmaxf(a, -448.0f), 448.0f);
    b = fminf(fmaxf(b, -448.0f), 448.0f);
    c = fminf(fmaxf(c, -448.0f), 448.0f);
    d = fminf(fmaxf(d, -448.0f), 448.0f);
    int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
    return (uint32_t)w;
}

#ifndef NSG_ATT_DB8
#define NSG_ATT_DB8 0  // 1: fp8 pages keep the register double buffer in multi-pair workgroups too (A/B)
#endif
#ifndef NSG_ATT_DB8_WPE
#define NSG_ATT_DB8_WPE 3  // ... at this many waves per SIMD
#endif
#ifndef NSG_ATT_F8_NI
#define NSG_ATT_F8_NI 2  // 16-row wave-loads per fp8 chunk
#endif

struct FmtF8 {
    static constexpr int DPL = 16, LPR = 4, RPI = 16, NI = NSG_ATT_F8_NI;
    typedef uint8_t Elem;
    typedef u32x4 Raw;
    struct Q {
        f16x8 a, b;  // the lane's 16 query dims, fp16
    };
    static __device__ __forceinline__ Q load_q(const _Float16* p) {
        return Q{*(const f16x8*)p, *(const f16x8*)(p + 8)};
    }
    static __device__ __forceinline__ Raw from_qkv(const _Float16* p) {  // the new token's k or v, quantised
        const f16x8 a = *(const f16x8*)p, b = *(const f16x8*)(p + 8);
        Raw r;
        r[0] = pack4_fp8((float)a[0], (float)a[1], (float)a[2], (float)a[3]);
        r[1] = pack4_fp8((float)a[4], (float)a[5], (float)a[6], (float)a[7]);
        r[2] = pack4_fp8((float)b[0], (float)b[1], (float)b[2], (float)b[3]);
        r[3] = pack4_fp8((float)b[4], (float)b[5], (float)b[6], (float)b[7]);
        return r;
    }
    // v (fp8, exact in f32) for the PV accumulation: one v_cvt_pk_f32_fp8 per 2 values
    static __device__ __forceinline__ void unpack(Raw v, float* f) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const auto lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)v[i], false);
            const auto hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)v[i], true);
            f[4 * i + 0] = lo[0];
            f[4 * i + 1] = lo[1];
            f[4 * i + 2] = hi[0];
            f[4 * i + 3] = hi[1];
        }
    }
    // q.k: every e4m3 value is exact in fp16, so k goes fp8 -> fp16 pairs (v_cvt_scalef32_pk_f16_fp8, scale 1) and
    // the products run on v_dot2c_f32_f16 like the fp16 cache's, two dims per instruction
    static __device__ __forceinline__ float dot(const Q& q, Raw k) {
        const f16x2 qp[8] = {__builtin_shufflevector(q.a, q.a, 0, 1), __builtin_shufflevector(q.a, q.a, 2, 3),
                             __builtin_shufflevector(q.a, q.a, 4, 5), __builtin_shufflevector(q.a, q.a, 6, 7),
                             __builtin_shufflevector(q.b, q.b, 0, 1), __builtin_shufflevector(q.b, q.b, 2, 3),
                             __builtin_shufflevector(q.b, q.b, 4, 5), __builtin_shufflevector(q.b, q.b, 6, 7)};
        float s = 0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const f16x2 lo = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8((int)k[i], 1.0f, false);
            const f16x2 hi = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8((int)k[i], 1.0f, true);
            s = __builtin_amdgcn_fdot2(lo, qp[2 * i], s, false);
            s = __builtin_amdgcn_fdot2(hi, qp[2 * i + 1], s, false);
        }
        return s;
    }
};

// Workgroup = 8 waves serving P consecutive pairs (P = 1 for small batches, 8 otherwise; P changes only which
// workgroup computes a pair, not how).  With S = att_split(L0 + 1), the waves form 8/S groups of S; group
// q takes pairs q, q + 8/S, ... of the workgroup, one round per pair, all waves running the same number of
// rounds so the LDS merge's barriers are uniform.
// Positions [0, T0) come from a prefix shared by every stream (kp/vp, head stride ph: the common context,
// stored once), positions [T0, L0] from the stream's own cache at index position - T0.  Same values, same
// order: the output bits do not depend on where a row is stored.
// Which (stream, head) pair slot j of workgroup g serves (-1: none).  Work placement only: the math of a pair does
// not depend on it.
template <int P>
__device__ __forceinline__ int att_pair(int g, int j, int B, int H) {
    if (P > 1 && NSG_ATT_HEAD_MAJOR) {
        const int h = g % H, b = (g / H) * P + j;
        return b < B ? b * H + h : -1;
    }
    const int pair = g * P + j;
    return pair < B * H ? pair : -1;
}

template <class F, int P>
__global__ __launch_bounds__(512) void decode_attn_kernel(const _Float16* __restrict__ qkv, int64_t qkv_stride,
                                                          typename F::Elem* kc, typename F::Elem* vc, int64_t cb,
                                                          int64_t ch, int64_t cz, const typename F::Elem* __restrict__ kp,
                                                          const typename F::Elem* __restrict__ vp, int64_t ph, int T0,
                                                          int B, int H, int L0, const int32_t* __restrict__ L0p,
                                                          int cap, int window,
                                                          const uint32_t* __restrict__ done, int64_t done_stride,
                                                          const int32_t* __restrict__ stop,
                                                          _Float16* __restrict__ out, int64_t out_stride,
                                                          float scale_log2) {
    typedef typename F::Elem E;
    typedef typename F::Raw Raw;
    constexpr int DPL = F::DPL, LPR = F::LPR, RPI = F::RPI, NI = F::NI;
    if (L0p) L0 = __builtin_amdgcn_readfirstlane(*L0p);  // graph replays: the cache length lives on the device
    if (L0 < T0 || L0 >= cap) {  // never write past the cache (the host checks capacity); with a device-side L0
        // the host cannot see an overflow before the launch, so poison this workgroup's output rows: the NaNs
        // reach the logits and the coder rejects them, instead of the next GEMM reusing stale rows
        for (int i = threadIdx.x; i < P * ATT_D; i += blockDim.x) {
            const int pair = att_pair<P>(blockIdx.x, i / ATT_D, B, H);
            if (pair >= 0)
                out[(int64_t)(pair / H) * out_stride + (pair % H) * ATT_D + i % ATT_D] = (_Float16)__builtin_nanf("");
        }
        return;
    }
    __shared__ float s_m[8], s_l[8];
    __shared__ float s_acc[8][ATT_D];
    const int Lk = L0 + 1;
    // attention window (opt-in, 0 = the reference's unbounded cache): keys [s0, L0], s0 = max(0, L0 + 1 - window)
    const int s0 = window > 0 ? max(0, Lk - window) : 0;
    const int S = att_split(Lk - s0);
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int grp = wave / S, wv = wave - grp * S, ngrp = 8 / S;
    const int g = lane / LPR;  // row within an RPI-row slab
    const int c = lane % LPR;  // DPL-dim slice
    const int C = H * ATT_D;
    const int last_cached = L0 > 0 ? L0 - 1 : 0;
    const int rounds = (P + ngrp - 1) / ngrp;
    for (int rd = 0; rd < rounds; ++rd) {
        const int j = grp + rd * ngrp;
        const int pair = j < P ? att_pair<P>(blockIdx.x, j, B, H) : -1;
        // uniform per wave group; a finished stream (done flag bit 0, e.g. the coder state's NS_ST_DONE, or a cache
        // length at its stop position) is skipped: no KV append, no cache read, its output row keeps its old (finite)
        // values, which nothing uses again
        const int sb = pair / H;
        const bool active = pair >= 0 && !(done && (done[(int64_t)sb * done_stride] & 1u)) &&
                            !(stop && L0 >= stop[sb]);
        float m = -1e30f, l = 0.0f;
        float acc[DPL];
#pragma unroll
        for (int d = 0; d < DPL; ++d) acc[d] = 0.0f;
        int b = 0, h = 0;
        if (active) {
            b = pair / H;
            h = pair - b * H;
            const _Float16* qrow = qkv + (int64_t)b * qkv_stride + h * ATT_D + c * DPL;
            const typename F::Q q = F::load_q(qrow);
            const Raw knew = F::from_qkv(qrow + C);
            const Raw vnew = F::from_qkv(qrow + 2 * C);
            // stream rows are addressed by position (index position - T0 folded into the base)
            // stream row j (position T0 + j) at (j / 32) * cz + (j % 32) * D: rows grouped in 32-row chunks, the
            // chunks of all (stream, head) pairs at one position range side by side (cz = chunk plane stride;
            // cz = 32 * D is the plain row-contiguous layout)
            E* kb = kc + (int64_t)b * cb + (int64_t)h * ch + c * DPL;
            E* vb = vc + (int64_t)b * cb + (int64_t)h * ch + c * DPL;
            auto soff = [&](int row) -> int64_t {
                const int jj = row - T0;
                return (int64_t)(jj >> 5) * cz + (int64_t)(jj & 31) * ATT_D;
            };
            const E* kpb = kp + (int64_t)h * ph + c * DPL;
            const E* vpb = vp + (int64_t)h * ph + c * DPL;
            if (g == 0 && wv == 0) {  // KV append of the new token (position L0)
                *(Raw*)(kb + soff(L0)) = knew;
                *(Raw*)(vb + soff(L0)) = vnew;
            }
            // one chunk of RPI*NI rows; GENERAL handles the prefix boundary, the clamp past the cache, rows past
            // Lk and the new token from registers -- an interior chunk (all rows stream rows < L0) skips those
            // selects (same operations on the same values: the bits do not depend on the path).  Small batches
            // (P = 1) issue the next chunk's loads before this chunk's math (register double buffer): a wave's
            // chunks are otherwise one dependent memory round trip each, which is what a lone stream waits on.
            auto load_chunk = [&](int j0, auto general, Raw (&kr)[NI], Raw (&vr)[NI]) {
                constexpr bool GEN = decltype(general)::value;
#pragma unroll
                for (int u = 0; u < NI; ++u) {
                    if constexpr (GEN) {
                        const int row = min(j0 + RPI * u + g, last_cached);
                        const bool pre = row < T0;
                        const E* ka = pre ? kpb + (int64_t)row * ATT_D : kb + soff(row);
                        const E* va = pre ? vpb + (int64_t)row * ATT_D : vb + soff(row);
                        kr[u] = att_load((const Raw*)ka);
                        vr[u] = att_load((const Raw*)va);
                    } else {
                        const int row = j0 + RPI * u + g;
                        const int64_t o = soff(row);
                        kr[u] = att_load((const Raw*)(kb + o));
                        vr[u] = att_load((const Raw*)(vb + o));
                    }
                }
            };
            auto math_chunk = [&](int j0, auto general, Raw (&kr)[NI], Raw (&vr)[NI]) {
                constexpr bool GEN = decltype(general)::value;
                float sc[NI];
                bool valid[NI];
                float mx = m;
#pragma unroll
                for (int u = 0; u < NI; ++u) {
                    const int row = j0 + RPI * u + g;
                    valid[u] = GEN ? row < Lk : true;
                    if (GEN && row == L0) {  // the new token: from registers, not from the cache just written
                        kr[u] = knew;
                        vr[u] = vnew;
                    }
                    float sv = F::dot(q, kr[u]);
#pragma unroll
                    for (int off = 1; off < LPR; off <<= 1) sv += __shfl_xor(sv, off);
                    sc[u] = sv * scale_log2;
                    if (valid[u]) mx = fmaxf(mx, sc[u]);
                }
                const float alpha = exp2f(m - mx);
                l *= alpha;
#pragma unroll
                for (int d = 0; d < DPL; ++d) acc[d] *= alpha;
#pragma unroll
                for (int u = 0; u < NI; ++u) {
                    const float p = valid[u] ? exp2f(sc[u] - mx) : 0.0f;
                    l += p;
                    float v[DPL];
                    F::unpack(vr[u], v);
#pragma unroll
                    for (int d = 0; d < DPL; ++d) acc[d] = fmaf(p, v[d], acc[d]);
                }
                m = mx;
            };
            auto interior = [&](int j0) { return j0 >= T0 && j0 + RPI * NI <= L0; };  // wave-uniform
            const int step = S * RPI * NI;
            Raw kr[NI], vr[NI];
            int j0 = s0 + wv * RPI * NI;
            if constexpr (P > 1) {  // large batches: other waves hide the latency; no second register buffer
                for (; j0 < Lk; j0 += step) {
                    if (interior(j0)) {
                        load_chunk(j0, std::false_type{}, kr, vr);
                        math_chunk(j0, std::false_type{}, kr, vr);
                    } else {
                        load_chunk(j0, std::true_type{}, kr, vr);
                        math_chunk(j0, std::true_type{}, kr, vr);
                    }
                }
            } else {
            Raw kn[NI], vn[NI];
            if (j0 < Lk) {
                if (interior(j0))
                    load_chunk(j0, std::false_type{}, kr, vr);
                else
                    load_chunk(j0, std::true_type{}, kr, vr);
            }
            for (; j0 < Lk; j0 += step) {
                const int j1 = j0 + step;
                if (j1 < Lk) {
                    if (interior(j1))
                        load_chunk(j1, std::false_type{}, kn, vn);
                    else
                        load_chunk(j1, std::true_type{}, kn, vn);
                }
                if (interior(j0))
                    math_chunk(j0, std::false_type{}, kr, vr);
                else
                    math_chunk(j0, std::true_type{}, kr, vr);
#pragma unroll
                for (int u = 0; u < NI; ++u) {
                    kr[u] = kn[u];
                    vr[u] = vn[u];
                }
            }
            }
            // merge the row groups (lanes c, c + LPR, ... hold the same dims)
#pragma unroll
            for (int off = LPR; off < 64; off <<= 1) {
                const float mo = __shfl_xor(m, off);
                const float lo = __shfl_xor(l, off);
                const float mn = fmaxf(m, mo);
                const float fa = exp2f(m - mn), fo = exp2f(mo - mn);
                l = l * fa + lo * fo;
#pragma unroll
                for (int d = 0; d < DPL; ++d) {
                    const float ao = __shfl_xor(acc[d], off);
                    acc[d] = acc[d] * fa + ao * fo;
                }
                m = mn;
            }
        }
        if (S > 1) {  // uniform over the workgroup: hand the S partials of each group to its first wave
            if (active && g == 0) {
#pragma unroll
                for (int d = 0; d < DPL; ++d) s_acc[wave][c * DPL + d] = acc[d];
                if (c == 0) {
                    s_m[wave] = m;
                    s_l[wave] = l;
                }
            }
            __syncthreads();
            if (active && wv == 0) {
                const int w0 = grp * S;
                float mt = s_m[w0];
                for (int w = 1; w < S; ++w) mt = fmaxf(mt, s_m[w0 + w]);
                l = 0.0f;
#pragma unroll
                for (int d = 0; d < DPL; ++d) acc[d] = 0.0f;
                for (int w = 0; w < S; ++w) {
                    const float f = exp2f(s_m[w0 + w] - mt);
                    l += s_l[w0 + w] * f;
#pragma unroll
                    for (int d = 0; d < DPL; ++d) acc[d] += s_acc[w0 + w][c * DPL + d] * f;
                }
            }
            __syncthreads();  // the LDS slots are reused by the next round
        }
        if (active && wv == 0 && g == 0) {
            const float inv = 1.0f / l;
#pragma unroll
            for (int h8 = 0; h8 < DPL / 8; ++h8) {
                f16x8 o;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    float t = acc[h8 * 8 + i] * inv;
                    asm volatile("" : "+v"(t));  // no fused multiply-convert (one rounding) in some variants only
                    o[i] = (_Float16)t;
                }
                *(f16x8*)(out + (int64_t)b * out_stride + h * ATT_D + c * DPL + h8 * 8) = o;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------------- paged KV
// The same attention over a PAGED cache with a cache length PER STREAM (include/nsg_attn.h,
// ns_decode_attention_paged).  A stream's rows live in 32-position pages it owns: d_table[b][c] is the device
// address of the page holding stream rows 32c..32c+31 (positions T0 + 32c ...), a page laid out [layer][K|V][H][32]
// [D], so growth only maps new pages (no copy, no second cache) and a finished stream's pages go to the next message
// (slot refill, reference: every message runs its own loop with its own cache, code_base/arithmetic.py:96-122).
//
// With per-stream lengths the row split S of a pair (att_split of its own key count) differs inside a workgroup, so
// the work is cut into TASKS: task (pair j, split w) streams rows s0 + 32w, s0 + 32(w + S), ... exactly as wave w of
// the lockstep kernel does, the 8 waves take the tasks round-robin, every task's partial goes to LDS, and wave j then
// merges pair j's S partials in split order with the lockstep kernel's arithmetic (an S = 1 "merge" is exact: *1,
// +0).  Same rows, same order, same operations: the output bits equal the lockstep kernel's for the same cache
// contents, and still depend on a pair's own key count only (batch-invariant).
struct PagedArgs {
    const _Float16* qkv;
    int64_t qkv_stride;
    const uint64_t* table;  // [B][tstride] page addresses (bytes), 0 = no page
    int64_t tstride;
    int max_chunks;         // table entries per stream in use
    int64_t layer_off;      // elements from a page's base to this layer's K block ([layer][K|V][H][32][D])
    int64_t v_off;          // elements from the K block to the V block (H * 32 * D)
    const void* kp;         // shared prefix [H][ph] (positions < T0), fp16 or fp8 like the pages
    const void* vp;
    int64_t ph;
    int T0, B, H;
    const int32_t* lens;    // [B] positions already cached per stream (the new token goes to position lens[b])
    int window;
    const uint32_t* done;
    int64_t done_stride;
    const int32_t* stop;
    _Float16* out;
    int64_t out_stride;
    float scale_log2;
};

#ifndef NSG_ATT_DPP
#define NSG_ATT_DPP 1  // paged kernel: the score sums over a row's LPR lanes and the lane ^ 8 step of the final
                       // row-group merge by DPP moves instead of ds_bpermute
#endif

// x + (x of lane l ^ 1), then + (lane ^ 2), then (LPR = 8) + the other quad's sum -- the xor butterfly's values in
// its order (the third step reads lane 7 - l, whose quad sum equals lane l ^ 4's), as VALU DPP moves instead of
// LDS permutes: the same bits as __shfl_xor's butterfly
template <int LPR>
__device__ __forceinline__ float row_group_sum(float x) {
    static_assert(LPR == 4 || LPR == 8, "rows of 4 or 8 lanes");
    auto dpp = [](float v, auto ctrl) {
        return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                                     decltype(ctrl)::value, 0xF, 0xF, false));
    };
    x += dpp(x, std::integral_constant<int, 0xB1>{});  // quad_perm [1,0,3,2]: lane ^ 1
    x += dpp(x, std::integral_constant<int, 0x4E>{});  // quad_perm [2,3,0,1]: lane ^ 2
    if constexpr (LPR == 8) x += dpp(x, std::integral_constant<int, 0x141>{});  // row_half_mirror: lane 7 - l
    return x;
}

__device__ __forceinline__ float row_ror8(float x) {  // the value of lane l ^ 8 (DPP row_ror:8 in a 16-lane row)
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x128, 0xF, 0xF, false));
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {  // lane uniform: the value lands in SGPRs
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

template <class F, int P>
constexpr int paged_waves_per_eu() {  // NSG_ATT_DB8 fp8: room for the second chunk's registers
    return P == 1 ? 1 : (NSG_ATT_DB8 && std::is_same<F, FmtF8>::value) ? NSG_ATT_DB8_WPE : 4;
}

template <class F, int P>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(paged_waves_per_eu<F, P>()))) void paged_attn_kernel(
    const PagedArgs a) {
    typedef typename F::Elem E;
    typedef typename F::Raw Raw;
    constexpr int DPL = F::DPL, LPR = F::LPR, RPI = F::RPI, NI = F::NI;
    static_assert(RPI * NI == 32, "one iteration = one page's worth of rows");
    constexpr int NT = 8 * P;  // at most 8 splits per pair
    __shared__ float s_m[NT], s_l[NT];
    __shared__ float s_acc[NT][ATT_D];
    __shared__ int s_pi[8][P][4];  // per wave: pair, L0, s0 and first task of each of the workgroup's pairs
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    // Every wave works out the workgroup's pairs itself (lane j < P: pair j's length, skip flags and new-token page;
    // the same few loads in every wave hit the caches) -- no barrier before the streaming starts; the wave keeps
    // them in its own LDS slots, not in registers.
    int pr = -1, pL0 = 0, ps0 = 0, pS = 0, pst = 0;  // status 0 none / skipped, 1 run, 2 poison
    if (lane < P) {
        pr = att_pair<P>(blockIdx.x, lane, a.B, a.H);
        if (pr >= 0) {
            const int b = pr / a.H;
            pL0 = a.lens[b];
            const bool skip = (a.done && (a.done[(int64_t)b * a.done_stride] & 1u)) || (a.stop && pL0 >= a.stop[b]);
            if (!skip) {
                // the new token's stream row: its page must exist (host invariant).  One pair per workgroup (P = 1,
                // small batches): checked here, once; multi-pair workgroups: only the row is checked here and the page
                // by the pair's tasks, one load fewer before their streaming starts (2-3 % at short keys, B = 4,096;
                // at B = 1 the setup check measured 3-4 % faster per token, profiles/r06/c2_attn_setup_ab.txt)
                const int jj = pL0 - a.T0;
                const bool inside = jj >= 0 && (jj >> 5) < a.max_chunks;
                uint64_t pg = inside ? 1u : 0u;
                if constexpr (P == 1) pg = inside ? a.table[(int64_t)b * a.tstride + (jj >> 5)] : 0;
                if (pg == 0 || (P == 1 && (pg & 15u))) {
                    pst = 2;  // no page: poison the output (NaN logits the coder rejects), never write
                } else {
                    pst = 1;
                    const int Lk = pL0 + 1;
                    ps0 = a.window > 0 ? max(0, Lk - a.window) : 0;
                    pS = att_split(Lk - ps0);
                }
            }
        }
    }
    int pfirst = 0, ntask = 0, multi = 0;  // task index of pair (lane)'s split 0; tasks; any pair split S > 1
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const int sk = __shfl(pS, k);
        pfirst += k < lane ? sk : 0;
        ntask += sk;
        multi |= sk > 1;
    }
    if (wave < P && __shfl(pst, wave) == 2) {  // poisoned pair: NaN rows
        const int pair = __shfl(pr, wave);
        a.out[(int64_t)(pair / a.H) * a.out_stride + (pair % a.H) * ATT_D + lane] = (_Float16)__builtin_nanf("");
    }
    if (lane < P) {
        s_pi[wave][lane][0] = pr;
        s_pi[wave][lane][1] = pL0;
        s_pi[wave][lane][2] = ps0;
        s_pi[wave][lane][3] = pfirst;
    }
    const int myS = wave < P ? __shfl(pS, wave) : 0;  // the merge phase's pair (wave) split
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's own LDS slots are written before they are read
    __builtin_amdgcn_wave_barrier();
    const int g = lane / LPR;  // row within an RPI-row slab
    const int c = lane % LPR;  // DPL-dim slice
    const int C = a.H * ATT_D;
    for (int t = wave; t < ntask; t += 8) {  // wave-uniform
        int j = 0;
#pragma unroll
        for (int k = 1; k < P; ++k)
            if (t >= s_pi[wave][k][3]) j = k;  // the last pair whose first task is <= t (pairs without tasks share
                                               // the next one's first task and are passed over)
        const int pair = __builtin_amdgcn_readfirstlane(s_pi[wave][j][0]);
        const int L0 = __builtin_amdgcn_readfirstlane(s_pi[wave][j][1]);
        const int s0 = __builtin_amdgcn_readfirstlane(s_pi[wave][j][2]);
        const int wv = t - __builtin_amdgcn_readfirstlane(s_pi[wave][j][3]);
        const int S = att_split(L0 + 1 - s0);
        const int T0 = a.T0;
        const int Lk = L0 + 1;
        const int last_cached = L0 > 0 ? L0 - 1 : 0;
        const int b = pair / a.H, h = pair - b * a.H;
        const uint64_t* trow = a.table + (int64_t)b * a.tstride;
        const _Float16* qrow = a.qkv + (int64_t)b * a.qkv_stride + h * ATT_D + c * DPL;
        const typename F::Q q = F::load_q(qrow);
        const Raw knew = F::from_qkv(qrow + C);
        const Raw vnew = F::from_qkv(qrow + 2 * C);
        const int64_t hoff = a.layer_off + (int64_t)h * 32 * ATT_D + c * DPL;  // this layer's K rows of head h
        auto kaddr = [&](uint64_t page, int jj) -> E* { return (E*)page + hoff + (int64_t)(jj & 31) * ATT_D; };
        const E* kpb = (const E*)a.kp + (int64_t)h * a.ph + c * DPL;
        const E* vpb = (const E*)a.vp + (int64_t)h * a.ph + c * DPL;
        if constexpr (P == 1) {
            if (g == 0 && wv == 0) {  // KV append of the new token (position L0, page checked in the setup)
                E* kd = kaddr(trow[(L0 - T0) >> 5], L0 - T0);
                *(Raw*)kd = knew;
                *(Raw*)(kd + a.v_off) = vnew;
            }
        }
        float m = -1e30f, l = 0.0f;
        float acc[DPL];
#pragma unroll
        for (int d = 0; d < DPL; ++d) acc[d] = 0.0f;
        const int step = S * RPI * NI;
        const int jbeg = s0 + wv * RPI * NI;
        // page addresses of 64 iterations at a time, one per lane (lane i: iteration kbase + i; the first and the
        // last page of the stream rows it reads -- rows past the cache are clamped to the last cached one), read
        // back with readlane: no dependent table load inside the stream
        const int hi_row = last_cached - T0;  // the last stream row an iteration reads (< 0: prefix rows only)
        int kbase = -64;
        uint64_t pgA = 0, pgB = 0;
        auto pages_of = [&](int k, uint64_t& pa, uint64_t& pb) {
            if (k - kbase >= 64) {
                kbase = k;
                const int jj = jbeg + (k + lane) * step - T0;
                // rows read: [jj, jj + 31] clamped to the last cached row (as load_chunk clamps them); stream rows
                // only (< 0: the shared prefix); beyond the job's iterations the lane loads nothing
                const int lo = max(min(jj, hi_row), 0), hi = min(jj + RPI * NI - 1, hi_row);
                const bool any = hi >= 0 && jj <= L0 - T0;
                pgA = any ? trow[lo >> 5] : 0;
                pgB = any && (hi >> 5) != (lo >> 5) ? trow[hi >> 5] : pgA;
            }
            pa = readlane64(pgA, k - kbase);
            pb = readlane64(pgB, k - kbase);
        };
        // multi-pair workgroups: the new token's page -- a missing one (host invariant broken) poisons the pair: every
        // one of its tasks reads the same entry, writes nothing and hands NaN on (S = 1: the output row; S > 1: the
        // partials, which the merge turns into NaN).  The first iterations' page addresses are requested before it,
        // so both table reads are in flight together (the prefetch reads entries of cached rows only).
        bool bad = false;
        if constexpr (P > 1) {
            {
                uint64_t pa0, pb0;
                pages_of(0, pa0, pb0);
            }
            const uint64_t apage = trow[(L0 - T0) >> 5];
            bad = apage == 0 || (apage & 15u);
            if (g == 0 && wv == 0 && !bad) {  // KV append of the new token (position L0)
                E* kd = kaddr(apage, L0 - T0);
                *(Raw*)kd = knew;
                *(Raw*)(kd + a.v_off) = vnew;
            }
        }
        const int Lend = bad ? 0 : Lk;  // the streaming loops run while j0 < Lend
        // one iteration = RPI*NI = 32 consecutive rows from j0; GENERAL handles the prefix boundary, the clamp past
        // the cache and the new token; an interior run (stream rows < L0 only) spans at most two pages
        auto load_chunk = [&](int j0, int k, auto general, Raw (&kr)[NI], Raw (&vr)[NI]) {
            constexpr bool GEN = decltype(general)::value;
            uint64_t pa, pb;
            pages_of(k, pa, pb);
            if constexpr (GEN) {
                const int ca = max(min(j0 - T0, hi_row), 0) >> 5;  // the chunk of the first stream row read (pa)
#pragma unroll
                for (int u = 0; u < NI; ++u) {
                    const int row = min(j0 + RPI * u + g, last_cached);
                    if (row < T0) {
                        kr[u] = att_load((const Raw*)(kpb + (int64_t)row * ATT_D));
                        vr[u] = att_load((const Raw*)(vpb + (int64_t)row * ATT_D));
                    } else {
                        const int jj = row - T0;
                        const E* ka = kaddr((jj >> 5) == ca ? pa : pb, jj);
                        kr[u] = att_load((const Raw*)ka);
                        vr[u] = att_load((const Raw*)(ka + a.v_off));
                    }
                }
            } else {
                const int jj0 = j0 - T0;
                const int ca = jj0 >> 5;
#pragma unroll
                for (int u = 0; u < NI; ++u) {
                    const int jj = jj0 + RPI * u + g;
                    const E* ka = kaddr((jj >> 5) == ca ? pa : pb, jj);
                    kr[u] = att_load((const Raw*)ka);
                    vr[u] = att_load((const Raw*)(ka + a.v_off));
                }
            }
        };
        auto math_chunk = [&](int j0, auto general, Raw (&kr)[NI], Raw (&vr)[NI]) {
            constexpr bool GEN = decltype(general)::value;
            float sc[NI];
            bool valid[NI];
            float mx = m;
#pragma unroll
            for (int u = 0; u < NI; ++u) {
                const int row = j0 + RPI * u + g;
                valid[u] = GEN ? row < Lk : true;
                if (GEN && row == L0) {
                    kr[u] = knew;
                    vr[u] = vnew;
                }
                float sv = F::dot(q, kr[u]);
                if constexpr (NSG_ATT_DPP) {
                    sv = row_group_sum<LPR>(sv);
                } else {
#pragma unroll
                    for (int off = 1; off < LPR; off <<= 1) sv += __shfl_xor(sv, off);
                }
                sc[u] = sv * a.scale_log2;
                if (valid[u]) mx = fmaxf(mx, sc[u]);
            }
            const float alpha = exp2f(m - mx);
            l *= alpha;
#pragma unroll
            for (int d = 0; d < DPL; ++d) acc[d] *= alpha;
#pragma unroll
            for (int u = 0; u < NI; ++u) {
                const float p = valid[u] ? exp2f(sc[u] - mx) : 0.0f;
                l += p;
                float v[DPL];
                F::unpack(vr[u], v);
#pragma unroll
                for (int d = 0; d < DPL; ++d) acc[d] = fmaf(p, v[d], acc[d]);
            }
            m = mx;
        };
        auto interior = [&](int j0) { return j0 >= T0 && j0 + RPI * NI <= L0; };
        Raw kr[NI], vr[NI];
        if constexpr (P > 1 && !(NSG_ATT_DB8 && std::is_same<F, FmtF8>::value)) {
            int k = 0;
            for (int j0 = jbeg; j0 < Lend; j0 += step, ++k) {
                if (interior(j0)) {
                    load_chunk(j0, k, std::false_type{}, kr, vr);
                    math_chunk(j0, std::false_type{}, kr, vr);
                } else {
                    load_chunk(j0, k, std::true_type{}, kr, vr);
                    math_chunk(j0, std::true_type{}, kr, vr);
                }
            }
        } else {  // one pair per workgroup (small batches; NSG_ATT_DB8: fp8 always): register double buffer, as the
                  // lockstep kernel
            Raw kn[NI], vn[NI];
            int j0 = jbeg, k = 0;
            if (j0 < Lend) {
                if (interior(j0))
                    load_chunk(j0, 0, std::false_type{}, kr, vr);
                else
                    load_chunk(j0, 0, std::true_type{}, kr, vr);
            }
            for (; j0 < Lend; j0 += step, ++k) {
                const int j1 = j0 + step;
                if (j1 < Lend) {
                    if (interior(j1))
                        load_chunk(j1, k + 1, std::false_type{}, kn, vn);
                    else
                        load_chunk(j1, k + 1, std::true_type{}, kn, vn);
                }
                if (interior(j0))
                    math_chunk(j0, std::false_type{}, kr, vr);
                else
                    math_chunk(j0, std::true_type{}, kr, vr);
#pragma unroll
                for (int u = 0; u < NI; ++u) {
                    kr[u] = kn[u];
                    vr[u] = vn[u];
                }
            }
        }
        // merge the row groups (lanes c, c + LPR, ... hold the same dims); the lane ^ 8 step as a DPP row_ror:8
        // (within a 16-lane row that IS lane ^ 8; the merge is symmetric in the two lanes, so the same bits), the
        // others through ds_bpermute
#pragma unroll
        for (int off = LPR; off < 64; off <<= 1) {
            const bool dpp8 = NSG_ATT_DPP && off == 8;
            const float mo = dpp8 ? row_ror8(m) : __shfl_xor(m, off);
            const float lo = dpp8 ? row_ror8(l) : __shfl_xor(l, off);
            const float mn = fmaxf(m, mo);
            const float fa = exp2f(m - mn), fo = exp2f(mo - mn);
            l = l * fa + lo * fo;
#pragma unroll
            for (int d = 0; d < DPL; ++d) {
                const float ao = dpp8 ? row_ror8(acc[d]) : __shfl_xor(acc[d], off);
                acc[d] = acc[d] * fa + ao * fo;
            }
            m = mn;
        }
        if (bad) {
            m = l = __builtin_nanf("");
#pragma unroll
            for (int d = 0; d < DPL; ++d) acc[d] = __builtin_nanf("");
        }
        if (S == 1) {  // the whole pair in this wave: out = acc / l, as the lockstep kernel (a 1-way merge is exact)
            if (g == 0) {
                const float inv = 1.0f / l;
#pragma unroll
                for (int h8 = 0; h8 < DPL / 8; ++h8) {
                    f16x8 o;
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        float tv = acc[h8 * 8 + i] * inv;
                        asm volatile("" : "+v"(tv));
                        o[i] = (_Float16)tv;
                    }
                    *(f16x8*)(a.out + (int64_t)b * a.out_stride + h * ATT_D + c * DPL + h8 * 8) = o;
                }
            }
        } else if (g == 0) {
#pragma unroll
            for (int d = 0; d < DPL; ++d) s_acc[t][c * DPL + d] = acc[d];
            if (c == 0) {
                s_m[t] = m;
                s_l[t] = l;
            }
        }
    }
    if (!multi) return;  // uniform: no pair was split over waves
    __syncthreads();
    // pair (wave) split over S > 1 waves: merge the S partials in split order, as the lockstep kernel does
    if (wave >= P || lane >= LPR) return;
    const int S = myS;
    if (S <= 1) return;
    const int w0 = s_pi[wave][wave][3];
    const int pair = s_pi[wave][wave][0];
    const int b = pair / a.H, h = pair - b * a.H;
    float mt = s_m[w0];
    for (int w = 1; w < S; ++w) mt = fmaxf(mt, s_m[w0 + w]);
    float l = 0.0f;
    float acc[DPL];
#pragma unroll
    for (int d = 0; d < DPL; ++d) acc[d] = 0.0f;
    for (int w = 0; w < S; ++w) {
        const float f = exp2f(s_m[w0 + w] - mt);
        l += s_l[w0 + w] * f;
#pragma unroll
        for (int d = 0; d < DPL; ++d) acc[d] += s_acc[w0 + w][lane * DPL + d] * f;
    }
    const float inv = 1.0f / l;
#pragma unroll
    for (int h8 = 0; h8 < DPL / 8; ++h8) {
        f16x8 o;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float tv = acc[h8 * 8 + i] * inv;
            asm volatile("" : "+v"(tv));
            o[i] = (_Float16)tv;
        }
        *(f16x8*)(a.out + (int64_t)b * a.out_stride + h * ATT_D + lane * DPL + h8 * 8) = o;
    }
}

// fp16 -> fp8 (e4m3fn) with the same saturating round-to-nearest-even conversion as the kernel's KV append
__global__ void quantize_fp8_kernel(const _Float16* __restrict__ src, uint32_t* __restrict__ dst, int64_t n4) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    const _Float16* s4 = src + 4 * i;
    dst[i] = pack4_fp8((float)s4[0], (float)s4[1], (float)s4[2], (float)s4[3]);
}

// ------------------------------------------------------------------------------------------ causal sequences
// softmax(q k^T / sqrt(D) + causal mask) v over B sequences of T tokens at once: the shared-context prefill
// (code_base/arithmetic.py:115-122, first call), the guard's scoring forward (metrics/lm_scorer.py:121-131) and
// the max_context window forward of the src provider (lm/arithmetic.py:45-74).  Flash attention on the
// v_mfma_f32_16x16x32_f16 matrix cores: a workgroup of 4 waves owns 64 queries of one (sequence, head), each wave
// 16; key blocks of 64 are staged in LDS (K as [key][d], V transposed as [d][key], 16-byte chunks XOR-swizzled
// by (row >> 1) & 7 so every ds_read_b128 of a 16-lane group hits distinct banks); per block S = K Q^T (lane
// (r, c) holds query r's scores of keys 4c..4c+3 of each 16-key tile), an online softmax in fp32 (exp2, log2 e
// folded into the scale), P staged through LDS as fp16, O += V^T P (lane holds dims 4c..4c+3 of each 16-dim tile
// of query r).  A query's result depends only on its own sequence (fixed block order 0..its block, fixed MFMA
// chains), never on B or on the other queries of the tile: batch-invariant like the decode step.
typedef _Float16 sq_f16x4 __attribute__((ext_vector_type(4)));
typedef float sq_f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ sq_f32x4 sq_mfma(f16x8 a, f16x8 b, sq_f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int sq_swz(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ _Float16 sq_h(float v) {  // fp32 pinned before the conversion (no fused rounding)
    asm volatile("" : "+v"(v));
    return (_Float16)v;
}

__global__ __launch_bounds__(256) void seq_attn_kernel(const _Float16* __restrict__ qkv, int64_t qkv_stride,
                                                       _Float16* __restrict__ out, int64_t out_stride, int T, int H,
                                                       float scale_log2) {
    __shared__ __attribute__((aligned(16))) _Float16 sK[64 * ATT_D];
    __shared__ __attribute__((aligned(16))) _Float16 sVt[ATT_D * 64];
    __shared__ __attribute__((aligned(16))) _Float16 sP[4][16 * 64];
    const int nqb = (T + 63) / 64;
    const int qb = nqb - 1 - (int)(blockIdx.x % nqb);  // the longest query blocks of a pair are dispatched first
    const int bh = (int)(blockIdx.x / nqb);
    const int h = bh % H, b = bh / H;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 15, c = lane >> 4;
    const int C = H * ATT_D;
    const _Float16* base = qkv + (int64_t)b * T * qkv_stride + h * ATT_D;
    const int tq = qb * 64 + wave * 16 + r;  // this lane's query (padding rows past T are computed, not stored)
    f16x8 qf[2];
#pragma unroll
    for (int dc = 0; dc < 2; ++dc) qf[dc] = *(const f16x8*)(base + (int64_t)min(tq, T - 1) * qkv_stride + dc * 32 + c * 8);
    sq_f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = sq_f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -1e30f, l = 0.0f;
    _Float16* Pw = sP[wave];
    for (int kb = 0; kb <= qb; ++kb) {
        __syncthreads();  // the previous block's K / V reads are done
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int id = (int)threadIdx.x + 256 * u;
            const int key = id >> 3, ch = id & 7;
            const _Float16* src = base + (int64_t)min(kb * 64 + key, T - 1) * qkv_stride + ch * 8;
            const f16x8 kv = *(const f16x8*)(src + C);
            const f16x8 vv = *(const f16x8*)(src + 2 * C);
            *(f16x8*)(sK + key * 64 + ((ch ^ sq_swz(key)) * 8)) = kv;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int d = ch * 8 + i;
                sVt[d * 64 + (((key >> 3) ^ sq_swz(d)) * 8) + (key & 7)] = vv[i];
            }
        }
        __syncthreads();
        float s[4][4];
        float mx = -1e30f;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
            sq_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
            const int krow = kt * 16 + r;
#pragma unroll
            for (int dc = 0; dc < 2; ++dc)
                acc = sq_mfma(*(const f16x8*)(sK + krow * 64 + (((dc * 4 + c) ^ sq_swz(krow)) * 8)), qf[dc], acc);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int key = kb * 64 + kt * 16 + 4 * c + i;
                s[kt][i] = (key <= tq && key < T) ? acc[i] * scale_log2 : -__builtin_inff();
                mx = fmaxf(mx, s[kt][i]);
            }
        }
        mx = fmaxf(mx, __shfl_xor(mx, 16));
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        const float mnew = fmaxf(m, mx);
        const float alpha = __builtin_amdgcn_exp2f(m - mnew);
        l *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
            sq_f16x4 pv;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float pe = __builtin_amdgcn_exp2f(s[kt][i] - mnew);
                l += pe;
                pv[i] = sq_h(pe);
            }
            *(sq_f16x4*)(Pw + r * 64 + (((kt * 2 + (c >> 1)) ^ sq_swz(r)) * 8) + (c & 1) * 4) = pv;
        }
        m = mnew;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own P: every lane's writes have landed
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const f16x8 pf = *(const f16x8*)(Pw + r * 64 + (((ks * 4 + c) ^ sq_swz(r)) * 8));
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                const int drow = dt * 16 + r;
                o[dt] = sq_mfma(*(const f16x8*)(sVt + drow * 64 + (((ks * 4 + c) ^ sq_swz(drow)) * 8)), pf, o[dt]);
            }
        }
    }
    l += __shfl_xor(l, 16);
    l += __shfl_xor(l, 32);
    if (tq >= T) return;
    const float inv = 1.0f / l;
    _Float16* orow = out + (int64_t)(b * T + tq) * out_stride + h * ATT_D;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
        sq_f16x4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = sq_h(o[dt][i] * inv);
        *(sq_f16x4*)(orow + dt * 16 + 4 * c) = v;
    }
}

}  // namespace nsg

template <class F>
static int decode_attention(const void* d_qkv, int64_t qkv_stride, void* d_k_cache, void* d_v_cache,
                            int64_t cache_b_stride, int64_t cache_h_stride, int64_t cache_chunk_stride,
                            const void* d_k_prefix,
                            const void* d_v_prefix, int64_t prefix_h_stride, int T0, int B, int H, int D, int L0,
                            const int32_t* d_L0, int cap, int window, void* d_out, int64_t out_stride, float scale,
                            void* hip_stream, const uint32_t* d_done = nullptr, int64_t done_stride = 0,
                            const int32_t* d_stop = nullptr) {
    if (d_done && done_stride < 1) return NS_ERR_CONFIG;
    typedef typename F::Elem E;
    if (window < 0) return NS_ERR_CONFIG;
    if (!d_qkv || !d_k_cache || !d_v_cache || !d_out || B <= 0 || H <= 0 || L0 < 0 || T0 < 0) return NS_ERR_CONFIG;
    if (D != nsg::ATT_D) return NS_ERR_UNSUPPORTED;
    constexpr int ALIGN_E = 16 / (int)sizeof(E);  // elements per 16-byte unit of the cache
    if (T0 > 0 && (!d_k_prefix || !d_v_prefix || prefix_h_stride < (int64_t)T0 * D || (prefix_h_stride % ALIGN_E)))
        return NS_ERR_CONFIG;
    if (!d_L0 && L0 < T0) return NS_ERR_CONFIG;
    const uintptr_t align = (uintptr_t)d_qkv | (uintptr_t)d_k_cache | (uintptr_t)d_v_cache | (uintptr_t)d_out |
                            (uintptr_t)(T0 > 0 ? d_k_prefix : d_qkv) | (uintptr_t)(T0 > 0 ? d_v_prefix : d_qkv);
    if (cache_chunk_stride == 0) cache_chunk_stride = 32LL * D;  // plain layout: rows contiguous per (b, h)
    if ((align & 15u) || (qkv_stride & 7) || (out_stride & 7) || (cache_b_stride % ALIGN_E) ||
        (cache_h_stride % ALIGN_E) || (cache_chunk_stride % ALIGN_E))
        return NS_ERR_CONFIG;  // 16-byte rows
    if (qkv_stride < 3LL * H * D || out_stride < (int64_t)H * D) return NS_ERR_CONFIG;
    // the stream cache holds positions [T0, cap): cap - T0 rows per (stream, head), in 32-row chunks
    if (cap <= T0) return NS_ERR_CONFIG;
    const int64_t nchunks = (cap - T0 + 31) / 32;
    if (cache_chunk_stride == 32LL * D && cache_h_stride >= (int64_t)(cap - T0) * D) {
        // plain: a pair's rows contiguous, pairs apart by the h / b strides
        if (cache_b_stride < (int64_t)H * cache_h_stride) return NS_ERR_CONFIG;
    } else {  // chunked: a plane of B*H chunks per 32 positions
        if (cache_h_stride < 32LL * D || cache_b_stride < (int64_t)H * cache_h_stride ||
            cache_chunk_stride < (int64_t)B * cache_b_stride || nchunks < 1)
            return NS_ERR_CONFIG;
    }
    if (!d_L0 && L0 >= cap) return NS_ERR_CONFIG;
    if ((int64_t)B * H > 0x7FFFFFFF) return NS_ERR_UNSUPPORTED;
    const int pairs = B * H;
    const float scale_log2 = scale * 1.4426950408889634f;
    // The row split per pair (att_split) depends on the key count only, so a stream's output -- and the logits the
    // coder sees -- does not depend on how many other streams share the launch (a cover encoded at B = 4096 is
    // decoded alone).  Pairs per workgroup follow the batch: 8 when there are enough pairs to fill the chip.
    const hipStream_t st = (hipStream_t)hip_stream;
    const _Float16* q = (const _Float16*)d_qkv;
    E *k = (E*)d_k_cache, *v = (E*)d_v_cache;
    _Float16* o = (_Float16*)d_out;
    const E* kp = T0 > 0 ? (const E*)d_k_prefix : k;
    const E* vp = T0 > 0 ? (const E*)d_v_prefix : v;
    if (pairs <= NSG_ATT_SMALL_PAIRS)
        hipLaunchKernelGGL((nsg::decode_attn_kernel<F, 1>), dim3(pairs), dim3(512), 0, st, q, qkv_stride, k, v,
                           cache_b_stride, cache_h_stride, cache_chunk_stride, kp, vp, prefix_h_stride, T0, B, H,
                           L0, d_L0, cap, window, d_done, done_stride, d_stop, o, out_stride, scale_log2);
    else
        hipLaunchKernelGGL((nsg::decode_attn_kernel<F, 8>), dim3(NSG_ATT_HEAD_MAJOR ? H * ((B + 7) / 8) : (pairs + 7) / 8),
                           dim3(512), 0, st, q, qkv_stride, k,
                           v, cache_b_stride, cache_h_stride, cache_chunk_stride, kp, vp, prefix_h_stride, T0, B,
                           H, L0, d_L0, cap, window, d_done, done_stride, d_stop, o, out_stride, scale_log2);
    return hipGetLastError() == hipSuccess ? NS_OK : NS_ERR_HIP;
}

extern "C" int ns_decode_attention(const void* d_qkv, int64_t qkv_stride, void* d_k_cache, void* d_v_cache,
                                   int64_t cache_b_stride, int64_t cache_h_stride, int B, int H, int D, int L0,
                                   void* d_out, int64_t out_stride, float scale, void* hip_stream) {
    return decode_attention<nsg::FmtF16>(d_qkv, qkv_stride, d_k_cache, d_v_cache, cache_b_stride, cache_h_stride, 0,
                                         nullptr, nullptr, 0, 0, B, H, D, L0, nullptr, L0 + 1, 0, d_out, out_stride,
                                         scale, hip_stream);
}

extern "C" int ns_decode_attention_dev(const void* d_qkv, int64_t qkv_stride, void* d_k_cache, void* d_v_cache,
                                       int64_t cache_b_stride, int64_t cache_h_stride, int B, int H, int D,
                                       const int32_t* d_L0, int cap, void* d_out, int64_t out_stride, float scale,
                                       void* hip_stream) {
    if (!d_L0 || cap < 1) return NS_ERR_CONFIG;
    return decode_attention<nsg::FmtF16>(d_qkv, qkv_stride, d_k_cache, d_v_cache, cache_b_stride, cache_h_stride, 0,
                                         nullptr, nullptr, 0, 0, B, H, D, 0, d_L0, cap, 0, d_out, out_stride, scale,
                                         hip_stream);
}

extern "C" int ns_decode_attention_prefix(const void* d_qkv, int64_t qkv_stride, void* d_k_cache, void* d_v_cache,
                                          int64_t cache_b_stride, int64_t cache_h_stride, int64_t cache_chunk_stride,
                                          const void* d_k_prefix, const void* d_v_prefix, int64_t prefix_h_stride,
                                          int T0, int B, int H, int D, int L0, const int32_t* d_L0, int cap, int window,
                                          void* d_out, int64_t out_stride, float scale, void* hip_stream) {
    return decode_attention<nsg::FmtF16>(d_qkv, qkv_stride, d_k_cache, d_v_cache, cache_b_stride, cache_h_stride,
                                         cache_chunk_stride, d_k_prefix, d_v_prefix, prefix_h_stride, T0, B, H, D,
                                         d_L0 ? 0 : L0, d_L0, cap, window, d_out, out_stride, scale, hip_stream);
}

extern "C" int ns_decode_attention_fp8(const void* d_qkv, int64_t qkv_stride, void* d_k_cache, void* d_v_cache,
                                       int64_t cache_b_stride, int64_t cache_h_stride, int64_t cache_chunk_stride,
                                       const void* d_k_prefix, const void* d_v_prefix, int64_t prefix_h_stride,
                                       int T0, int B, int H, int D, int L0, const int32_t* d_L0, int cap, int window,
                                       void* d_out, int64_t out_stride, float scale, void* hip_stream) {
    return decode_attention<nsg::FmtF8>(d_qkv, qkv_stride, d_k_cache, d_v_cache, cache_b_stride, cache_h_stride,
                                        cache_chunk_stride, d_k_prefix, d_v_prefix, prefix_h_stride, T0, B, H, D,
                                        d_L0 ? 0 : L0, d_L0, cap, window, d_out, out_stride, scale, hip_stream);
}

extern "C" int ns_decode_attention_ex(const void* d_qkv, int64_t qkv_stride, void* d_k_cache, void* d_v_cache,
                                      int64_t cache_b_stride, int64_t cache_h_stride, int64_t cache_chunk_stride,
                                      const void* d_k_prefix, const void* d_v_prefix, int64_t prefix_h_stride, int T0,
                                      int B, int H, int D, int L0, const int32_t* d_L0, int cap, int window,
                                      int kv_format, const uint32_t* d_done, int64_t done_stride,
                                      const int32_t* d_stop, void* d_out, int64_t out_stride, float scale,
                                      void* hip_stream) {
    if (kv_format == NS_KV_FP16)
        return decode_attention<nsg::FmtF16>(d_qkv, qkv_stride, d_k_cache, d_v_cache, cache_b_stride, cache_h_stride,
                                             cache_chunk_stride, d_k_prefix, d_v_prefix, prefix_h_stride, T0, B, H, D,
                                             d_L0 ? 0 : L0, d_L0, cap, window, d_out, out_stride, scale, hip_stream,
                                             d_done, done_stride, d_stop);
    if (kv_format == NS_KV_FP8)
        return decode_attention<nsg::FmtF8>(d_qkv, qkv_stride, d_k_cache, d_v_cache, cache_b_stride, cache_h_stride,
                                            cache_chunk_stride, d_k_prefix, d_v_prefix, prefix_h_stride, T0, B, H, D,
                                            d_L0 ? 0 : L0, d_L0, cap, window, d_out, out_stride, scale, hip_stream,
                                            d_done, done_stride, d_stop);
    return NS_ERR_CONFIG;
}

template <class F>
static int paged_attention(nsg::PagedArgs a, void* hip_stream) {
    const hipStream_t st = (hipStream_t)hip_stream;
    const int pairs = a.B * a.H;
    if (pairs <= NSG_ATT_SMALL_PAIRS)
        hipLaunchKernelGGL((nsg::paged_attn_kernel<F, 1>), dim3(pairs), dim3(512), 0, st, a);
    else
        hipLaunchKernelGGL((nsg::paged_attn_kernel<F, 8>), dim3(a.H * ((a.B + 7) / 8)), dim3(512), 0, st, a);
    return hipGetLastError() == hipSuccess ? NS_OK : NS_ERR_HIP;
}

extern "C" int ns_decode_attention_paged(const void* d_qkv, int64_t qkv_stride, const uint64_t* d_page_table,
                                         int64_t table_stride, int max_chunks, int64_t layer_offset,
                                         const void* d_k_prefix,
                                         const void* d_v_prefix, int64_t prefix_h_stride, int T0, int B, int H, int D,
                                         const int32_t* d_lens, int window, int kv_format, const uint32_t* d_done,
                                         int64_t done_stride, const int32_t* d_stop, void* d_out, int64_t out_stride,
                                         float scale, void* hip_stream) {
    if (!d_qkv || !d_page_table || !d_lens || !d_out || B <= 0 || H <= 0 || T0 < 0 || layer_offset < 0 || window < 0)
        return NS_ERR_CONFIG;
    if (D != nsg::ATT_D) return NS_ERR_UNSUPPORTED;
    if (kv_format != NS_KV_FP16 && kv_format != NS_KV_FP8) return NS_ERR_CONFIG;
    if (max_chunks < 1 || table_stride < max_chunks || (d_done && done_stride < 1)) return NS_ERR_CONFIG;
    const int64_t esz = kv_format == NS_KV_FP8 ? 1 : 2;
    if (T0 > 0 && (!d_k_prefix || !d_v_prefix || prefix_h_stride < (int64_t)T0 * D || ((prefix_h_stride * esz) & 15)))
        return NS_ERR_CONFIG;
    const uintptr_t align = (uintptr_t)d_qkv | (uintptr_t)d_out | (uintptr_t)(T0 > 0 ? d_k_prefix : d_qkv) |
                            (uintptr_t)(T0 > 0 ? d_v_prefix : d_qkv);
    if ((align & 15u) || (qkv_stride & 7) || (out_stride & 7) || ((uintptr_t)d_lens & 3u) ||
        ((uintptr_t)d_page_table & 7u))  // table entries are read one uint64 at a time: any row of a table works
        return NS_ERR_CONFIG;
    if (qkv_stride < 3LL * H * D || out_stride < (int64_t)H * D) return NS_ERR_CONFIG;
    if ((int64_t)B * H > 0x7FFFFFFF) return NS_ERR_UNSUPPORTED;
    nsg::PagedArgs a;
    a.qkv = (const _Float16*)d_qkv;
    a.qkv_stride = qkv_stride;
    a.table = d_page_table;
    a.tstride = table_stride;
    a.max_chunks = max_chunks;
    a.v_off = (int64_t)H * 32 * D;
    if (layer_offset % (16 / esz)) return NS_ERR_CONFIG;  // 16-byte rows
    a.layer_off = layer_offset;
    a.kp = T0 > 0 ? d_k_prefix : d_qkv;
    a.vp = T0 > 0 ? d_v_prefix : d_qkv;
    a.ph = prefix_h_stride;
    a.T0 = T0;
    a.B = B;
    a.H = H;
    a.lens = d_lens;
    a.window = window;
    a.done = d_done;
    a.done_stride = done_stride;
    a.stop = d_stop;
    a.out = (_Float16*)d_out;
    a.out_stride = out_stride;
    a.scale_log2 = scale * 1.4426950408889634f;
    return kv_format == NS_KV_FP8 ? paged_attention<nsg::FmtF8>(a, hip_stream)
                                  : paged_attention<nsg::FmtF16>(a, hip_stream);
}

extern "C" int ns_quantize_fp8(const void* d_src, void* d_dst, int64_t n, void* hip_stream) {
    if (!d_src || !d_dst || n < 0 || (n & 3) || (((uintptr_t)d_src | (uintptr_t)d_dst) & 7u)) return NS_ERR_CONFIG;
    if (n == 0) return NS_OK;
    const int64_t n4 = n / 4;
    hipLaunchKernelGGL(nsg::quantize_fp8_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0,
                       (hipStream_t)hip_stream, (const _Float16*)d_src, (uint32_t*)d_dst, n4);
    return hipGetLastError() == hipSuccess ? NS_OK : NS_ERR_HIP;
}

extern "C" int ns_seq_attention(const void* d_qkv, int64_t qkv_stride, void* d_out, int64_t out_stride, int B, int T,
                                int H, int D, float scale, void* hip_stream) {
    if (!d_qkv || !d_out || B < 1 || T < 1 || H < 1) return NS_ERR_CONFIG;
    if (D != nsg::ATT_D) return NS_ERR_UNSUPPORTED;
    if (qkv_stride < 3LL * H * D || out_stride < (int64_t)H * D || (qkv_stride & 7) || (out_stride & 3) ||
        (((uintptr_t)d_qkv | (uintptr_t)d_out) & 15u))
        return NS_ERR_CONFIG;
    const int64_t nwg = (int64_t)B * H * ((T + 63) / 64);
    if (nwg > 0x7FFFFFFF) return NS_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(nsg::seq_attn_kernel, dim3((unsigned)nwg), dim3(256), 0, (hipStream_t)hip_stream,
                       (const _Float16*)d_qkv, qkv_stride, (_Float16*)d_out, out_stride, T, H,
                       scale * 1.4426950408889634f);
    return hipGetLastError() == hipSuccess ? NS_OK : NS_ERR_HIP;
}

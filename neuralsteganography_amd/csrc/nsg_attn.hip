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

#include "nsg_attn.h"
#include "nsg_coder.h"

namespace nsg {

#ifndef NSG_ATT_ROWS1
#define NSG_ATT_ROWS1 128  // keys per pair up to which one wave takes the whole pair (then 2, 4, 8 waves)
#endif
#ifndef NSG_ATT_SMALL_PAIRS
#define NSG_ATT_SMALL_PAIRS 1024  // up to this many (stream, head) pairs: one pair per workgroup
#endif

constexpr int ATT_D = 64;
constexpr int ATT_U = 4;      // 8-row chunks per loop iteration: 32 keys per wave in flight

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

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

// Workgroup = 8 waves serving P consecutive pairs (P = 1 for small batches, 8 otherwise; P changes only which
// workgroup computes a pair, not how).  With S = att_split(L0 + 1), the waves form 8/S groups of S; group
// q takes pairs q, q + 8/S, ... of the workgroup, one round per pair, all waves running the same number of
// rounds so the LDS merge's barriers are uniform.
// Positions [0, T0) come from a prefix shared by every stream (kp/vp, head stride ph: the common context,
// stored once), positions [T0, L0] from the stream's own cache at index position - T0.  Same values, same
// order: the output bits do not depend on where a row is stored.
template <int P>
__global__ __launch_bounds__(512) void decode_attn_kernel(const _Float16* __restrict__ qkv, int64_t qkv_stride,
                                                          _Float16* kc, _Float16* vc, int64_t cb, int64_t ch,
                                                          const _Float16* __restrict__ kp,
                                                          const _Float16* __restrict__ vp, int64_t ph, int T0, int B,
                                                          int H, int L0, const int32_t* __restrict__ L0p, int cap,
                                                          _Float16* __restrict__ out, int64_t out_stride,
                                                          float scale_log2) {
    if (L0p) L0 = __builtin_amdgcn_readfirstlane(*L0p);  // graph replays: the cache length lives on the device
    if (L0 < T0 || L0 >= cap) return;                    // never write past the cache (host checks capacity)
    __shared__ float s_m[8], s_l[8];
    __shared__ float s_acc[8][ATT_D];
    const int Lk = L0 + 1;
    const int S = att_split(Lk);
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int grp = wave / S, wv = wave - grp * S, ngrp = 8 / S;
    const int g = lane >> 3;  // row within an 8-row chunk
    const int c = lane & 7;   // 8-dim slice
    const int C = H * ATT_D;
    const int last_cached = L0 > 0 ? L0 - 1 : 0;
    const int rounds = (P + ngrp - 1) / ngrp;
    for (int rd = 0; rd < rounds; ++rd) {
        const int j = grp + rd * ngrp;
        const int pair = blockIdx.x * P + j;
        const bool active = j < P && pair < B * H;  // uniform per wave group
        float m = -1e30f, l = 0.0f;
        float acc[8];
#pragma unroll
        for (int d = 0; d < 8; ++d) acc[d] = 0.0f;
        int b = 0, h = 0;
        if (active) {
            b = pair / H;
            h = pair - b * H;
            const _Float16* qrow = qkv + (int64_t)b * qkv_stride + h * ATT_D + c * 8;
            const f16x8 q = *(const f16x8*)qrow;
            const f16x8 knew = *(const f16x8*)(qrow + C);
            const f16x8 vnew = *(const f16x8*)(qrow + 2 * C);
            // stream rows are addressed by position (index position - T0 folded into the base)
            _Float16* kb = kc + (int64_t)b * cb + (int64_t)h * ch + c * 8 - (int64_t)T0 * ATT_D;
            _Float16* vb = vc + (int64_t)b * cb + (int64_t)h * ch + c * 8 - (int64_t)T0 * ATT_D;
            const _Float16* kpb = kp + (int64_t)h * ph + c * 8;
            const _Float16* vpb = vp + (int64_t)h * ph + c * 8;
            if (g == 0 && wv == 0) {  // KV append of the new token (position L0)
                *(f16x8*)(kb + (int64_t)L0 * ATT_D) = knew;
                *(f16x8*)(vb + (int64_t)L0 * ATT_D) = vnew;
            }
            for (int j0 = wv * 8 * ATT_U; j0 < Lk; j0 += S * 8 * ATT_U) {
                f16x8 kr[ATT_U], vr[ATT_U];
#pragma unroll
                for (int u = 0; u < ATT_U; ++u) {
                    const int row = min(j0 + 8 * u + g, last_cached);
                    const bool pre = row < T0;
                    const _Float16* ka = (pre ? kpb : kb) + (int64_t)row * ATT_D;
                    const _Float16* va = (pre ? vpb : vb) + (int64_t)row * ATT_D;
                    kr[u] = __builtin_nontemporal_load((const f16x8*)ka);
                    vr[u] = __builtin_nontemporal_load((const f16x8*)va);
                }
                float sc[ATT_U];
                bool valid[ATT_U];
                float mx = m;
#pragma unroll
                for (int u = 0; u < ATT_U; ++u) {
                    const int row = j0 + 8 * u + g;
                    valid[u] = row < Lk;
                    if (row == L0) {  // the new token: from registers, not from the cache just written
                        kr[u] = knew;
                        vr[u] = vnew;
                    }
                    float sv = dot8(q, kr[u]);
                    sv += __shfl_xor(sv, 1);
                    sv += __shfl_xor(sv, 2);
                    sv += __shfl_xor(sv, 4);
                    sc[u] = sv * scale_log2;
                    if (valid[u]) mx = fmaxf(mx, sc[u]);
                }
                const float alpha = exp2f(m - mx);
                l *= alpha;
#pragma unroll
                for (int d = 0; d < 8; ++d) acc[d] *= alpha;
#pragma unroll
                for (int u = 0; u < ATT_U; ++u) {
                    const float p = valid[u] ? exp2f(sc[u] - mx) : 0.0f;
                    l += p;
                    float v[8];
                    unpack8(vr[u], v);
#pragma unroll
                    for (int d = 0; d < 8; ++d) acc[d] = fmaf(p, v[d], acc[d]);
                }
                m = mx;
            }
            // merge the 8 row groups (lanes c, c+8, ..., c+56 hold the same dims)
#pragma unroll
            for (int off = 8; off < 64; off <<= 1) {
                const float mo = __shfl_xor(m, off);
                const float lo = __shfl_xor(l, off);
                const float mn = fmaxf(m, mo);
                const float fa = exp2f(m - mn), fo = exp2f(mo - mn);
                l = l * fa + lo * fo;
#pragma unroll
                for (int d = 0; d < 8; ++d) {
                    const float ao = __shfl_xor(acc[d], off);
                    acc[d] = acc[d] * fa + ao * fo;
                }
                m = mn;
            }
        }
        if (S > 1) {  // uniform over the workgroup: hand the S partials of each group to its first wave
            if (active && g == 0) {
#pragma unroll
                for (int d = 0; d < 8; ++d) s_acc[wave][c * 8 + d] = acc[d];
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
                for (int d = 0; d < 8; ++d) acc[d] = 0.0f;
                for (int w = 0; w < S; ++w) {
                    const float f = exp2f(s_m[w0 + w] - mt);
                    l += s_l[w0 + w] * f;
#pragma unroll
                    for (int d = 0; d < 8; ++d) acc[d] += s_acc[w0 + w][c * 8 + d] * f;
                }
            }
            __syncthreads();  // the LDS slots are reused by the next round
        }
        if (active && wv == 0 && g == 0) {
            const float inv = 1.0f / l;
            f16x8 o;
#pragma unroll
            for (int i = 0; i < 8; ++i) o[i] = (_Float16)(acc[i] * inv);
            *(f16x8*)(out + (int64_t)b * out_stride + h * ATT_D + c * 8) = o;
        }
    }
}

}  // namespace nsg

static int decode_attention(const void* d_qkv, int64_t qkv_stride, void* d_k_cache, void* d_v_cache,
                            int64_t cache_b_stride, int64_t cache_h_stride, const void* d_k_prefix,
                            const void* d_v_prefix, int64_t prefix_h_stride, int T0, int B, int H, int D, int L0,
                            const int32_t* d_L0, int cap, void* d_out, int64_t out_stride, float scale,
                            void* hip_stream) {
    if (!d_qkv || !d_k_cache || !d_v_cache || !d_out || B <= 0 || H <= 0 || L0 < 0 || T0 < 0) return NS_ERR_CONFIG;
    if (D != nsg::ATT_D) return NS_ERR_UNSUPPORTED;
    if (T0 > 0 && (!d_k_prefix || !d_v_prefix || prefix_h_stride < (int64_t)T0 * D || (prefix_h_stride & 7)))
        return NS_ERR_CONFIG;
    if (!d_L0 && L0 < T0) return NS_ERR_CONFIG;
    const uintptr_t align = (uintptr_t)d_qkv | (uintptr_t)d_k_cache | (uintptr_t)d_v_cache | (uintptr_t)d_out |
                            (uintptr_t)(T0 > 0 ? d_k_prefix : d_qkv) | (uintptr_t)(T0 > 0 ? d_v_prefix : d_qkv);
    if ((align & 15u) || (qkv_stride & 7) || (out_stride & 7) || (cache_b_stride & 7) || (cache_h_stride & 7))
        return NS_ERR_CONFIG;  // 16-byte rows
    if (qkv_stride < 3LL * H * D || out_stride < (int64_t)H * D) return NS_ERR_CONFIG;
    // the stream cache holds positions [T0, cap): cap - T0 rows per (stream, head)
    if (cap <= T0 || cache_h_stride < (int64_t)(cap - T0) * D || cache_b_stride < (int64_t)H * cache_h_stride)
        return NS_ERR_CONFIG;
    if (!d_L0 && L0 >= cap) return NS_ERR_CONFIG;
    if ((int64_t)B * H > 0x7FFFFFFF) return NS_ERR_UNSUPPORTED;
    const int pairs = B * H;
    const float scale_log2 = scale * 1.4426950408889634f;
    // The row split per pair (att_split) depends on the key count only, so a stream's output -- and the logits the
    // coder sees -- does not depend on how many other streams share the launch (a cover encoded at B = 4096 is
    // decoded alone).  Pairs per workgroup follow the batch: 8 when there are enough pairs to fill the chip.
    const hipStream_t st = (hipStream_t)hip_stream;
    const _Float16* q = (const _Float16*)d_qkv;
    _Float16 *k = (_Float16*)d_k_cache, *v = (_Float16*)d_v_cache, *o = (_Float16*)d_out;
    const _Float16* kp = T0 > 0 ? (const _Float16*)d_k_prefix : k;
    const _Float16* vp = T0 > 0 ? (const _Float16*)d_v_prefix : v;
    if (pairs <= NSG_ATT_SMALL_PAIRS)
        hipLaunchKernelGGL(nsg::decode_attn_kernel<1>, dim3(pairs), dim3(512), 0, st, q, qkv_stride, k, v,
                           cache_b_stride, cache_h_stride, kp, vp, prefix_h_stride, T0, B, H, L0, d_L0, cap, o,
                           out_stride, scale_log2);
    else
        hipLaunchKernelGGL(nsg::decode_attn_kernel<8>, dim3((pairs + 7) / 8), dim3(512), 0, st, q, qkv_stride, k, v,
                           cache_b_stride, cache_h_stride, kp, vp, prefix_h_stride, T0, B, H, L0, d_L0, cap, o,
                           out_stride, scale_log2);
    return hipGetLastError() == hipSuccess ? NS_OK : NS_ERR_HIP;
}

extern "C" int ns_decode_attention(const void* d_qkv, int64_t qkv_stride, void* d_k_cache, void* d_v_cache,
                                   int64_t cache_b_stride, int64_t cache_h_stride, int B, int H, int D, int L0,
                                   void* d_out, int64_t out_stride, float scale, void* hip_stream) {
    return decode_attention(d_qkv, qkv_stride, d_k_cache, d_v_cache, cache_b_stride, cache_h_stride, nullptr, nullptr,
                            0, 0, B, H, D, L0, nullptr, L0 + 1, d_out, out_stride, scale, hip_stream);
}

extern "C" int ns_decode_attention_dev(const void* d_qkv, int64_t qkv_stride, void* d_k_cache, void* d_v_cache,
                                       int64_t cache_b_stride, int64_t cache_h_stride, int B, int H, int D,
                                       const int32_t* d_L0, int cap, void* d_out, int64_t out_stride, float scale,
                                       void* hip_stream) {
    if (!d_L0 || cap < 1) return NS_ERR_CONFIG;
    return decode_attention(d_qkv, qkv_stride, d_k_cache, d_v_cache, cache_b_stride, cache_h_stride, nullptr, nullptr,
                            0, 0, B, H, D, 0, d_L0, cap, d_out, out_stride, scale, hip_stream);
}

extern "C" int ns_decode_attention_prefix(const void* d_qkv, int64_t qkv_stride, void* d_k_cache, void* d_v_cache,
                                          int64_t cache_b_stride, int64_t cache_h_stride, const void* d_k_prefix,
                                          const void* d_v_prefix, int64_t prefix_h_stride, int T0, int B, int H,
                                          int D, int L0, const int32_t* d_L0, int cap, void* d_out,
                                          int64_t out_stride, float scale, void* hip_stream) {
    return decode_attention(d_qkv, qkv_stride, d_k_cache, d_v_cache, cache_b_stride, cache_h_stride, d_k_prefix,
                            d_v_prefix, prefix_h_stride, T0, B, H, D, d_L0 ? 0 : L0, d_L0, cap, d_out, out_stride,
                            scale, hip_stream);
}

// Per-row log-softmax scores (include/nsg_score.h): nll of the label and the entropy of the row, for the
// cover-text quality guard's perplexity / average-entropy metrics.
//
// One wavefront per row; lane l reads 16-byte vectors l, l+64, ... of the row (coalesced 1 KiB wave loads,
// non-temporal: every row is read exactly once).  Per lane an online softmax over vectors: the vector max
// rescales the running sums once per vector, so the loop costs one extra exp per 4 (fp32) / 8 (fp16) elements.
// The 64 lane states are merged in float64.

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "nsg_coder.h"
#include "nsg_score.h"

namespace nsg {

constexpr int SC_WAVES = 4;  // rows per 256-thread workgroup

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <typename T>
struct ScoreVec;

template <>
struct ScoreVec<float> {
    static constexpr int N = 4;
    typedef f32x4 V;
    __device__ static void load(const char* p, float* x) {
        const V v = __builtin_nontemporal_load((const V*)p);
        x[0] = v.x;
        x[1] = v.y;
        x[2] = v.z;
        x[3] = v.w;
    }
    __device__ static float at(const char* row, int j) { return ((const float*)row)[j]; }
};

template <>
struct ScoreVec<_Float16> {
    static constexpr int N = 8;
    typedef f16x8 V;
    __device__ static void load(const char* p, float* x) {
        const V v = __builtin_nontemporal_load((const V*)p);
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = (float)v[i];
    }
    __device__ static float at(const char* row, int j) { return (float)((const _Float16*)row)[j]; }
};

template <typename T>
__global__ __launch_bounds__(64 * SC_WAVES) void score_rows_kernel(const char* __restrict__ logits, int64_t ld,
                                                                  int64_t nrows, int V,
                                                                  const int32_t* __restrict__ labels,
                                                                  double* __restrict__ nll, double* __restrict__ ent) {
    constexpr int N = ScoreVec<T>::N;
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * SC_WAVES + (threadIdx.x >> 6);
    if (r >= nrows) return;
    const char* row = logits + r * ld * (int64_t)sizeof(T);
    const int nvec = V / N;  // full vectors; the tail (V % N ids) is handled element-wise below
    // lane state: m = running max, s = sum e^(x - m), u = sum e^(x - m) (x - m)
    float m = -INFINITY, s = 0.0f, u = 0.0f;
    auto rebase = [&](float mv) {  // new max mv > m: u' = a (u + s (m - mv)), s' = a s, a = e^(m - mv)
        if (s > 0.0f) {
            const float a = __expf(m - mv);
            u = a * fmaf(s, m - mv, u);
            s *= a;
        }
        m = mv;
    };
    for (int v = lane; v < nvec; v += 64) {
        float x[N];
        ScoreVec<T>::load(row + (int64_t)v * N * sizeof(T), x);
        float mv = x[0];
#pragma unroll
        for (int i = 1; i < N; ++i) mv = fmaxf(mv, x[i]);
        if (mv > m) rebase(mv);
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const float d = x[i] - m;
            const float e = __expf(d);
            s += e;
            u = fmaf(e, d, u);
        }
    }
    for (int j = nvec * N + lane; j < V; j += 64) {  // ragged tail (V % N ids)
        const float x = ScoreVec<T>::at(row, j);
        if (x > m) rebase(x);
        const float d = x - m;
        const float e = __expf(d);
        s += e;
        u = fmaf(e, d, u);
    }
    double M = (double)m, S = (double)s, U = (double)u;
    for (int off = 32; off >= 1; off >>= 1) {
        const double Mo = __shfl_xor(M, off), So = __shfl_xor(S, off), Uo = __shfl_xor(U, off);
        const double Mn = fmax(M, Mo);
        const double fa = (S > 0.0) ? exp(M - Mn) : 0.0, fo = (So > 0.0) ? exp(Mo - Mn) : 0.0;
        // u relative to Mn: sum e_i (x_i - Mn) = f*(u + s*(M - Mn))
        U = (S > 0.0 ? fa * (U + S * (M - Mn)) : 0.0) + (So > 0.0 ? fo * (Uo + So * (Mo - Mn)) : 0.0);
        S = fa * S + fo * So;
        M = Mn;
    }
    if (lane == 0) {
        const double lse = M + log(S);
        // entropy = lse - sum p x = -(sum e (x - M))/S + log S
        if (ent) ent[r] = log(S) - U / S;
        if (nll) {
            const int lab = labels ? labels[r] : -1;
            nll[r] = (lab >= 0 && lab < V) ? lse - (double)ScoreVec<T>::at(row, lab) : 0.0;
        }
    }
}

}  // namespace nsg

extern "C" int ns_score_rows(const void* d_logits, int64_t ld, int64_t nrows, int V, int dtype,
                             const int32_t* d_labels, double* d_nll, double* d_entropy, void* hip_stream) {
    if (!d_logits || nrows < 0 || V <= 0 || ld < V) return NS_ERR_CONFIG;
    if (nrows == 0) return NS_OK;
    const size_t esz = dtype == NS_DTYPE_F16 ? 2 : 4;
    if (dtype != NS_DTYPE_F16 && dtype != NS_DTYPE_F32) return NS_ERR_CONFIG;
    if (((uintptr_t)d_logits & 15u) || ((ld * (int64_t)esz) & 15)) return NS_ERR_CONFIG;
    if (!d_nll && !d_entropy) return NS_OK;
    const int64_t blocks = (nrows + nsg::SC_WAVES - 1) / nsg::SC_WAVES;
    if (blocks > 0x7FFFFFFF) return NS_ERR_UNSUPPORTED;
    hipStream_t s = (hipStream_t)hip_stream;
    if (dtype == NS_DTYPE_F16)
        hipLaunchKernelGGL(nsg::score_rows_kernel<_Float16>, dim3((unsigned)blocks), dim3(64 * nsg::SC_WAVES), 0, s,
                           (const char*)d_logits, ld, nrows, V, d_labels, d_nll, d_entropy);
    else
        hipLaunchKernelGGL(nsg::score_rows_kernel<float>, dim3((unsigned)blocks), dim3(64 * nsg::SC_WAVES), 0, s,
                           (const char*)d_logits, ld, nrows, V, d_labels, d_nll, d_entropy);
    return hipGetLastError() == hipSuccess ? NS_OK : NS_ERR_HIP;
}

// Batch-invariant decode-step kernels of the batched GPT-2 forward (include/nsg_lm.h).
//
// Reference semantics: Hugging Face GPT2Block / GPT2LMHeadModel for one new token per stream
// (code_base/arithmetic.py:115-122).  What matters here beyond the semantics is that a stream's logits do not
// depend on the batch it runs in: the arithmetic decoder must reproduce the encoder's integer CDF exactly,
// and a cover encoded among B streams is revealed alone.
//
// GEMM: Y[m, n] = epi(sum_k X[m, k] * Wt[n, k] + bias[n]).  Every element is the in-order sum of SK = 1, 2
// or 4 (by K only) fp32 accumulator chains of v_mfma_f32_16x16x32_f16 over consecutive k ranges, with the
// weight row in MFMA row position n & 15 and the activation row in MFMA column position m & 15 -- in every
// kernel variant.  The variants differ only in how many elements a wave owns and how the operands reach the
// registers:
//   * gemm_direct<FM, SK>  (small batches): a wave owns 16 weight rows x 16*FM activation rows x one chain
//     and loads its fragments straight from global memory (small batches are latency- and weight-bandwidth-
//     bound, an LDS round trip would only add latency); the chains of one weight block meet in LDS;
//   * gemm_tiled<BN, BM>: a workgroup of 4 waves owns a BN x BM tile; both operands are staged into LDS with
//     global_load_lds (16 B per lane, two buffers, counted vmcnt + raw s_barrier so the next K-tile's copy
//     overlaps this one's MFMAs), rows 128 B long and XOR-swizzled by (row >> 1) & 7 in 16-B chunks so the
//     16-lane groups of a ds_read_b128 hit distinct banks (the swizzle is applied to the global SOURCE
//     address; the LDS image is written linearly by the DMA).  Workgroup ids are remapped so each XCD
//     (private L2) runs a contiguous range of tiles that share weight panels.
// The accumulator layout of the 16x16 MFMA puts four consecutive n of one m in a lane, so each lane stores
// 8 bytes (fp16) or 16 bytes (fp32) per fragment and the bias is read as 4 consecutive values.
//
// LayerNorm: one wavefront per row; per-lane sums in a fixed order, xor butterfly (every lane ends with the
// same bits); two-pass variance.  fp-contract is off for the whole library, so no FMA is formed implicitly.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nsg_coder.h"
#include "nsg_lm.h"

namespace nsg {
namespace lm {

typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 64;  // K per staged tile: 128-byte rows

__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float gelu_tanh(float x) {
    // GPT-2 gelu_new: 0.5 x (1 + tanh(u)), u = sqrt(2/pi) (x + 0.044715 x^3), evaluated as the equal
    // x * sigmoid(2u) = x / (1 + 2^(-2u log2 e)): one v_exp_f32 and one v_rcp_f32 (about 1 ulp each) instead of the
    // library tanhf (a branchy polynomial / exp / IEEE-division sequence that cost as much VALU time per 128 x 128
    // tile as the tile's MFMAs).  Relative error a few fp32 ulp before the fp16 rounding of the output; large |u|
    // saturates cleanly (exp2 -> inf gives x * 0 = -0, exp2 -> 0 gives x).
    const float u = 0.7978845608028654f * (x + 0.044715f * (x * x * x));
    const float e = __builtin_amdgcn_exp2f(u * -2.8853900817779268f);  // -2 log2(e)
    return x * __builtin_amdgcn_rcpf(1.0f + e);
}

// fp32 -> fp16 with the fp32 value pinned first: without the barrier the compiler may fold the producing
// multiply / add into the conversion (v_fma_mix*_f16: ONE rounding to fp16 instead of fp32 then fp16), and it
// does so in some kernel variants and not in others -- the tile configurations must give the same bits.
__device__ __forceinline__ f16 to_f16(float v) {
    asm volatile("" : "+v"(v));
    return (f16)v;
}

// Epilogue of one 16x16 fragment: lane holds n0..n0+3 of row m.
template <int EPI>
__device__ __forceinline__ void store4(void* Y, int64_t ldy, const f16* __restrict__ bias, int m, int n, f32x4 acc) {
    float v[4];
    if (bias) {
        const f16x4 bb = *(const f16x4*)(bias + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[r] + (float)bb[r];
    } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[r];
    }
    if constexpr (EPI == NS_LM_EPI_STORE_F32) {
        float* y = (float*)Y + (int64_t)m * ldy + n;
        *(f32x4*)y = f32x4{v[0], v[1], v[2], v[3]};
    } else {
        f16* y = (f16*)Y + (int64_t)m * ldy + n;
        f16x4 o;
        if constexpr (EPI == NS_LM_EPI_RESIDUAL) {
            const f16x4 h = *(const f16x4*)y;
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = to_f16((float)h[r] + v[r]);
        } else if constexpr (EPI == NS_LM_EPI_GELU) {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = to_f16(gelu_tanh(v[r]));
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = to_f16(v[r]);
        }
        *(f16x4*)y = o;
    }
}

// The same epilogue with its operands (bias, residual) loaded ahead: small-batch kernels issue those loads before
// the K loop, so they land during it instead of costing one more dependent memory round trip at the end.
template <int EPI>
__device__ __forceinline__ void store4_pre(void* Y, int64_t ldy, bool has_bias, f16x4 bb, f16x4 h, int m, int n,
                                           f32x4 acc) {
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = has_bias ? acc[r] + (float)bb[r] : acc[r];
    if constexpr (EPI == NS_LM_EPI_STORE_F32) {
        float* y = (float*)Y + (int64_t)m * ldy + n;
        *(f32x4*)y = f32x4{v[0], v[1], v[2], v[3]};
    } else {
        f16* y = (f16*)Y + (int64_t)m * ldy + n;
        f16x4 o;
        if constexpr (EPI == NS_LM_EPI_RESIDUAL) {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = to_f16((float)h[r] + v[r]);
        } else if constexpr (EPI == NS_LM_EPI_GELU) {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = to_f16(gelu_tanh(v[r]));
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = to_f16(v[r]);
        }
        *(f16x4*)y = o;
    }
}

// ------------------------------------------------------------------------------------------ canonical order
// The K range is cut into SK = chains(K) consecutive chains of 64-wide tiles (SK = 1 up to K = 1024, 2 up to
// 2048, else 4; tiles_per_chain = ceil(KT / SK)); each chain is ONE fp32 MFMA accumulation from zero, and the
// chains are added in order, ((c0 + c1) + c2) + c3, before the epilogue.  Every kernel variant follows this
// order, so the split is part of the result's definition, not of the tile choice -- and it lets a small batch
// spread a long-K GEMM (GPT-2's mlp c_proj: K = 4C) over SK waves per weight block.
__host__ __device__ constexpr int k_chains(int K) { return K <= 1024 ? 1 : K <= 2048 ? 2 : 4; }

// ---------------------------------------------------------------------------------------------------- direct
// Workgroup = 4 waves = (4 / SK) weight blocks x SK chains: wave w owns weight rows [16 * nb, +16) with
// nb = 4 / SK * blockIdx.x + w / SK, activation rows [16 * FM * blockIdx.y, +16 * FM) and chain w % SK; the
// fragments come straight from global memory (small batches are latency- and weight-bandwidth-bound; an LDS
// round trip would only add latency).  Chains meet in LDS and the chain-0 wave adds them in order.
template <int FM, int SK, int EPI, int NW = 4>
__global__ __launch_bounds__(64 * NW) void gemm_direct(const f16* __restrict__ X, int64_t ldx,
                                                       const f16* __restrict__ Wt, int64_t ldw,
                                                       const f16* __restrict__ bias, void* Y, int64_t ldy, int M, int N,
                                                       int K) {
    static_assert(NW % SK == 0, "a workgroup holds whole weight blocks");
    __shared__ f32x4 s_part[SK > 1 ? NW : 1][SK > 1 ? FM : 1][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nb = blockIdx.x * (NW / SK) + wave / SK;
    const int chain = wave % SK;
    const bool live = nb * 16 < N;  // uniform per wave; no early return: the chain hand-off has a barrier
    const int m0 = blockIdx.y * 16 * FM;
    const int r = lane & 15, c = lane >> 4;
    const int KT = K / 64, TPC = (KT + SK - 1) / SK;
    const int k_begin = min(chain * TPC, KT) * 64, k_end = min((chain + 1) * TPC, KT) * 64;
    const f16* wrow = Wt + (int64_t)min(nb * 16 + r, N - 1) * ldw + c * 8;
    const f16* xrow[FM];
#pragma unroll
    for (int f = 0; f < FM; ++f) xrow[f] = X + (int64_t)min(m0 + f * 16 + r, M - 1) * ldx + c * 8;
    f32x4 acc[FM];
#pragma unroll
    for (int f = 0; f < FM; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
    // epilogue operands first (bias, the residual row): in flight with the K loop's loads
    const int n = nb * 16 + 4 * c;
    const bool ep = live && n < N && (SK == 1 || chain == 0);
    f16x4 pb = {}, ph[FM];
#pragma unroll
    for (int f = 0; f < FM; ++f) ph[f] = f16x4{};
    if (ep) {
        if (bias) pb = *(const f16x4*)(bias + n);
        if constexpr (EPI == NS_LM_EPI_RESIDUAL) {
#pragma unroll
            for (int f = 0; f < FM; ++f) {
                const int m = m0 + f * 16 + r;
                if (m < M) ph[f] = *(const f16x4*)((const f16*)Y + (int64_t)m * ldy + n);
            }
        }
    }
    constexpr int U = FM == 1 ? 24 : FM == 2 ? 12 : 8;  // 32-wide k-steps per batch of loads in flight (K = 768: one)
    int k = k_begin;
    if (live) {
        for (; k + 32 * U <= k_end; k += 32 * U) {
            f16x8 a[U], b[U][FM];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                a[u] = *(const f16x8*)(wrow + k + 32 * u);
#pragma unroll
                for (int f = 0; f < FM; ++f) b[u][f] = *(const f16x8*)(xrow[f] + k + 32 * u);
            }
            // keep every load of the batch ahead of the MFMAs (the scheduler would otherwise interleave them to
            // save registers, leaving a dozen in flight: at small M each batch costs one memory round trip)
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int f = 0; f < FM; ++f) acc[f] = mfma16(a[u], b[u][f], acc[f]);
        }
        for (; k < k_end; k += 32) {
            const f16x8 a = *(const f16x8*)(wrow + k);
#pragma unroll
            for (int f = 0; f < FM; ++f) acc[f] = mfma16(a, *(const f16x8*)(xrow[f] + k), acc[f]);
        }
    }
    if constexpr (SK > 1) {
#pragma unroll
        for (int f = 0; f < FM; ++f) s_part[wave][f][lane] = acc[f];
        __syncthreads();
        if (chain != 0) return;
        for (int q = 1; q < SK; ++q)
#pragma unroll
            for (int f = 0; f < FM; ++f) acc[f] += s_part[wave + q][f][lane];
    }
    if (!ep) return;
#pragma unroll
    for (int f = 0; f < FM; ++f) {
        const int m = m0 + f * 16 + r;
        if (m < M) store4_pre<EPI>(Y, ldy, bias != nullptr, pb, ph[f], m, n, acc[f]);
    }
}

// ----------------------------------------------------------------------------------------------------- tiled
__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

template <int N_>
__device__ __forceinline__ void wait_vm() {
    static_assert(N_ >= 0 && N_ < 64, "vmcnt range");
    // s_waitcnt encoding (gfx9): vmcnt[3:0] | expcnt[6:4]=7 | lgkmcnt[11:8]=15 | vmcnt_hi[15:14]
    __builtin_amdgcn_s_waitcnt((N_ & 15) | (7 << 4) | (15 << 8) | ((N_ >> 4) << 14));
}

__device__ __forceinline__ void lds_fence_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// XCD-aware bijective remap: hardware dispatches workgroup i to XCD i % 8; give each XCD a contiguous range.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int q = nwg >> 3, rr = nwg & 7, x = bid & 7;
    return (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + (bid >> 3);
}

template <int BN, int BM, int WN, int WM, int NST, bool SPLIT, int EPI>
__global__ __launch_bounds__(64 * WN * WM) void gemm_tiled(const f16* __restrict__ X, int64_t ldx,
                                                            const f16* __restrict__ Wt, int64_t ldw,
                                                            const f16* __restrict__ bias, void* Y, int64_t ldy, int M,
                                                            int N, int K) {
    constexpr int NT = 64 * WN * WM;
    constexpr int NW = WN * WM;
    constexpr int FN = BN / (16 * WN), FM = BM / (16 * WM);
    constexpr int ROWS = BN + BM;                // staged rows per K-tile (weights first, then activations)
    constexpr int GL = ROWS * 8 / NT;            // 16-byte DMA instructions per thread per K-tile
    static_assert(ROWS * 8 % NT == 0 && BN % (16 * WN) == 0 && BM % (16 * WM) == 0 && BN % 16 == 0, "tile shape");
    static_assert(NST >= 2 && NST <= 4, "stages");
    __shared__ __attribute__((aligned(16))) char smem[NST * ROWS * 128];

    const int tiles_m = (M + BM - 1) / BM;
    const int tiles_n = (N + BN - 1) / BN;
    const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
    // grouped order: GN weight panels x every activation panel, m fastest inside a group -- the tiles an XCD
    // runs at once share a few panels of BOTH operands, so both stay in its 4 MiB L2 (m-fastest over all of M
    // would cycle the whole activation matrix through L2 once per weight panel)
    constexpr int GN = 1024 / BN;
    const int grp = t / (GN * tiles_m), within = t - grp * (GN * tiles_m);
    const int gn = min(GN, tiles_n - grp * GN);
    const int tm = within / gn, tn = grp * GN + (within - tm * gn);
    const int n0 = tn * BN, m0 = tm * BM;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wn = wave / WM, wm = wave - wn * WM;

    // staging: instruction g of wave w fills LDS rows q*8 .. q*8+7, q = g*NW + w; lane -> row q*8 + lane/8,
    // physical chunk lane%8, i.e. logical chunk (lane%8) ^ swz(row).
    const f16* src[GL];
    int lds_off[GL];
#pragma unroll
    for (int g = 0; g < GL; ++g) {
        const int q = g * NW + wave;
        const int row = q * 8 + (lane >> 3);
        const int chunk = (lane & 7) ^ swz(row);
        if (row < BN)
            src[g] = Wt + (int64_t)min(n0 + row, N - 1) * ldw + chunk * 8;
        else
            src[g] = X + (int64_t)min(m0 + row - BN, M - 1) * ldx + chunk * 8;
        lds_off[g] = q * 8 * 128;  // wave-uniform destination base; the DMA adds lane * 16
    }
    auto stage = [&](int kt, int buf) {
#pragma unroll
        for (int g = 0; g < GL; ++g)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src[g] + kt * BK),
                                             (__attribute__((address_space(3))) void*)(smem + buf * ROWS * 128 +
                                                                                       lds_off[g]),
                                             16, 0, 0);
    };

    f32x4 acc[FN][FM];
    f32x4 tot[SPLIT ? FN : 1][SPLIT ? FM : 1];  // sum of the finished chains (canonical order)
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int KT = K / BK;
    const int SK = k_chains(K), TPC = (KT + SK - 1) / SK;
    const int fr = lane & 15, fc = lane >> 4;
#pragma unroll
    for (int s0 = 0; s0 < NST - 1; ++s0)
        if (s0 < KT) stage(s0, s0);
    int buf = 0;
    for (int kt = 0; kt < KT; ++kt) {
        const int ahead = KT - 1 - kt;  // tiles after kt
        if constexpr (NST >= 3) {
            // one barrier per K-tile: wait for this thread's copies of tile kt (the NST-2 younger tiles may stay in
            // flight), then the barrier both publishes tile kt and certifies that every wave has finished reading
            // the buffer of tile kt-1, which is the one tile kt+NST-1 is copied into right after it
            if (ahead >= NST - 2) {
                wait_vm<GL * (NST - 2)>();
            } else if (NST >= 4 && ahead == 1) {
                wait_vm<GL>();
            } else {
                wait_vm<0>();
            }
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if (ahead >= NST - 1) {
                int nb = buf + NST - 1;
                nb -= nb >= NST ? NST : 0;
                stage(kt + NST - 1, nb);
            }
        } else {
            // two buffers: issue tile kt+1, then wait until tile kt's copies (this thread's) landed
            if (ahead >= 1) {
                stage(kt + 1, buf ^ 1);
                wait_vm<GL>();
            } else {
                wait_vm<0>();
            }
            __builtin_amdgcn_s_barrier();  // ... and every other wave's
            asm volatile("" ::: "memory");
        }
        if constexpr (SPLIT) {
            if (kt > 0 && kt % TPC == 0) {  // a chain ends: fold it into the running total, start the next at 0
#pragma unroll
                for (int i = 0; i < FN; ++i)
#pragma unroll
                    for (int j = 0; j < FM; ++j) {
                        tot[i][j] = kt == TPC ? acc[i][j] : tot[i][j] + acc[i][j];
                        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
                    }
            }
        }
        const char* base = smem + buf * ROWS * 128;
        f16x8 a[2][FN], b[2][FM];  // both 32-wide k-steps of the tile: every LDS read in flight at once
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int ch = kk * 4 + fc;
#pragma unroll
            for (int i = 0; i < FN; ++i) {
                const int row = wn * FN * 16 + i * 16 + fr;
                a[kk][i] = *(const f16x8*)(base + row * 128 + ((ch ^ swz(row)) << 4));
            }
#pragma unroll
            for (int j = 0; j < FM; ++j) {
                const int row = BN + wm * FM * 16 + j * 16 + fr;
                b[kk][j] = *(const f16x8*)(base + row * 128 + ((ch ^ swz(row)) << 4));
            }
        }
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = 0; i < FN; ++i)
#pragma unroll
                for (int j = 0; j < FM; ++j) acc[i][j] = mfma16(a[kk][i], b[kk][j], acc[i][j]);
        if constexpr (NST == 2) lds_fence_barrier();  // every wave is done reading this buffer before it is refilled
        buf = buf + 1 == NST ? 0 : buf + 1;
    }
    if constexpr (SPLIT) {
        if (KT > TPC) {
#pragma unroll
            for (int i = 0; i < FN; ++i)
#pragma unroll
                for (int j = 0; j < FM; ++j) acc[i][j] = tot[i][j] + acc[i][j];
        }
    }
#pragma unroll
    for (int i = 0; i < FN; ++i) {
        const int n = n0 + wn * FN * 16 + i * 16 + 4 * fc;
        if (n >= N) continue;
#pragma unroll
        for (int j = 0; j < FM; ++j) {
            const int m = m0 + wm * FM * 16 + j * 16 + fr;
            if (m < M) store4<EPI>(Y, ldy, bias, m, n, acc[i][j]);
        }
    }
}

// ------------------------------------------------------------------------------------------------ persistent
// gemm_persist<NST, SPLIT, EPI>: 128 x 128 tiles, 4 waves of 64 x 64, ONE workgroup per CU looping over the tiles
// t = g, g + G, g + 2G, ... (g = XCD-remapped id, same grouped tile order as gemm_tiled).  The LDS ring runs over
// the concatenated K-tile sequence of all of the workgroup's tiles, so the next tile's first K-tiles are in flight
// during this tile's last ones and its epilogue: at K = 768 a tile is only 12 K-tiles, and in the one-tile-per-
// workgroup kernel the pipeline fill and the epilogue of every tile were exposed.
// The waits are counted exactly: the epilogue stores go through a buffer resource whose range check drops the
// rows >= M, so every wave issues exactly FN * FM stores per tile, none of them branched around; the bias (N <=
// PB_BIAS_MAX) is staged in LDS once, so the epilogue issues no vector-memory load (a plain load in flight beside
// the LDS-DMA makes the compiler drain the whole ring with vmcnt(0)).  Requires N % 128 == 0 and the output within
// 32-bit buffer offsets (host check); every element is the same canonical MFMA chain as in gemm_tiled.
constexpr int PB_BIAS_MAX = 4096;

template <int N_>
__device__ __forceinline__ void wait_vm_le(int n) {
    // s_waitcnt vmcnt(k) for the largest multiple of 8 not above n (waiting for MORE is always safe)
    if constexpr (N_ > 0) {
        if (n >= N_) {
            wait_vm<N_>();
            return;
        }
        wait_vm_le<N_ - 8>(n);
    } else {
        wait_vm<0>();
    }
}

template <int NST, bool SPLIT, int EPI>
__global__ __launch_bounds__(256) void gemm_persist(const f16* __restrict__ X, int64_t ldx,
                                                    const f16* __restrict__ Wt, int64_t ldw,
                                                    const f16* __restrict__ bias, void* Y, int64_t ldy, int M, int N,
                                                    int K) {
    constexpr int BN = 128, BM = 128, WM = 2, NT = 256, NW = 4, FN = 4, FM = 4;
    constexpr int ROWS = BN + BM, GL = ROWS * 8 / NT, SB = ROWS * 128;
    constexpr int NSTO = FN * FM;  // epilogue stores per wave and tile
    constexpr int ESZ = EPI == NS_LM_EPI_STORE_F32 ? 4 : 2;
    static_assert(NST >= 2 && NST <= 4 && GL == 8, "ring");
    __shared__ __attribute__((aligned(16))) char smem[NST * SB + PB_BIAS_MAX * 2];
    f16* s_bias = (f16*)(smem + NST * SB);

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wn = wave / WM, wm = wave - wn * WM;
    const int fr = lane & 15, fc = lane >> 4;
    const int tiles_m = (M + BM - 1) / BM, tiles_n = N / BN, T = tiles_m * tiles_n;
    const int G = gridDim.x, g = xcd_remap(blockIdx.x, G);
    const int KT = K / BK, SK = k_chains(K), TPC = (KT + SK - 1) / SK;
    const int ntl = g < T ? (T - 1 - g) / G + 1 : 0;
    const int S = ntl * KT;  // K-tiles this workgroup runs, all tiles concatenated

    if (bias) {
        for (int i = threadIdx.x * 8; i < N; i += NT * 8) *(f16x8*)(s_bias + i) = *(const f16x8*)(bias + i);
    }
    __syncthreads();  // no LDS-DMA in flight yet

    auto origin = [&](int i, int& n0, int& m0) {
        constexpr int GN = 1024 / BN;
        const int t = g + i * G;
        const int grp = t / (GN * tiles_m), within = t - grp * (GN * tiles_m);
        const int gn = min(GN, tiles_n - grp * GN);
        const int tm = within / gn;
        n0 = (grp * GN + (within - tm * gn)) * BN;
        m0 = tm * BM;
    };
    // staging: instruction q of the wave fills LDS rows (q * NW + wave) * 8 .. +7; q < GL/2 are weight rows
    const int srow = lane >> 3;
    auto stage = [&](int i, int kt, int buf) {
        int n0, m0;
        origin(i, n0, m0);
        char* dst = smem + buf * SB;
#pragma unroll
        for (int q = 0; q < GL; ++q) {
            const int qq = q * NW + wave;
            const int row = qq * 8 + srow;
            const int chunk = (lane & 7) ^ swz(row);
            const f16* src = q < GL / 2 ? Wt + (int64_t)(n0 + row) * ldw
                                        : X + (int64_t)min(m0 + row - BN, M - 1) * ldx;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + chunk * 8 + kt * BK),
                                             (__attribute__((address_space(3))) void*)(dst + qq * 8 * 128), 16, 0, 0);
        }
    };

    // output resource: offsets past M rows fail the range check and the store is dropped
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(Y, (short)0, (int)((int64_t)M * ldy * ESZ), 0x00020000);

    f32x4 acc[FN][FM];
    f32x4 tot[SPLIT ? FN : 1][SPLIT ? FM : 1];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    int is_i = 0, is_k = 0, is_n = 0;  // next stage to issue: tile, K-tile, sequence number
    auto issue = [&]() {
        stage(is_i, is_k, is_n % NST);
        ++is_n;
        if (++is_k == KT) {
            is_k = 0;
            ++is_i;
        }
    };
#pragma unroll
    for (int p = 0; p < NST - 1; ++p)
        if (is_n < S) issue();

    int ci = 0, ck = 0;
    unsigned epmask = 0;  // bit d: the iteration d + 1 back ran an epilogue
    for (int s = 0; s < S; ++s) {
        // younger than stage s's copies: stages s+1 .. s+NST-2 and the stores of epilogues since its issue
        const int ahead = min(NST - 2, S - 1 - s);
        const int nep = __builtin_popcount(epmask & ((1u << (NST - 1)) - 1u));
        wait_vm_le<56>(GL * ahead + NSTO * nep);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (is_n < S) issue();  // into the buffer read one iteration ago (every wave is past this barrier)
        if constexpr (SPLIT) {
            if (ck > 0 && ck % TPC == 0) {
#pragma unroll
                for (int i = 0; i < FN; ++i)
#pragma unroll
                    for (int j = 0; j < FM; ++j) {
                        tot[i][j] = ck == TPC ? acc[i][j] : tot[i][j] + acc[i][j];
                        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
                    }
            }
        }
        const char* base = smem + (s % NST) * SB;
        f16x8 a[2][FN], b[2][FM];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int ch = kk * 4 + fc;
#pragma unroll
            for (int i = 0; i < FN; ++i) {
                const int row = wn * FN * 16 + i * 16 + fr;
                a[kk][i] = *(const f16x8*)(base + row * 128 + ((ch ^ swz(row)) << 4));
            }
#pragma unroll
            for (int j = 0; j < FM; ++j) {
                const int row = BN + wm * FM * 16 + j * 16 + fr;
                b[kk][j] = *(const f16x8*)(base + row * 128 + ((ch ^ swz(row)) << 4));
            }
        }
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = 0; i < FN; ++i)
#pragma unroll
                for (int j = 0; j < FM; ++j) acc[i][j] = mfma16(a[kk][i], b[kk][j], acc[i][j]);
        epmask <<= 1;
        if (ck == KT - 1) {
            if constexpr (SPLIT) {
                if (KT > TPC) {
#pragma unroll
                    for (int i = 0; i < FN; ++i)
#pragma unroll
                        for (int j = 0; j < FM; ++j) acc[i][j] = tot[i][j] + acc[i][j];
                }
            }
            int n0, m0;
            origin(ci, n0, m0);
#pragma unroll
            for (int i = 0; i < FN; ++i) {
                const int n = n0 + wn * FN * 16 + i * 16 + 4 * fc;
                f16x4 bb = f16x4{};
                if (bias) bb = *(const f16x4*)(s_bias + n);
#pragma unroll
                for (int j = 0; j < FM; ++j) {
                    const int m = m0 + wm * FM * 16 + j * 16 + fr;
                    float v[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = bias ? acc[i][j][r] + (float)bb[r] : acc[i][j][r];
                    const int off = (int)(((int64_t)m * ldy + n) * ESZ);
                    if constexpr (EPI == NS_LM_EPI_STORE_F32) {
                        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                        const u32x4 w = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                                         __float_as_uint(v[3])};
                        __builtin_amdgcn_raw_buffer_store_b128(w, rs, off, 0, 0);
                    } else {
                        f16x4 o;
#pragma unroll
                        for (int r = 0; r < 4; ++r) o[r] = EPI == NS_LM_EPI_GELU ? to_f16(gelu_tanh(v[r])) : to_f16(v[r]);
                        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), rs, off, 0, 0);
                    }
                    acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
                }
            }
            epmask |= 1u;
            ck = 0;
            ++ci;
        } else {
            ++ck;
        }
    }
}

// ----------------------------------------------------------------------------------------------------- big
// gemm_big<EPI>: 256 x 256 tiles, 8 waves (4 along N x 2 along M) of 64 x 128, K <= 1024 (one K chain), one
// workgroup per CU (two 64 KiB LDS buffers).  Why this shape: per K-tile a wave issues 8 LDS-DMA pieces
// whatever the tile, but a 64 x 128 wave tile gives it 64 MFMAs to hide them behind (a 128 x 128 tile's 64 x 64
// wave tiles: 32), and the operand bytes per MFMA out of LDS halve.  One barrier per K-tile: tile kt + 1's
// copies are issued in the first half of tile kt's MFMAs (into the buffer every wave finished reading before the
// previous barrier) and waited for at its end.  Ragged N and M: rows clamped on load, columns / rows >= N / M
// not stored.
template <int EPI>
__global__ __launch_bounds__(512) void gemm_big(const f16* __restrict__ X, int64_t ldx, const f16* __restrict__ Wt,
                                                int64_t ldw, const f16* __restrict__ bias, void* Y, int64_t ldy,
                                                int M, int N, int K) {
    constexpr int BN = 256, BM = 256, NW = 8, WM = 2, FN = 4, FM = 8, FH = FM / 2;
    constexpr int ROWS = BN + BM, GL = ROWS * 8 / (64 * NW), SB = ROWS * 128;
    static_assert(GL == 8, "staging");
    __shared__ __attribute__((aligned(16))) char smem[2 * SB];

    const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
    const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
    constexpr int GN = 4;  // weight panels per group (1024 rows)
    const int grp = t / (GN * tiles_m), within = t - grp * (GN * tiles_m);
    const int gn = min(GN, tiles_n - grp * GN);
    const int tm = within / gn, tn = grp * GN + (within - tm * gn);
    const int n0 = tn * BN, m0 = tm * BM;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wn = wave / WM, wm = wave - wn * WM;
    const int fr = lane & 15, fc = lane >> 4;

    const f16* src[GL];
    int lds_off[GL];
#pragma unroll
    for (int q = 0; q < GL; ++q) {
        const int qq = q * NW + wave;
        const int row = qq * 8 + (lane >> 3);
        const int chunk = (lane & 7) ^ swz(row);
        src[q] = (q < GL / 2 ? Wt + (int64_t)min(n0 + row, N - 1) * ldw
                             : X + (int64_t)min(m0 + row - BN, M - 1) * ldx) + chunk * 8;
        lds_off[q] = qq * 8 * 128;
    }
    auto piece = [&](int q, int kt, int buf) {
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src[q] + kt * BK),
                                         (__attribute__((address_space(3))) void*)(smem + buf * SB + lds_off[q]), 16,
                                         0, 0);
    };

    f32x4 acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int KT = K / BK;
#pragma unroll
    for (int q = 0; q < GL; ++q) piece(q, 0, 0);
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    for (int kt = 0; kt < KT; ++kt) {
        const int buf = kt & 1;
        const bool nxt = kt + 1 < KT;
        const char* base = smem + buf * SB;
        f16x8 a[2][FN], b0[2][FH], b1[2][FH];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int ch = kk * 4 + fc;
#pragma unroll
            for (int i = 0; i < FN; ++i) {
                const int row = wn * FN * 16 + i * 16 + fr;
                a[kk][i] = *(const f16x8*)(base + row * 128 + ((ch ^ swz(row)) << 4));
            }
#pragma unroll
            for (int j = 0; j < FH; ++j) {
                const int row = BN + wm * FM * 16 + j * 16 + fr;
                b0[kk][j] = *(const f16x8*)(base + row * 128 + ((ch ^ swz(row)) << 4));
            }
        }
        if (nxt) {
#pragma unroll
            for (int q = 0; q < GL; ++q) piece(q, kt + 1, buf ^ 1);
        }
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int ch = kk * 4 + fc;
#pragma unroll
            for (int j = 0; j < FH; ++j) {
                const int row = BN + wm * FM * 16 + (FH + j) * 16 + fr;
                b1[kk][j] = *(const f16x8*)(base + row * 128 + ((ch ^ swz(row)) << 4));
            }
        }
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = 0; i < FN; ++i)
#pragma unroll
                for (int j = 0; j < FH; ++j) acc[i][j] = mfma16(a[kk][i], b0[kk][j], acc[i][j]);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = 0; i < FN; ++i)
#pragma unroll
                for (int j = 0; j < FH; ++j) acc[i][FH + j] = mfma16(a[kk][i], b1[kk][j], acc[i][FH + j]);
        if (nxt) wait_vm<0>();
        lds_fence_barrier();  // tile kt + 1 landed everywhere; every wave is done reading buffer kt & 1
    }
#pragma unroll
    for (int i = 0; i < FN; ++i) {
        const int n = n0 + wn * FN * 16 + i * 16 + 4 * fc;
        if (n >= N) continue;
#pragma unroll
        for (int j = 0; j < FM; ++j) {
            const int m = m0 + wm * FM * 16 + j * 16 + fr;
            if (m < M) store4<EPI>(Y, ldy, bias, m, n, acc[i][j]);
        }
    }
}

// ------------------------------------------------------------------------------------------------ ping-pong
// gemm_pp<EPI>: the 256 x 256 tile of gemm_big with its two wave groups (g = 0: activation rows 0..127 of the
// tile, g = 1: rows 128..255; each 4 waves of 64 weight rows x 128 rows) run half a K-tile apart, so that on every
// SIMD (one wave of each group) one wave issues MFMAs while the other reads its next fragments and stages the
// next K-tile (ping-pong; the MFMA wave runs at raised priority).  Time is cut into slots by workgroup barriers;
// group 0 runs L(t) (LDS reads of K-tile t, staging of t + 1) in slot 2t+1 and M(t) (64 MFMAs) in slot 2t+2,
// group 1 one slot later (one extra barrier up front, group 0 one extra at the end).  Staging: group 0 copies the
// weight panel and its activation rows (12 pieces per wave), group 1 its activation rows (4 pieces).  Hazards,
// by slot: a wave ends every L slot with lgkmcnt(0) (its reads of buffer t & 1 are complete at that barrier) and
// every M slot with vmcnt(0) (its copies of t + 1 have landed): K-tile t+1 goes into the buffer last read in slot
// 2t (group 1's L(t-1)), and is read from slot 2t+3 (group 0) / 2t+4 (group 1) on, after the barriers that follow
// its writers' waits.  One K chain (K <= 1024); ragged N / M clamped on load, not stored.
// BN = 192 (FN = 3): the same kernel with 48 weight rows per wave -- GPT-2's c_fc at B = 4,096 is then 16 x 16 =
// 256 tiles, one per CU, where 256-wide panels leave a quarter of the CUs idle (192 tiles).
template <int EPI, int BN = 256>
__global__ __launch_bounds__(512) void gemm_pp(const f16* __restrict__ X, int64_t ldx, const f16* __restrict__ Wt,
                                               int64_t ldw, const f16* __restrict__ bias, void* Y, int64_t ldy, int M,
                                               int N, int K) {
    static_assert(BN == 256 || BN == 192, "weight panel");
    constexpr int BM = 256, FN = BN / 64, FM = 8, SB = (BN + BM) * 128;
    constexpr int WP = BN / 32;  // weight pieces (32 rows each) staged by group 0
    __shared__ __attribute__((aligned(16))) char smem[2 * SB];

    const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
    const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
    constexpr int GN = 4;
    const int grp = t / (GN * tiles_m), within = t - grp * (GN * tiles_m);
    const int gn = min(GN, tiles_n - grp * GN);
    const int tm = within / gn, tn = grp * GN + (within - tm * gn);
    const int n0 = tn * BN, m0 = tm * BM;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = wave >> 2, wn = wave & 3;
    const int fr = lane & 15, fc = lane >> 4;
    const int lr = lane >> 3;
    // piece q of a wave covers LDS rows qq * 8 + lr; (qq * 8 >> 1) & 7 == (wn * 4) & 7 for every q, so the swizzle
    // chunk is the same for all of a wave's pieces
    const int chunk = (lane & 7) ^ ((wn * 4 + (lane >> 4)) & 7);
    auto stage = [&](int kt, int buf) {
        char* dst = smem + buf * SB;
        // the twelve row pointers are recomputed per call (an opaque copy of the lane's row keeps the compiler from
        // hoisting them out of the K loop: 24 live VGPRs would spill next to the 96 fragment and 128 accumulator
        // registers)
        int r8 = wn * 8 + lr;
        asm volatile("" : "+v"(r8));
        if (g == 0) {
#pragma unroll
            for (int q = 0; q < WP + 4; ++q) {
                const f16* p = q < WP ? Wt + (int64_t)min(n0 + q * 32 + r8, N - 1) * ldw
                                      : X + (int64_t)min(m0 + (q - WP) * 32 + r8, M - 1) * ldx;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p + chunk * 8 + kt * BK),
                                                 (__attribute__((address_space(3))) void*)(dst + (q * 4 + wn) * 1024),
                                                 16, 0, 0);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const f16* p = X + (int64_t)min(m0 + 128 + q * 32 + r8, M - 1) * ldx;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p + chunk * 8 + kt * BK),
                                                 (__attribute__((address_space(3))) void*)(dst + ((BN + 128) / 8 + q * 4 + wn) * 1024),
                                                 16, 0, 0);
            }
        }
    };
    auto barrier = []() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };

    f32x4 acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int KT = K / BK;
    stage(0, 0);
    wait_vm<0>();
    barrier();
    if (g == 1) barrier();  // group 1 starts one slot late
    for (int kt = 0; kt < KT; ++kt) {
        const int buf = kt & 1;
        const char* base = smem + buf * SB;
        // ---- L slot: this K-tile's fragments, the next K-tile's copies
        f16x8 a[2][FN], b[2][FM];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int ch = kk * 4 + fc;
#pragma unroll
            for (int i = 0; i < FN; ++i) {
                const int row = wn * FN * 16 + i * 16 + fr;
                a[kk][i] = *(const f16x8*)(base + row * 128 + ((ch ^ swz(row)) << 4));
            }
#pragma unroll
            for (int j = 0; j < FM; ++j) {
                const int row = BN + g * FM * 16 + j * 16 + fr;
                b[kk][j] = *(const f16x8*)(base + row * 128 + ((ch ^ swz(row)) << 4));
            }
        }
        if (kt + 1 < KT) stage(kt + 1, buf ^ 1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier();
        // ---- M slot
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = 0; i < FN; ++i)
#pragma unroll
                for (int j = 0; j < FM; ++j) acc[i][j] = mfma16(a[kk][i], b[kk][j], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
        if (kt + 1 < KT) wait_vm<0>();
        barrier();
    }
    if (g == 0) barrier();  // same barrier count for both groups
#pragma unroll
    for (int i = 0; i < FN; ++i) {
        const int n = n0 + wn * FN * 16 + i * 16 + 4 * fc;
        if (n >= N) continue;
#pragma unroll
        for (int j = 0; j < FM; ++j) {
            const int m = m0 + g * FM * 16 + j * 16 + fr;
            if (m < M) store4<EPI>(Y, ldy, bias, m, n, acc[i][j]);
        }
    }
}

// ------------------------------------------------------------------------------------------------ chains
// gemm_chains<SK, EPI> (round 5): the SK = k_chains(K) = 2 or 4 K chains of the canonical order computed side by
// side instead of one after the other.  A workgroup of 4 * SK waves owns one 64 x 64 tile; wave group c (4 waves of
// 32 x 32, laid out as in gemm_tiled<64, 64, 2, 2>) runs chain c -- K-tiles [c * TPC, min((c + 1) * TPC, KT)) --
// through its own two-stage LDS ring, and the chains meet in LDS, where group 0 adds them in order,
// ((c0 + c1) + c2) + c3, and stores.  The same MFMA chains and the same additions as gemm_tiled's sequential SPLIT
// form, so the bits are the same; what changes is how many waves a long-K GEMM with few output tiles keeps busy
// (GPT-2-medium's mlp c_proj at B = 1,024: 256 tiles, one 4-wave workgroup per CU in the sequential form).
template <int SK, int EPI>
__global__ __launch_bounds__(256 * SK) void gemm_chains(const f16* __restrict__ X, int64_t ldx,
                                                         const f16* __restrict__ Wt, int64_t ldw,
                                                         const f16* __restrict__ bias, void* Y, int64_t ldy, int M,
                                                         int N, int K) {
    constexpr int BN = 64, BM = 64, WM = 2, FN = 2, FM = 2;
    constexpr int ROWS = BN + BM, GL = ROWS * 8 / 256;  // 16-byte DMA pieces per thread per K-tile (4)
    constexpr int SB = ROWS * 128;                      // one stage: 16 KiB
    static_assert(SK == 2 || SK == 4, "chains");
    __shared__ __attribute__((aligned(16))) char smem[SK * 2 * SB];

    const int tiles_m = (M + BM - 1) / BM;
    const int tiles_n = (N + BN - 1) / BN;
    const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
    constexpr int GN = 1024 / BN;
    const int grp = t / (GN * tiles_m), within = t - grp * (GN * tiles_m);
    const int gn = min(GN, tiles_n - grp * GN);
    const int tm = within / gn, tn = grp * GN + (within - tm * gn);
    const int n0 = tn * BN, m0 = tm * BM;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int c = wave >> 2, ww = wave & 3;  // chain, wave within the chain group
    const int wn = ww / WM, wm = ww - wn * WM;
    char* ring = smem + c * 2 * SB;

    const f16* src[GL];
    int lds_off[GL];
#pragma unroll
    for (int g = 0; g < GL; ++g) {
        const int q = g * 4 + ww;
        const int row = q * 8 + (lane >> 3);
        const int chunk = (lane & 7) ^ swz(row);
        if (row < BN)
            src[g] = Wt + (int64_t)min(n0 + row, N - 1) * ldw + chunk * 8;
        else
            src[g] = X + (int64_t)min(m0 + row - BN, M - 1) * ldx + chunk * 8;
        lds_off[g] = q * 8 * 128;
    }
    auto stage = [&](int kt, int buf) {
#pragma unroll
        for (int g = 0; g < GL; ++g)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src[g] + kt * BK),
                                             (__attribute__((address_space(3))) void*)(ring + buf * SB + lds_off[g]),
                                             16, 0, 0);
    };

    f32x4 acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int KT = K / BK, TPC = (KT + SK - 1) / SK;
    const int k0 = c * TPC, nk = max(0, min(k0 + TPC, KT) - k0);  // wave-uniform
    const int fr = lane & 15, fc = lane >> 4;
    if (nk > 0) stage(k0, 0);
    int buf = 0;
    for (int i = 0; i < TPC; ++i) {  // every chain runs TPC rounds: the workgroup barriers stay uniform
        if (i + 1 < nk) {
            stage(k0 + i + 1, buf ^ 1);
            wait_vm<GL>();
        } else {
            wait_vm<0>();
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (i < nk) {
            const char* base = ring + buf * SB;
            f16x8 a[2][FN], b[2][FM];
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                const int ch = kk * 4 + fc;
#pragma unroll
                for (int ii = 0; ii < FN; ++ii) {
                    const int row = wn * FN * 16 + ii * 16 + fr;
                    a[kk][ii] = *(const f16x8*)(base + row * 128 + ((ch ^ swz(row)) << 4));
                }
#pragma unroll
                for (int j = 0; j < FM; ++j) {
                    const int row = BN + wm * FM * 16 + j * 16 + fr;
                    b[kk][j] = *(const f16x8*)(base + row * 128 + ((ch ^ swz(row)) << 4));
                }
            }
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                for (int ii = 0; ii < FN; ++ii)
#pragma unroll
                    for (int j = 0; j < FM; ++j) acc[ii][j] = mfma16(a[kk][ii], b[kk][j], acc[ii][j]);
        }
        lds_fence_barrier();  // every wave is done reading this buffer before it is refilled
        buf ^= 1;
    }
    // chains 1.. hand their accumulators to group 0 through LDS (the rings are idle: every copy landed, every read
    // completed before the last barrier); lane-fastest layout, conflict-free
    float* red = (float*)smem;
    if (c > 0) {
#pragma unroll
        for (int ii = 0; ii < FN; ++ii)
#pragma unroll
            for (int j = 0; j < FM; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    red[((((c - 1) * 4 + ww) * 16) + (ii * FM + j) * 4 + r) * 64 + lane] = acc[ii][j][r];
    }
    __syncthreads();
    if (c != 0) return;
    f32x4 tot[FN][FM];
#pragma unroll
    for (int ii = 0; ii < FN; ++ii)
#pragma unroll
        for (int j = 0; j < FM; ++j) tot[ii][j] = acc[ii][j];
#pragma unroll
    for (int cc = 1; cc < SK; ++cc) {
#pragma unroll
        for (int ii = 0; ii < FN; ++ii)
#pragma unroll
            for (int j = 0; j < FM; ++j) {
                f32x4 v;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = red[((((cc - 1) * 4 + ww) * 16) + (ii * FM + j) * 4 + r) * 64 + lane];
                tot[ii][j] = tot[ii][j] + v;  // ((c0 + c1) + c2) + c3, as gemm_tiled's SPLIT form
            }
    }
#pragma unroll
    for (int ii = 0; ii < FN; ++ii) {
        const int n = n0 + wn * FN * 16 + ii * 16 + 4 * fc;
        if (n >= N) continue;
#pragma unroll
        for (int j = 0; j < FM; ++j) {
            const int m = m0 + wm * FM * 16 + j * 16 + fr;
            if (m < M) store4<EPI>(Y, ldy, bias, m, n, tot[ii][j]);
        }
    }
}

// ------------------------------------------------------------------------------------------------ layernorm
constexpr int LN_MAXV = 8;  // f16x4 vectors per lane: C <= 2048

__device__ __forceinline__ float wave_sum(float s) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off);
    return s;
}

// Normalise the row held in x[] (NV4 = C/4 vectors, lane holds vectors lane, lane+64, ...), write fp16.
__device__ __forceinline__ void ln_row(float (&x)[LN_MAXV][4], int NV4, int C, const f16* __restrict__ w,
                                       const f16* __restrict__ b, f16* __restrict__ y, float eps) {
    const int lane = threadIdx.x & 63;
    // the affine parameters do not depend on the row: load them before the reductions (one round trip, not two)
    f16x4 wv[LN_MAXV], bv[LN_MAXV];
#pragma unroll
    for (int v = 0; v < LN_MAXV; ++v) {
        const int i = lane + 64 * v;
        if (i < NV4) {
            wv[v] = *(const f16x4*)(w + 4 * i);
            bv[v] = *(const f16x4*)(b + 4 * i);
        }
    }
    float s = 0.0f;
#pragma unroll
    for (int v = 0; v < LN_MAXV; ++v)
        if (lane + 64 * v < NV4)
#pragma unroll
            for (int e = 0; e < 4; ++e) s += x[v][e];
    const float mean = wave_sum(s) / (float)C;
    float q = 0.0f;
#pragma unroll
    for (int v = 0; v < LN_MAXV; ++v)
        if (lane + 64 * v < NV4)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float d = x[v][e] - mean;
                q += d * d;
            }
    const float var = wave_sum(q) / (float)C;
    const float rstd = 1.0f / sqrtf(var + eps);
#pragma unroll
    for (int v = 0; v < LN_MAXV; ++v) {
        const int i = lane + 64 * v;
        if (i < NV4) {
            f16x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = to_f16(((x[v][e] - mean) * rstd) * (float)wv[v][e] + (float)bv[v][e]);
            *(f16x4*)(y + 4 * i) = o;
        }
    }
}

// counter (optional): the decode step's device-side cache length, advanced by one thread here -- ln_f runs after
// every attention layer of the step has read it, and a separate add kernel would cost one more launch per token
// (graph replays at B = 1 are launch-latency bound)
__global__ __launch_bounds__(256) void layernorm_kernel(const f16* __restrict__ X, int64_t ldx,
                                                        const f16* __restrict__ w, const f16* __restrict__ b,
                                                        f16* __restrict__ Y, int64_t ldy, int M, int C, float eps,
                                                        int32_t* __restrict__ counter, int32_t* __restrict__ row_counter) {
    if (counter && blockIdx.x == 0 && threadIdx.x == 0) *counter += 1;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const int lane = threadIdx.x & 63, NV4 = C >> 2;
    if (row_counter && lane == 0) row_counter[row] += 1;  // per-stream cache lengths (paged decode step)
    const f16* xr = X + (int64_t)row * ldx;
    float x[LN_MAXV][4];
#pragma unroll
    for (int v = 0; v < LN_MAXV; ++v) {
        const int i = lane + 64 * v;
        if (i < NV4) {
            const f16x4 t = *(const f16x4*)(xr + 4 * i);
#pragma unroll
            for (int e = 0; e < 4; ++e) x[v][e] = (float)t[e];
        }
    }
    ln_row(x, NV4, C, w, b, Y + (int64_t)row * ldy, eps);
}

__global__ __launch_bounds__(256) void embed_ln_kernel(const int32_t* __restrict__ tokens, const f16* __restrict__ wte,
                                                       const f16* __restrict__ wpe, int V, int n_positions, int L,
                                                       const int32_t* __restrict__ dL, f16* __restrict__ H,
                                                       int64_t ldh, const f16* __restrict__ w,
                                                       const f16* __restrict__ b, f16* __restrict__ A, int64_t lda,
                                                       int M, int C, float eps, int seq_T,
                                                       const int32_t* __restrict__ rowL) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    if (dL) L = *dL;
    if (rowL) L = rowL[row];  // per-stream cache lengths (paged decode step, slot refill)
    // decode step: pos = L mod n_positions (code_base/arithmetic.py:44-48, L >= 0); whole sequences (seq_T > 0):
    // row b*T + t is position t (the first call's default positions)
    const int pos = seq_T > 0 ? (row % seq_T) % n_positions : L % n_positions;
    const int lane = threadIdx.x & 63, NV4 = C >> 2;
    const int tok = tokens[row];
    const bool ok = tok >= 0 && tok < V;
    const f16* er = wte + (int64_t)(ok ? tok : 0) * C;
    const f16* pr = wpe + (int64_t)pos * C;
    f16* hr = H + (int64_t)row * ldh;
    float x[LN_MAXV][4];
#pragma unroll
    for (int v = 0; v < LN_MAXV; ++v) {
        const int i = lane + 64 * v;
        if (i < NV4) {
            const f16x4 te = *(const f16x4*)(er + 4 * i);
            const f16x4 tp = *(const f16x4*)(pr + 4 * i);
            f16x4 h;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                h[e] = ok ? (f16)((float)te[e] + (float)tp[e]) : (f16)__builtin_nanf("");
                x[v][e] = (float)h[e];
            }
            *(f16x4*)(hr + 4 * i) = h;
        }
    }
    ln_row(x, NV4, C, w, b, A + (int64_t)row * lda, eps);
}


// ------------------------------------------------------------------------------------------- LN + direct GEMM
// LayerNorm fused into the small-batch GEMM (M <= 16, K <= 1024: one chain, the shapes auto_cfg gives the direct
// kernel): every workgroup normalises the M activation rows itself -- wave w rows w, w + 4, ... with ln_row's
// arithmetic, so the values are bit-identical to layernorm_kernel's -- into an LDS tile, and its MFMA activation
// fragments come from there; the weight fragments (the whole K of the wave's 16 rows, <= 32 x 16 B per lane) are
// issued before the normalisation so their latency hides it.  One launch per LN + GEMM pair instead of two: at
// B = 1 the decode step is a chain of ~85 launch-latency-bound kernels.
constexpr int LNG_MAXK = 1024;
template <int EPI, int NW = 4>
__global__ __launch_bounds__(64 * NW) void gemm_direct_ln(const f16* __restrict__ X, int64_t ldx,
                                                          const f16* __restrict__ lw, const f16* __restrict__ lb,
                                                          float eps, const f16* __restrict__ Wt, int64_t ldw,
                                                          const f16* __restrict__ bias, void* Y, int64_t ldy, int M,
                                                          int N, int K) {
    __shared__ __attribute__((aligned(16))) f16 sA[16][LNG_MAXK + 8];  // +16 B per row: conflict-free b128 reads
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nb = blockIdx.x * NW + wave;
    const bool live = nb * 16 < N;
    const int r = lane & 15, c = lane >> 4;
    const int KS = K / 32;  // 32-wide k-steps
    const f16* wrow = Wt + (int64_t)min(nb * 16 + r, N - 1) * ldw + c * 8;
    f16x8 a[LNG_MAXK / 32];
    if (live) {
#pragma unroll
        for (int u = 0; u < LNG_MAXK / 32; ++u)
            if (u < KS) a[u] = *(const f16x8*)(wrow + 32 * u);
    }
    const int n = nb * 16 + 4 * c;
    const bool ep = live && n < N;
    f16x4 pb = {}, ph = {};
    if (ep) {
        if (bias) pb = *(const f16x4*)(bias + n);
        if constexpr (EPI == NS_LM_EPI_RESIDUAL) {
            if (r < M) ph = *(const f16x4*)((const f16*)Y + (int64_t)r * ldy + n);
        }
    }
    const int NV4 = K >> 2;
    for (int row = wave; row < M; row += NW) {
        const f16* xr = X + (int64_t)row * ldx;
        float x[LN_MAXV][4];
#pragma unroll
        for (int v = 0; v < LN_MAXV; ++v) {
            const int i = lane + 64 * v;
            if (i < NV4) {
                const f16x4 t = *(const f16x4*)(xr + 4 * i);
#pragma unroll
                for (int e = 0; e < 4; ++e) x[v][e] = (float)t[e];
            }
        }
        ln_row(x, NV4, K, lw, lb, &sA[row][0], eps);
    }
    __syncthreads();
    if (!ep) return;
    const f16* arow = &sA[min(r, M - 1)][c * 8];
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < LNG_MAXK / 32; ++u)
        if (u < KS) acc = mfma16(a[u], *(const f16x8*)(arow + 32 * u), acc);
    if (r < M) store4_pre<EPI>(Y, ldy, bias != nullptr, pb, ph, r, n, acc);
}

}  // namespace lm
}  // namespace nsg

using namespace nsg::lm;

// Tile configurations (ns_lm_gemm_config).  All of them compute every element by the same MFMA chain, so the
// choice is a speed choice only (tests check equality across configurations bit for bit).
enum GemmCfg {
    CFG_DIRECT16 = 0, CFG_DIRECT32, CFG_DIRECT64,     // 16 weight rows x 16/32/64 activation rows per wave
    CFG_T64_2, CFG_T64_3,                             // 64 x 64 tile, 4 waves, 2 / 3 LDS stages
    CFG_T128_2, CFG_T128_3, CFG_T128_4,               // 128 x 128, 4 waves (64 x 64 each)
    CFG_T256x128_2, CFG_T256x128_3,                   // 256 weight rows x 128 activation rows, 8 waves
    CFG_T128x256_2,                                   // 128 x 256, 8 waves
    CFG_T64_4,                                        // 64 x 64, 4 stages
    CFG_T128x64_3,                                    // 128 weight rows x 64 activation rows, 4 waves, 3 stages
    CFG_B256,                                         // 256 x 256, 8 waves of 64 x 128 (K <= 1024)
    CFG_P128_2, CFG_P128_3, CFG_P128_4,               // persistent 128 x 128, 2 / 3 / 4 stages (2 / 1 / 1 per CU)
    CFG_PP256,                                        // 256 x 256, two ping-pong wave groups (K <= 1024)
    CFG_PP192,                                        // 192 weight rows x 256, the same ping-pong kernel
    CFG_C64,                                          // 64 x 64, the K chains side by side (K > 1024; round 5)
    CFG_COUNT
};

static int cu_count() {
    static int n = 0;
    if (n == 0) {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
            n = v;
        else
            n = 256;
    }
    return n;
}

// gemm_persist's preconditions (else the persistent configurations run the 128 x 128 tiled kernel: same bits)
static bool persist_ok(int epi, const void* bias, int64_t ldy, int M, int N) {
    const int64_t esz = epi == NS_LM_EPI_STORE_F32 ? 4 : 2;
    return epi != NS_LM_EPI_RESIDUAL && N % 128 == 0 && (!bias || N <= PB_BIAS_MAX) &&
           ((int64_t)M + 128) * ldy * esz < ((int64_t)1 << 31);
}

#ifndef NSG_DIRECT_NW
#define NSG_DIRECT_NW 1  // waves per workgroup of the direct kernels when one chain per weight block (K <= 1024)
#endif

template <int FM, int EPI>
static void launch_direct(const f16* x, int64_t ldx, const f16* wt, int64_t ldw, const f16* bias, void* y,
                          int64_t ldy, int M, int N, int K, hipStream_t st) {
    const int nbk = N / 16, my = (M + 16 * FM - 1) / (16 * FM);
    constexpr int NW1 = NSG_DIRECT_NW;
    switch (k_chains(K)) {
        case 1:
            hipLaunchKernelGGL((gemm_direct<FM, 1, EPI, NW1>), dim3((nbk + NW1 - 1) / NW1, my), dim3(64 * NW1), 0, st,
                               x, ldx, wt, ldw, bias, y, ldy, M, N, K);
            break;
        case 2:
            hipLaunchKernelGGL((gemm_direct<FM, 2, EPI>), dim3((nbk + 1) / 2, my), dim3(256), 0, st, x, ldx, wt, ldw,
                               bias, y, ldy, M, N, K);
            break;
        default:
            hipLaunchKernelGGL((gemm_direct<FM, 4, EPI>), dim3(nbk, my), dim3(256), 0, st, x, ldx, wt, ldw, bias, y,
                               ldy, M, N, K);
            break;
    }
}

template <int EPI>
static void launch_cfg(int cfg, const f16* x, int64_t ldx, const f16* wt, int64_t ldw, const f16* bias, void* y,
                       int64_t ldy, int M, int N, int K, hipStream_t st) {
    auto tiles = [&](int bn, int bm) { return dim3((unsigned)(((M + bm - 1) / bm) * (long)((N + bn - 1) / bn))); };
    const bool split = k_chains(K) > 1;
    switch (cfg) {
#define NSG_DIRECT(FMv) launch_direct<FMv, EPI>(x, ldx, wt, ldw, bias, y, ldy, M, N, K, st)
#define NSG_TILED(BNv, BMv, WNv, WMv, NSTv)                                                                     \
    if (split)                                                                                                  \
        hipLaunchKernelGGL((gemm_tiled<BNv, BMv, WNv, WMv, NSTv, true, EPI>), tiles(BNv, BMv), dim3(64 * WNv * WMv), \
                           0, st, x, ldx, wt, ldw, bias, y, ldy, M, N, K);                                      \
    else                                                                                                        \
        hipLaunchKernelGGL((gemm_tiled<BNv, BMv, WNv, WMv, NSTv, false, EPI>), tiles(BNv, BMv),                 \
                           dim3(64 * WNv * WMv), 0, st, x, ldx, wt, ldw, bias, y, ldy, M, N, K)
        case CFG_DIRECT16: NSG_DIRECT(1); break;
        case CFG_DIRECT32: NSG_DIRECT(2); break;
        case CFG_DIRECT64: NSG_DIRECT(4); break;
        case CFG_T64_2: NSG_TILED(64, 64, 2, 2, 2); break;
        case CFG_T64_3: NSG_TILED(64, 64, 2, 2, 3); break;
        case CFG_T128_2: NSG_TILED(128, 128, 2, 2, 2); break;
        case CFG_T128_3: NSG_TILED(128, 128, 2, 2, 3); break;
        case CFG_T128_4: NSG_TILED(128, 128, 2, 2, 4); break;
        case CFG_T256x128_2: NSG_TILED(256, 128, 4, 2, 2); break;
        case CFG_T256x128_3: NSG_TILED(256, 128, 4, 2, 3); break;
        case CFG_T128x256_2: NSG_TILED(128, 256, 2, 4, 2); break;
        case CFG_T64_4: NSG_TILED(64, 64, 2, 2, 4); break;
        case CFG_T128x64_3: NSG_TILED(128, 64, 2, 2, 3); break;
        case CFG_B256:
            if (split) {  // one K chain only (K <= 1024); else the 128 x 128 tiles (same bits)
                NSG_TILED(128, 128, 2, 2, 2);
            } else {
                hipLaunchKernelGGL((gemm_big<EPI>), tiles(256, 256), dim3(512), 0, st, x, ldx, wt, ldw, bias, y, ldy,
                                   M, N, K);
            }
            break;
        case CFG_PP256:
            if (split) {
                NSG_TILED(128, 128, 2, 2, 2);
            } else {
                hipLaunchKernelGGL((gemm_pp<EPI>), tiles(256, 256), dim3(512), 0, st, x, ldx, wt, ldw, bias, y, ldy, M,
                                   N, K);
            }
            break;
        case CFG_PP192:
            if (split) {
                NSG_TILED(128, 128, 2, 2, 2);
            } else {
                hipLaunchKernelGGL((gemm_pp<EPI, 192>), tiles(192, 256), dim3(512), 0, st, x, ldx, wt, ldw, bias, y,
                                   ldy, M, N, K);
            }
            break;
        case CFG_C64: {
            const int sk = k_chains(K);
            if (sk == 4)
                hipLaunchKernelGGL((gemm_chains<4, EPI>), tiles(64, 64), dim3(1024), 0, st, x, ldx, wt, ldw, bias, y, ldy,
                                   M, N, K);
            else if (sk == 2)
                hipLaunchKernelGGL((gemm_chains<2, EPI>), tiles(64, 64), dim3(512), 0, st, x, ldx, wt, ldw, bias, y, ldy,
                                   M, N, K);
            else
                NSG_TILED(64, 64, 2, 2, 2);  // one chain: the plain 64 x 64 kernel (same bits)
            break;
        }
        case CFG_P128_2:
        case CFG_P128_3:
        case CFG_P128_4: {
            if (!persist_ok(EPI, bias, ldy, M, N)) {
                NSG_TILED(128, 128, 2, 2, 2);
                break;
            }
            const int T = ((M + 127) / 128) * (N / 128);
            const int G = min(T, cu_count() * (cfg == CFG_P128_2 ? 2 : 1));
            if constexpr (EPI != NS_LM_EPI_RESIDUAL) {
#define NSG_PERSIST(NSTv)                                                                                        \
    if (split)                                                                                                   \
        hipLaunchKernelGGL((gemm_persist<NSTv, true, EPI>), dim3(G), dim3(256), 0, st, x, ldx, wt, ldw, bias, y, \
                           ldy, M, N, K);                                                                        \
    else                                                                                                         \
        hipLaunchKernelGGL((gemm_persist<NSTv, false, EPI>), dim3(G), dim3(256), 0, st, x, ldx, wt, ldw, bias, y, \
                           ldy, M, N, K)
                if (cfg == CFG_P128_2) {
                    NSG_PERSIST(2);
                } else if (cfg == CFG_P128_3) {
                    NSG_PERSIST(3);
                } else {
                    NSG_PERSIST(4);
                }
#undef NSG_PERSIST
            }
            break;
        }
#undef NSG_DIRECT
#undef NSG_TILED
        default: break;
    }
}

// Automatic choice by shape (speed only: every configuration gives the same bits).  From the per-config sweep
// at M = 16 ... 4096 on GPT-2 shapes (profiles/lmprobe_r02j_*.jsonl): 64 x 64 LDS tiles for the short-K GEMMs
// from M = 16 up; direct waves for the long-K (split) GEMM up to M = 256, where spreading the chains over
// waves beats tiling; 128 x 128 tiles only for the vocabulary-wide head at large M.
static int auto_cfg(int M, int N, int K) {
    const bool split = k_chains(K) > 1;
    if (M <= 16) return (N >= 8192 && !split) ? CFG_T64_2 : CFG_DIRECT16;
    if (split && M <= 256) return M <= 64 ? CFG_DIRECT16 : M <= 128 ? CFG_DIRECT32 : CFG_DIRECT64;
    // the vocabulary-wide head: 256 x 256 ping-pong tiles below B = 2048 (GPT-2-medium B = 1024: 786 vs 740
    // TFLOP/s), 128 x 128 above (B = 4096: 752 vs 726; profiles/r04/lmprobe_r04aa_*.jsonl)
    if (N >= 8192 && M >= 512) return (!split && M < 2048) ? CFG_PP256 : CFG_T128_2;
    // B >= 4096, K <= 1024, wide N: the ping-pong kernel, with 192- or 256-wide weight panels, whichever needs fewer
    // panel-rows of work per CU (GPT-2's c_fc: 256 tiles of 192 = one per CU, 644 vs 579 TFLOP/s for 192 tiles of
    // 256; c_attn 556 vs 487 on 64 x 64 tiles; profiles/r04/lmprobe_r04ag_*.jsonl).  GPT-2-medium's c_fc (N = 4096)
    // at B = 1024 on 128 x 64 tiles (506 vs 471); the other shapes and smaller batches stay on 64 x 64 tiles.
    if (!split && M >= 4096 && N >= 2048) {
        const long cu = cu_count(), tm = (M + 255) / 256;
        const long w256 = (tm * ((N + 255) / 256) + cu - 1) / cu * 256;
        const long w192 = (tm * ((N + 191) / 192) + cu - 1) / cu * 192;
        return w192 < w256 ? CFG_PP192 : CFG_PP256;
    }
    if (!split && M >= 1024 && N >= 4096) return CFG_T128x64_3;
    // long K (two or four chains) with few 64 x 64 tiles: the chains side by side (GPT-2-medium's mlp c_proj at
    // B = 1,024: 416 vs 292 TFLOP/s sequential, hipBLASLt 365); with more tiles than two per CU the sequential
    // form keeps more workgroups in flight (GPT-2's at B = 4,096: 540 vs 423; profiles/r05/lmprobe_r05k_*.jsonl)
    if (split && (long)((M + 63) / 64) * ((N + 63) / 64) <= 2L * cu_count()) return CFG_C64;
    return CFG_T64_2;
}

static int gemm_checked(const void* d_x, int64_t ldx, const void* d_wt, int64_t ldw, const void* d_bias, void* d_y,
                        int64_t ldy, int M, int N, int K, int epilogue, int cfg, void* hip_stream) {
    if (!d_x || !d_wt || !d_y || M <= 0 || N <= 0 || K <= 0) return NS_ERR_CONFIG;
    if (K % 64 || N % 16) return NS_ERR_UNSUPPORTED;
    if (ldx < K || ldw < K || ldy < N) return NS_ERR_CONFIG;
    const uintptr_t al = (uintptr_t)d_x | (uintptr_t)d_wt | (uintptr_t)d_y | (uintptr_t)(d_bias ? d_bias : d_x);
    if ((al & 15u) || (ldx & 7) || (ldw & 7) || (ldy & 3)) return NS_ERR_CONFIG;
    if ((int64_t)((M + 15) / 16) * ((N + 15) / 16) > 0x7FFFFFFF) return NS_ERR_UNSUPPORTED;
    if (cfg < 0) cfg = auto_cfg(M, N, K);
    if (cfg >= CFG_COUNT) return NS_ERR_CONFIG;
    const f16 *x = (const f16*)d_x, *wt = (const f16*)d_wt, *b = (const f16*)d_bias;
    const hipStream_t st = (hipStream_t)hip_stream;
    switch (epilogue) {
        case NS_LM_EPI_STORE: launch_cfg<NS_LM_EPI_STORE>(cfg, x, ldx, wt, ldw, b, d_y, ldy, M, N, K, st); break;
        case NS_LM_EPI_GELU: launch_cfg<NS_LM_EPI_GELU>(cfg, x, ldx, wt, ldw, b, d_y, ldy, M, N, K, st); break;
        case NS_LM_EPI_RESIDUAL: launch_cfg<NS_LM_EPI_RESIDUAL>(cfg, x, ldx, wt, ldw, b, d_y, ldy, M, N, K, st); break;
        case NS_LM_EPI_STORE_F32: launch_cfg<NS_LM_EPI_STORE_F32>(cfg, x, ldx, wt, ldw, b, d_y, ldy, M, N, K, st); break;
        default: return NS_ERR_CONFIG;
    }
    return hipGetLastError() == hipSuccess ? NS_OK : NS_ERR_HIP;
}

extern "C" int ns_lm_gemm(const void* d_x, int64_t ldx, const void* d_wt, int64_t ldw, const void* d_bias, void* d_y,
                          int64_t ldy, int M, int N, int K, int epilogue, void* hip_stream) {
    return gemm_checked(d_x, ldx, d_wt, ldw, d_bias, d_y, ldy, M, N, K, epilogue, -1, hip_stream);
}

extern "C" int ns_lm_gemm_config(const void* d_x, int64_t ldx, const void* d_wt, int64_t ldw, const void* d_bias,
                                 void* d_y, int64_t ldy, int M, int N, int K, int epilogue, int config,
                                 void* hip_stream) {
    return gemm_checked(d_x, ldx, d_wt, ldw, d_bias, d_y, ldy, M, N, K, epilogue, config, hip_stream);
}

extern "C" int ns_lm_gemm_configs(void) { return CFG_COUNT; }

extern "C" int ns_lm_layernorm_count(const void* d_x, int64_t ldx, const void* d_w, const void* d_b, void* d_y,
                                     int64_t ldy, int M, int C, float eps, int32_t* d_counter, void* hip_stream) {
    if (!d_x || !d_w || !d_b || !d_y || M <= 0 || C <= 0) return NS_ERR_CONFIG;
    if (C % 4 || C > 256 * LN_MAXV) return NS_ERR_UNSUPPORTED;
    const uintptr_t al = (uintptr_t)d_x | (uintptr_t)d_w | (uintptr_t)d_b | (uintptr_t)d_y;
    if ((al & 7u) || (ldx & 3) || (ldy & 3) || ldx < C || ldy < C || ((uintptr_t)d_counter & 3u)) return NS_ERR_CONFIG;
    hipLaunchKernelGGL(layernorm_kernel, dim3((M + 3) / 4), dim3(256), 0, (hipStream_t)hip_stream, (const f16*)d_x,
                       ldx, (const f16*)d_w, (const f16*)d_b, (f16*)d_y, ldy, M, C, eps, d_counter, nullptr);
    return hipGetLastError() == hipSuccess ? NS_OK : NS_ERR_HIP;
}

extern "C" int ns_lm_layernorm(const void* d_x, int64_t ldx, const void* d_w, const void* d_b, void* d_y, int64_t ldy,
                               int M, int C, float eps, void* hip_stream) {
    return ns_lm_layernorm_count(d_x, ldx, d_w, d_b, d_y, ldy, M, C, eps, nullptr, hip_stream);
}

extern "C" int ns_lm_ln_gemm(const void* d_x, int64_t ldx, const void* d_lw, const void* d_lb, float eps,
                             const void* d_wt, int64_t ldw, const void* d_bias, void* d_y, int64_t ldy, int M, int N,
                             int K, int epilogue, void* d_a, int64_t lda, void* hip_stream) {
    if (!d_x || !d_lw || !d_lb || !d_wt || !d_y || M <= 0 || N <= 0 || K <= 0) return NS_ERR_CONFIG;
    const bool fused = M <= 16 && K <= LNG_MAXK && K % 64 == 0 && N % 16 == 0 && auto_cfg(M, N, K) == CFG_DIRECT16;
    if (!fused) {  // the two kernels, same bits
        if (!d_a) return NS_ERR_CONFIG;
        const int rc = ns_lm_layernorm(d_x, ldx, d_lw, d_lb, d_a, lda, M, K, eps, hip_stream);
        if (rc != NS_OK) return rc;
        return gemm_checked(d_a, lda, d_wt, ldw, d_bias, d_y, ldy, M, N, K, epilogue, -1, hip_stream);
    }
    if (ldx < K || ldw < K || ldy < N) return NS_ERR_CONFIG;
    const uintptr_t al = (uintptr_t)d_x | (uintptr_t)d_wt | (uintptr_t)d_y | (uintptr_t)(d_bias ? d_bias : d_x) |
                         (uintptr_t)d_lw | (uintptr_t)d_lb;
    if ((al & 15u) || (ldx & 7) || (ldw & 7) || (ldy & 3)) return NS_ERR_CONFIG;
    const f16 *x = (const f16*)d_x, *wt = (const f16*)d_wt, *b = (const f16*)d_bias, *lw = (const f16*)d_lw,
              *lb = (const f16*)d_lb;
    const hipStream_t st = (hipStream_t)hip_stream;
    constexpr int NW1 = NSG_DIRECT_NW;
    const dim3 grid((N / 16 + NW1 - 1) / NW1), blk(64 * NW1);
    switch (epilogue) {
        case NS_LM_EPI_STORE:
            hipLaunchKernelGGL((gemm_direct_ln<NS_LM_EPI_STORE, NW1>), grid, blk, 0, st, x, ldx, lw, lb, eps, wt, ldw, b,
                               d_y, ldy, M, N, K);
            break;
        case NS_LM_EPI_GELU:
            hipLaunchKernelGGL((gemm_direct_ln<NS_LM_EPI_GELU, NW1>), grid, blk, 0, st, x, ldx, lw, lb, eps, wt, ldw, b,
                               d_y, ldy, M, N, K);
            break;
        case NS_LM_EPI_RESIDUAL:
            hipLaunchKernelGGL((gemm_direct_ln<NS_LM_EPI_RESIDUAL, NW1>), grid, blk, 0, st, x, ldx, lw, lb, eps, wt, ldw,
                               b, d_y, ldy, M, N, K);
            break;
        case NS_LM_EPI_STORE_F32:
            hipLaunchKernelGGL((gemm_direct_ln<NS_LM_EPI_STORE_F32, NW1>), grid, blk, 0, st, x, ldx, lw, lb, eps, wt,
                               ldw, b, d_y, ldy, M, N, K);
            break;
        default: return NS_ERR_CONFIG;
    }
    return hipGetLastError() == hipSuccess ? NS_OK : NS_ERR_HIP;
}

extern "C" int ns_lm_embed_ln(const int32_t* d_tokens, const void* d_wte, const void* d_wpe, int V, int n_positions,
                              int L, const int32_t* d_L, void* d_h, int64_t ldh, const void* d_w, const void* d_b,
                              void* d_a, int64_t lda, int M, int C, float eps, void* hip_stream) {
    if (!d_tokens || !d_wte || !d_wpe || !d_h || !d_w || !d_b || !d_a || M <= 0 || C <= 0 || V <= 0 ||
        n_positions <= 0 || (!d_L && L < 0))
        return NS_ERR_CONFIG;
    if (C % 4 || C > 256 * LN_MAXV) return NS_ERR_UNSUPPORTED;
    const uintptr_t al = (uintptr_t)d_wte | (uintptr_t)d_wpe | (uintptr_t)d_h | (uintptr_t)d_w | (uintptr_t)d_b |
                         (uintptr_t)d_a;
    if ((al & 7u) || (ldh & 3) || (lda & 3) || ldh < C || lda < C) return NS_ERR_CONFIG;
    hipLaunchKernelGGL(embed_ln_kernel, dim3((M + 3) / 4), dim3(256), 0, (hipStream_t)hip_stream, d_tokens,
                       (const f16*)d_wte, (const f16*)d_wpe, V, n_positions, L, d_L, (f16*)d_h, ldh, (const f16*)d_w,
                       (const f16*)d_b, (f16*)d_a, lda, M, C, eps, 0, nullptr);
    return hipGetLastError() == hipSuccess ? NS_OK : NS_ERR_HIP;
}

extern "C" int ns_lm_embed_seq_ln(const int32_t* d_tokens, const void* d_wte, const void* d_wpe, int V,
                                  int n_positions, int T, void* d_h, int64_t ldh, const void* d_w, const void* d_b,
                                  void* d_a, int64_t lda, int M, int C, float eps, void* hip_stream) {
    if (!d_tokens || !d_wte || !d_wpe || !d_h || !d_w || !d_b || !d_a || M <= 0 || C <= 0 || V <= 0 ||
        n_positions <= 0 || T <= 0 || M % T)
        return NS_ERR_CONFIG;
    if (C % 4 || C > 256 * LN_MAXV) return NS_ERR_UNSUPPORTED;
    const uintptr_t al = (uintptr_t)d_wte | (uintptr_t)d_wpe | (uintptr_t)d_h | (uintptr_t)d_w | (uintptr_t)d_b |
                         (uintptr_t)d_a;
    if ((al & 7u) || (ldh & 3) || (lda & 3) || ldh < C || lda < C) return NS_ERR_CONFIG;
    hipLaunchKernelGGL(embed_ln_kernel, dim3((M + 3) / 4), dim3(256), 0, (hipStream_t)hip_stream, d_tokens,
                       (const f16*)d_wte, (const f16*)d_wpe, V, n_positions, 0, nullptr, (f16*)d_h, ldh,
                       (const f16*)d_w, (const f16*)d_b, (f16*)d_a, lda, M, C, eps, T, nullptr);
    return hipGetLastError() == hipSuccess ? NS_OK : NS_ERR_HIP;
}

extern "C" int ns_lm_embed_ln_rows(const int32_t* d_tokens, const void* d_wte, const void* d_wpe, int V, int n_positions,
                                   const int32_t* d_lens, void* d_h, int64_t ldh, const void* d_w, const void* d_b,
                                   void* d_a, int64_t lda, int M, int C, float eps, void* hip_stream) {
    if (!d_tokens || !d_wte || !d_wpe || !d_lens || !d_h || !d_w || !d_b || !d_a || M <= 0 || C <= 0 || V <= 0 ||
        n_positions <= 0)
        return NS_ERR_CONFIG;
    if (C % 4 || C > 256 * LN_MAXV) return NS_ERR_UNSUPPORTED;
    const uintptr_t al = (uintptr_t)d_wte | (uintptr_t)d_wpe | (uintptr_t)d_h | (uintptr_t)d_w | (uintptr_t)d_b |
                         (uintptr_t)d_a;
    if ((al & 7u) || (ldh & 3) || (lda & 3) || ldh < C || lda < C || ((uintptr_t)d_lens & 3u)) return NS_ERR_CONFIG;
    hipLaunchKernelGGL(embed_ln_kernel, dim3((M + 3) / 4), dim3(256), 0, (hipStream_t)hip_stream, d_tokens,
                       (const f16*)d_wte, (const f16*)d_wpe, V, n_positions, 0, nullptr, (f16*)d_h, ldh, (const f16*)d_w,
                       (const f16*)d_b, (f16*)d_a, lda, M, C, eps, 0, d_lens);
    return hipGetLastError() == hipSuccess ? NS_OK : NS_ERR_HIP;
}

extern "C" int ns_lm_layernorm_rows(const void* d_x, int64_t ldx, const void* d_w, const void* d_b, void* d_y,
                                    int64_t ldy, int M, int C, float eps, int32_t* d_lens, void* hip_stream) {
    if (!d_x || !d_w || !d_b || !d_y || !d_lens || M <= 0 || C <= 0) return NS_ERR_CONFIG;
    if (C % 4 || C > 256 * LN_MAXV) return NS_ERR_UNSUPPORTED;
    const uintptr_t al = (uintptr_t)d_x | (uintptr_t)d_w | (uintptr_t)d_b | (uintptr_t)d_y;
    if ((al & 7u) || (ldx & 3) || (ldy & 3) || ldx < C || ldy < C || ((uintptr_t)d_lens & 3u)) return NS_ERR_CONFIG;
    hipLaunchKernelGGL(layernorm_kernel, dim3((M + 3) / 4), dim3(256), 0, (hipStream_t)hip_stream, (const f16*)d_x,
                       ldx, (const f16*)d_w, (const f16*)d_b, (f16*)d_y, ldy, M, C, eps, nullptr, d_lens);
    return hipGetLastError() == hipSuccess ? NS_OK : NS_ERR_HIP;
}

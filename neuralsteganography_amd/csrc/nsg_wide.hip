// nsg_wide.hip -- the coder step for top-k beyond the single-pass kernel's LDS candidate buffer
// (e.g. the api default topk 50,000 at precision 16, or the message->bits mode, precision 40 / topk 60,000,
// code_base/run_single.py:52-54), and the src rank coder.  Same canonical arithmetic as the single-pass kernel
// and the oracle.
//
// Coder step (ns_encode_step / ns_decode_step / ns_sample_step with K > the single-pass limit):
//   1. wide_scan_kernel    (512 threads/stream): pass 1 over the row -> max, second max, fast-sum interval;
//                          pass 2 -> every id that can clear the 1/R cutoff, plus the top two, as 49-bit
//                          (value desc, id asc) keys in LDS; <= 5,632 keys: LDS sort + the canonical tail
//                          (fast_tail).  Other streams: keys to global memory, stream id onto a work list.
//   2. rocprim::segmented_radix_sort_keys_desc : descending sort of the listed streams' keys (> 5,632 keys)
//   3. wide_cdf_kernel     (1024 threads/block, over the work list): cutoff, canonical sums (the exact row sum
//                          when the fast-sum interval is ambiguous), rint, int64 scan, overfill, selection,
//                          interval update
// Rank coder (ns_rank_*_step): wide_stats_kernel (wave per stream) -> wide_collect_kernel (blocks per chunk,
// every valid id) -> the device-wide sort -> wide_rank_kernel.
// An id left out of the collection has e_i < S_lo/R <= S/R, i.e. p_i < 1/R for certain, so the first rank
// below the cutoff lies inside the collected prefix or right after it.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <rocprim/device/device_segmented_radix_sort.hpp>

#include "nsg_common.h"
#include "nsg_host.h"

#pragma clang fp contract(off)

namespace nsg {

constexpr int WIDE_THREADS = 1024;
constexpr int WIDE_ROUND = 8192;  // doubles staged in LDS per round (64 KiB)
constexpr int COLLECT_CHUNK = 4096;

// 49-bit wide keys: ord(value) << 17 | (0x1FFFF - id); ids < 2^17
__device__ __forceinline__ uint64_t wkey(float x, uint32_t j) {
    return ((uint64_t)ord32(x) << 17) | (uint64_t)(0x1FFFFu - j);
}
__device__ __forceinline__ uint32_t wkey_id(uint64_t k) { return 0x1FFFFu - (uint32_t)(k & 0x1FFFFu); }
__device__ __forceinline__ float wkey_val(uint64_t k) { return unord32((uint32_t)(k >> 17)); }

// ------------------------------------------------------------------------------------------ pass 1
template <typename T, bool DECODE>
__global__ __launch_bounds__(WPB* WAVE) void wide_stats_kernel(StepParams p, WideStat* ws, unsigned int* count) {
    constexpr int W = Elem<T>::W;
    constexpr int TS = WAVE * W;
    const int lane = threadIdx.x & (WAVE - 1);
    const int b = __builtin_amdgcn_readfirstlane(blockIdx.x * WPB + (int)(threadIdx.x / WAVE));
    if (b >= p.B) return;
    const ns_stream_state st = p.state[b];
    bool active = !(st.flags & NS_ST_DONE);
    if (!DECODE && !p.sample && active && st.bit_pos >= p.nbits[b]) {
        if (lane == 0 && !(p.flags & NS_STEP_FINISH_SENT)) p.state[b].flags = st.flags | NS_ST_DONE;
        active = false;
    }
    if (DECODE && p.active && !p.active[b]) active = false;
    if (!active) {
        if (lane == 0) {
            ws[b].active = 0;
            count[b] = 0;
        }
        return;
    }
    const int V = p.V;
    const char* rowc = (const char*)p.logits + (int64_t)b * p.ld * (int64_t)sizeof(T);
    const RowReader rd(rowc, (uint32_t)(p.ld * (int64_t)sizeof(T)));
    const int ntiles = (V + TS - 1) / TS;
    float r = 0.0f, m1 = -__builtin_inff(), m2 = -__builtin_inff();
    double acc64 = 0.0, b64 = 0.0, u64 = 0.0;
    const bool stats = p.stats != nullptr;
    int bi = 0, next_ban = p.nbanned > 0 ? p.banned[0] : 0x7FFFFFFF;
    for (int tile = 0; tile < ntiles; ++tile) {
        float x[W];
        Elem<T>::unpack(rd.vec(tile * WAVE + lane), x);
        const int j0 = (tile * WAVE + lane) * W;
        if (tile == ntiles - 1) {
#pragma unroll
            for (int q = 0; q < W; ++q)
                if (j0 + q >= V) x[q] = -__builtin_inff();
        }
        while (next_ban < (tile + 1) * TS) {
#pragma unroll
            for (int q = 0; q < W; ++q)
                if (j0 + q == next_ban) x[q] = -__builtin_inff();
            ++bi;
            next_ban = bi < p.nbanned ? p.banned[bi] : 0x7FFFFFFF;
        }
        if (tile == 0) {
            float mx = x[0];
#pragma unroll
            for (int q = 1; q < W; ++q) mx = fmaxf(mx, x[q]);
            r = wave_max(mx);
            if (r == -__builtin_inff()) r = 0.0f;
        }
        float a = 0.0f, bb = 0.0f, uu = 0.0f;
#pragma unroll
        for (int q = 0; q < W; ++q) {
            const float dx = fmaxf(x[q] - r, -3.0e38f);
            const float e = __builtin_amdgcn_exp2f(dx * p.c32);
            a += e;
            if (stats) {
                bb += e * dx;
                uu += __builtin_amdgcn_exp2f(dx * L2E_F);
            }
            m2 = fmaxf(m2, fminf(m1, x[q]));
            m1 = fmaxf(m1, x[q]);
        }
        acc64 += (double)a;
        b64 += (double)bb;
        u64 += (double)uu;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const float o1 = __shfl_xor(m1, off), o2 = __shfl_xor(m2, off);
        m2 = fmaxf(fminf(m1, o1), fmaxf(m2, o2));
        m1 = fmaxf(m1, o1);
    }
    const double S_r = wave_sum_butterfly(acc64);
    const double B_r = wave_sum_butterfly(b64);
    const double U_r = wave_sum_butterfly(u64);
    double Sf = 0.0, S_lo = 0.0, S_hi = 0.0;
    const bool ok = fast_sum_interval(S_r, r, (double)(m1 + 0.0f), p.c32, p.inv_temp, W, Sf, S_lo, S_hi);
    if (lane == 0) {
        WideStat w;
        w.m = m1;
        w.m2 = m2;
        w.r = r;
        w.active = 1;
        w.S_lo = S_lo;
        w.S_hi = S_hi;
        w.S_fast = Sf;
        w.exact = (ok && !(p.flags & NS_STEP_FORCE_EXACT_SUM)) ? 0u : 1u;
        w.pad = 0;
        w.S_r = S_r;
        w.B_r = B_r;
        w.U_r = U_r;
        ws[b] = w;
        count[b] = 0;
    }
}

// ------------------------------------------------------------------------------------------ pass 2
template <typename T>
__global__ __launch_bounds__(256) void wide_collect_kernel(StepParams p, const WideStat* ws, uint64_t* keys,
                                                           unsigned int* count, int cap) {
    constexpr int W = Elem<T>::W;
    constexpr int PER_THREAD = COLLECT_CHUNK / 256;  // ids per thread
    const int b = blockIdx.y;
    const WideStat w = ws[b];
    if (!w.active) return;
    const int V = p.V;
    const int lane = threadIdx.x & (WAVE - 1);
    const ns_stream_state st = p.state[b];
    const double thr = 1.0 / (double)(st.hi - st.lo);
    float xt;
    if (p.rank) {
        xt = -__builtin_inff();  // the rank coder ranks every id
    } else if (p.sample) {
        // sampler support e_i >= 2^-60  <=>  x >= m + temp * ln(2^-60); widened (extra ids are harmless)
        const double temp = 1.0 / p.inv_temp;
        const double t = (double)w.m - temp * 41.58883083359672;
        xt = (float)(t - 1.0e-4 * (1.0 + fabs((double)w.m) + temp * 41.58883083359672));
    } else if (w.exact) {
        xt = -__builtin_inff();  // collect every valid id
    } else {
        // e(x) >= S_lo/R  <=>  x >= m + temp * ln(S_lo/R); widened generously (extra ids are harmless)
        const double temp = 1.0 / p.inv_temp;
        const double L = log(w.S_lo * thr);
        const double t = (double)w.m + temp * L;
        xt = (float)(t - 1.0e-4 * (1.0 + fabs((double)w.m) + fabs(temp * L)));
    }
    xt = fminf(xt, w.m2);  // at least the top two ids (k >= 2)
    const char* rowc = (const char*)p.logits + (int64_t)b * p.ld * (int64_t)sizeof(T);
    const RowReader rd(rowc, (uint32_t)(p.ld * (int64_t)sizeof(T)));
    const int base_id = blockIdx.x * COLLECT_CHUNK;
    // all loads first (NV in flight per lane), then ONE counter atomic per wave for the wave's whole chunk
    // (the per-stream counter is shared by every block of the row: fewer atomics = less serialisation)
    constexpr int NV = PER_THREAD / W;
    float x[NV][W];
#pragma unroll
    for (int i = 0; i < NV; ++i) Elem<T>::unpack(rd.vec((base_id + (i * 256 + (int)threadIdx.x) * W) / W), x[i]);
    uint64_t msk[NV][W];
    int tot = 0;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int j0 = base_id + (i * 256 + (int)threadIdx.x) * W;
#pragma unroll
        for (int q = 0; q < W; ++q) {
            const int j = j0 + q;
            const bool take = j < V && !is_banned(p, j) && x[i][q] >= xt;
            msk[i][q] = ballot(take);
            tot += popc64(msk[i][q]);
        }
    }
    // one counter atomic per block: wave totals through LDS, wave bases = block base + earlier waves' totals
    __shared__ unsigned int s_tot[256 / WAVE];
    __shared__ unsigned int s_base;
    const int wv = (int)threadIdx.x / WAVE;
    if (lane == 0) s_tot[wv] = (unsigned int)tot;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned int all = 0;
        for (int i = 0; i < 256 / WAVE; ++i) all += s_tot[i];
        s_base = all ? atomicAdd(&count[b], all) : 0u;
    }
    __syncthreads();
    if (tot == 0) return;
    unsigned int base = s_base;
    for (int i = 0; i < wv; ++i) base += s_tot[i];
    int off = 0;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int j0 = base_id + (i * 256 + (int)threadIdx.x) * W;
#pragma unroll
        for (int q = 0; q < W; ++q) {
            if ((msk[i][q] >> lane) & 1ull)
                keys[(int64_t)b * cap + base + off + lanes_below(msk[i][q])] = wkey(x[i][q], (uint32_t)(j0 + q));
            off += popc64(msk[i][q]);
        }
    }
}

// segments for the device-wide sort: only the streams with more than `small` keys (the rest are sorted in LDS by
// wide_fast_kernel; small = 0 sorts every segment)
__global__ void wide_offsets_kernel(int B, int cap, const WideStat* ws, const unsigned int* count,
                                    unsigned int* begin, unsigned int* end, unsigned int small,
                                    unsigned int* todo) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (todo && b == 0) todo[0] = 0u;
    if (b < B) {
        const unsigned int n = ws[b].active ? count[b] : 0u;
        begin[b] = (unsigned int)(b * cap);
        // more keys than the LDS sort holds, or keys collected by the one-pass kernel's fallback sweep (pad)
        end[b] = (unsigned int)(b * cap) + ((n > small || (ws[b].active && ws[b].pad)) ? n : 0u);
    }
}

// ------------------------------------------------------------------------------------------ pass 4
// the next P payload bits (LSB-first bytes) as an MSB-first integer, zero-padded past the end: one bit per lane
// and a ballot (every lane of the wave must be active); the loads are independent, not a P-long chain
__device__ __forceinline__ uint64_t payload_window(const StepParams& p, int b, int64_t bit_pos) {
    const int lane = (int)(threadIdx.x & (WAVE - 1));
    const int64_t bp = bit_pos + lane;
    uint32_t bit = 0u;
    if (lane < p.P && bp < p.nbits[b]) bit = (p.payload[(int64_t)b * p.payload_stride + (bp >> 3)] >> (bp & 7)) & 1u;
    return __builtin_bitreverse64(ballot(bit != 0u)) >> (64 - p.P);
}

// block helpers (1024 threads = 16 waves)
__device__ __forceinline__ int block_min_int(int v, int* sm) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = min(v, __shfl_xor(v, off));
    __syncthreads();
    if (lane == 0) sm[w] = v;
    __syncthreads();
    int r = sm[0];
    for (int i = 1; i < WIDE_THREADS / 64; ++i) r = min(r, sm[i]);
    __syncthreads();
    return r;
}

__device__ __forceinline__ int64_t block_excl_scan(int64_t v, int64_t* sm, int64_t& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t inc = wave_incl_scan(v, lane);
    __syncthreads();
    if (lane == 63) sm[w] = inc;
    __syncthreads();
    int64_t before = 0, all = 0;
    for (int i = 0; i < WIDE_THREADS / 64; ++i) {
        if (i < w) before += sm[i];
        all += sm[i];
    }
    __syncthreads();
    total = all;
    return before + inc - v;
}

// canonical butterfly over 64 lane partials held in sm64[0..63] (thread l < 64 owns lane l)
__device__ __forceinline__ double block_canonical_butterfly(double* sm64) {
    for (int off = 32; off >= 1; off >>= 1) {
        double t = 0.0;
        if (threadIdx.x < 64) t = sm64[threadIdx.x] + sm64[threadIdx.x ^ off];
        __syncthreads();
        if (threadIdx.x < 64) sm64[threadIdx.x] = t;
        __syncthreads();
    }
    return sm64[0];
}

template <typename T, int NT = WIDE_THREADS, int ROUND = WIDE_ROUND>
__device__ double block_exact_row_sum(const StepParams& p, const char* rowc, double m, double* ebuf, double* sm64) {
    // canonical order: id j -> lane (j>>2)&63, per-lane increasing; exps computed in parallel per round; the
    // next round's logits are loaded into registers before this round's ordered chain runs (a second LDS
    // buffer to overlap the chain with the next round's exps measured no faster).  NT threads, ROUND ids per
    // round staged as doubles in ebuf.
    static_assert(ROUND % NT == 0 && ROUND % 256 == 0, "round shape");
    constexpr int PT = ROUND / NT;
    double acc = 0.0;
    float xv[PT];
    auto load_round = [&](int base) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < PT; ++u) {
            const int j = base + u * NT + (int)threadIdx.x;
            xv[u] = j < p.V ? Elem<T>::load1(rowc, j) : 0.0f;
        }
    };
    load_round(0);
    for (int base = 0; base < p.V; base += ROUND) {
        double* eb = ebuf;
#pragma unroll
        for (int u = 0; u < PT; ++u) {
            const int i = u * NT + (int)threadIdx.x;
            const int j = base + i;
            double e = 0.0;
            if (j < p.V && !is_banned(p, j)) e = exp_canon(((double)(xv[u] + 0.0f) - m) * p.inv_temp);
            eb[i] = e;
        }
        if (base + ROUND < p.V) load_round(base + ROUND);
        __syncthreads();
        if (threadIdx.x < 64) {
            // groups of this round in increasing order: g = base/4 + g_local, lane = g & 63; four groups' loads
            // issued ahead of their (ordered) adds
            const int g0 = base / 4;
            int gl = ((int)threadIdx.x - g0 % 64 + 64) % 64;
            for (; gl + 3 * 64 < ROUND / 4; gl += 4 * 64) {
                double t[16];
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int q = 0; q < 4; ++q) t[4 * u + q] = eb[4 * (gl + 64 * u) + q];
#pragma unroll
                for (int v = 0; v < 16; ++v) acc += t[v];
            }
            for (; gl < ROUND / 4; gl += 64) {
#pragma unroll
                for (int q = 0; q < 4; ++q) acc += eb[4 * gl + q];
            }
        }
        __syncthreads();
    }
    if (threadIdx.x < 64) sm64[threadIdx.x] = acc;
    __syncthreads();
    return block_canonical_butterfly(sm64);
}

// block sum of one double per thread (statistics only: order not canonical)
__device__ __forceinline__ double block_sum(double v, double* sm64) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    __syncthreads();
    if (lane == 0) sm64[w] = v;
    __syncthreads();
    double r = 0.0;
    for (int i = 0; i < WIDE_THREADS / 64; ++i) r += sm64[i];
    __syncthreads();
    return r;
}

// statistics fallback (block version of wave_row_stats): float64 exps against the true max
template <typename T>
__device__ RowStats block_row_stats(const StepParams& p, const char* rowc, double m, double* sm64) {
    double s1 = 0.0, st = 0.0, at = 0.0;
    for (int j = threadIdx.x; j < p.V; j += WIDE_THREADS) {
        if (is_banned(p, j)) continue;
        const double d = (double)(Elem<T>::load1(rowc, j) + 0.0f) - m;
        const double et = exp(d * p.inv_temp);
        s1 += exp(d);
        st += et;
        at += et * (d * p.inv_temp);
    }
    s1 = block_sum(s1, sm64);
    st = block_sum(st, sm64);
    at = block_sum(at, sm64);
    RowStats rs;
    rs.lse1 = log(s1);
    rs.lst = log(st);
    rs.a_over_s = at / st;
    return rs;
}

// the kept mass E of ranks [0, k) (exact limb sums: any split over threads gives the same value); every
// thread of the block gets it
template <int NT = WIDE_THREADS, typename EOf>
__device__ double block_mass(int k, EOf e_of, double* sm64) {
    Mass ms{0.0, 0.0, 0.0, 0.0};
    for (int i = (int)threadIdx.x; i < k; i += NT) mass_add(ms, e_of(i));
    mass_wave_sum(ms);
    const int lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE;
    __syncthreads();
    if (lane == 0) {
        sm64[4 * wv + 0] = ms.a;
        sm64[4 * wv + 1] = ms.b;
        sm64[4 * wv + 2] = ms.c;
        sm64[4 * wv + 3] = ms.d;
    }
    __syncthreads();
    Mass t{0.0, 0.0, 0.0, 0.0};
    for (int w = 0; w < NT / WAVE; ++w) {
        t.a += sm64[4 * w + 0];
        t.b += sm64[4 * w + 1];
        t.c += sm64[4 * w + 2];
        t.d += sm64[4 * w + 3];
    }
    __syncthreads();
    return mass_value(t);
}

// interval update, bit emit and state/statistics writes of one finished step (thread 0; both CDF kernels)
template <bool DECODE>
__device__ __forceinline__ void wide_finish(const StepParams& p, int b, const ns_stream_state& st, int k, int kp, int sel, bool exact,
                            double S_used, int64_t cum_m1, int64_t cum_sel, int64_t shift, uint64_t sel_key, double m,
                            const RowStats& rs, double kl, bool want_stats) {
    const int P = p.P;
    const uint64_t mask = (P >= 64) ? ~0ull : ((1ull << P) - 1ull);
    const uint64_t new_lo = sel > 0 ? (uint64_t)(cum_m1 + shift) : st.lo;
    const uint64_t new_hi = (uint64_t)(cum_sel + shift);
    const uint64_t top = new_hi - 1ull;
    const uint64_t diff = (new_lo ^ top) & mask;
    const int n = diff == 0ull ? P - 1 : P - (64 - __builtin_clzll(diff));
    const int32_t token = (int32_t)wkey_id(sel_key);
    ns_stream_state ns = st;
    if (DECODE) {
        const bool last = p.is_last[b] != 0;
        const int cntb = last ? P : n;
        const uint64_t src = last ? new_lo : top;
        uint8_t* ob = p.out_bits + (int64_t)b * p.out_stride;
        for (int t = 0; t < cntb; ++t) {
            const int64_t bp = st.bit_pos + t;
            const uint8_t bitv = (uint8_t)((src >> (P - 1 - t)) & 1u);
            const uint8_t bm = (uint8_t)(1u << (bp & 7));
            ob[bp >> 3] = bitv ? (uint8_t)(ob[bp >> 3] | bm) : (uint8_t)(ob[bp >> 3] & ~bm);
        }
        ns.bit_pos = st.bit_pos + cntb;
    } else {
        ns.bit_pos = st.bit_pos + n;
    }
    ns.lo = (new_lo << n) & mask;
    ns.hi = (((top << n) & mask) | ((1ull << n) - 1ull)) + 1ull;
    ns.ntokens = st.ntokens + 1;
    ns.flags = (st.flags & ~NS_ST_EXACT_SUM) | (exact ? NS_ST_EXACT_SUM : 0u);
    if (!DECODE && ns.bit_pos >= p.nbits[b] && !(p.flags & NS_STEP_FINISH_SENT)) ns.flags |= NS_ST_DONE;
    p.state[b] = ns;
    if (!DECODE) {
        p.out_token[b] = token;
        if (p.hist && st.ntokens < p.hist_stride) p.hist[(int64_t)b * p.hist_stride + st.ntokens] = token;
    }
    if (p.trace) {
        ns_step_trace tr = {k, kp, sel, n, token, exact ? 1 : 0, S_used};
        p.trace[b] = tr;
    }
    if (want_stats) {
        double* a = p.stats + 4 * (int64_t)b;
        a[0] += ((double)wkey_val(sel_key) - m) - rs.lse1;
        a[1] += kl / 0.69315;
        a[2] += (rs.lst - rs.a_over_s) / 0.69315;
        a[3] += 1.0;
    }
    if (p.counters && exact) atomicAdd(&p.counters[4 * (b & (NS_COUNTER_SHARDS - 1))], 1ull);
}

// the canonical tail of one stream (keys_sorted: its collected keys in rank order); every thread of the block
template <typename T, bool DECODE>
__device__ __forceinline__ void wide_cdf_stream(const StepParams& p, const WideStat* ws, const uint64_t* keys_sorted,
                                                const unsigned int* count, int cap, const int b) {
    __shared__ double ebuf[WIDE_ROUND];
    __shared__ double sm64[64];
    __shared__ int smi[16];
    __shared__ int64_t sml[16];
    __shared__ int64_t cum_at[4];  // [0] cum(kp-1), [1] cum(sel-1), [2] cum(sel)
    __shared__ uint64_t sel_key;
    const WideStat w = ws[b];
    if (!w.active) return;
    const int tid = threadIdx.x;
    const ns_stream_state st = p.state[b];
    const uint64_t* sk = keys_sorted + (int64_t)b * cap;
    const int nC = (int)count[b];
    if (nC < 2) {  // every row has >= 2 valid ids and the collection keeps the top two: only NaN logits (never
        // collected) get here -- no CDF exists, report a range error instead of reading stale keys
        if (tid == 0) p.state[b].flags = st.flags | NS_ST_ERR_RANGE | NS_ST_DONE;
        return;
    }
    const int Kc = min(nC, p.K);
    const char* rowc = (const char*)p.logits + (int64_t)b * p.ld * (int64_t)sizeof(T);
    const double m = (double)wkey_val(sk[0]);
    const uint64_t R = st.hi - st.lo;
    const double Rd = (double)R;
    const double thr = 1.0 / Rd;
    auto e_of = [&](int i) -> double { return exp_canon(((double)wkey_val(sk[i]) - m) * p.inv_temp); };
    RowStats rs{0.0, 0.0, 0.0};
    const bool want_stats = !DECODE && p.stats != nullptr;
    if (want_stats && !row_stats_from_stream(w.S_r, w.B_r, w.U_r, w.r, m, p.inv_temp, rs))
        rs = block_row_stats<T>(p, rowc, m, sm64);

    if (!DECODE && p.sample) {  // sampler (oracle steps S2-S5): support, canonical E, 2^48 CDF, one draw
        int fl = Kc;
        for (int i = tid; i < Kc; i += WIDE_THREADS)
            if (e_of(i) < SAMPLE_SUPPORT && i < fl) fl = i;
        const int ks = block_min_int(fl, smi);
        double acc = 0.0;
        for (int base = 0; base < ks; base += WIDE_ROUND) {
            for (int i = tid; i < WIDE_ROUND; i += WIDE_THREADS) ebuf[i] = (base + i < ks) ? e_of(base + i) : 0.0;
            __syncthreads();
            if (tid < 64)
                for (int i = tid; i < WIDE_ROUND && base + i < ks; i += 64) acc += ebuf[i];
            __syncthreads();
        }
        if (tid < 64) sm64[tid] = acc;
        __syncthreads();
        const double E = block_canonical_butterfly(sm64);
        const int cs = (ks + WIDE_THREADS - 1) / WIDE_THREADS;
        const int i0 = min(ks, tid * cs), i1 = min(ks, i0 + cs);
        auto q_of = [&](int i) -> int64_t { return (int64_t)__builtin_rint((e_of(i) / E) * SAMPLE_SCALE); };
        int64_t local = 0;
        for (int i = i0; i < i1; ++i) local += q_of(i);
        int64_t total;
        const int64_t pre = block_excl_scan(local, sml, total);
        const uint64_t u = rand64(p.seed, p.stream_offset + b, st.ntokens);
        const uint64_t idx = __umul64hi(u, (uint64_t)total);
        int sel_l = 0x7FFFFFFF;
        {
            int64_t c = pre;
            for (int i = i0; i < i1; ++i) {
                c += q_of(i);
                if ((uint64_t)c > idx) {
                    sel_l = i;
                    break;
                }
            }
        }
        const int sel = block_min_int(sel_l, smi);
        double kl = 0.0, h = 0.0;
        if (want_stats) {
            const double logE = log(E);
            for (int i = i0; i < i1; ++i) {
                const double xi = (double)wkey_val(sk[i]) - m;
                const double lq = xi * p.inv_temp - logE;
                const double q = e_of(i) / E;
                kl += q * (lq - (xi - rs.lse1));
                h += q * lq;
            }
            kl = block_sum(kl, sm64);
            h = block_sum(h, sm64);
        }
        if (tid != 0) return;
        const int32_t token = (int32_t)wkey_id(sk[sel]);
        ns_stream_state ns = st;
        ns.ntokens = st.ntokens + 1;
        p.state[b] = ns;
        p.out_token[b] = token;
        if (p.hist && st.ntokens < p.hist_stride) p.hist[(int64_t)b * p.hist_stride + st.ntokens] = token;
        if (p.trace) {
            ns_step_trace tr = {Kc, ks, sel, 0, token, 0, E};
            p.trace[b] = tr;
        }
        if (want_stats) {
            double* a = p.stats + 4 * (int64_t)b;
            a[0] += ((double)wkey_val(sk[sel]) - m) - rs.lse1;
            a[1] += kl / 0.69315;
            a[2] += -h / 0.69315;
            a[3] += 1.0;
        }
        return;
    }

    // ---- 1. cutoff k0 = first rank with e_i/S < thr (ranks >= Kc are below for certain)
    bool exact = w.exact != 0;
    int k0 = Kc;
    double S_used = w.S_fast;
    if (!exact) {
        const double inv_lo = 1.0 / (w.S_lo * (1.0 - 1.0e-15));
        const double inv_hi = 1.0 / (w.S_hi * (1.0 + 1.0e-15));
        int fb = Kc, fa = Kc;
        for (int i = tid; i < Kc; i += WIDE_THREADS) {
            const double e = e_of(i);
            const bool below = e * inv_lo < thr;
            const bool above = e * inv_hi >= thr;
            if (below && i < fb) fb = i;
            if (!below && !above && i < fa) fa = i;
        }
        fb = block_min_int(fb, smi);
        fa = block_min_int(fa, smi);
        if (fa < fb)
            exact = true;
        else
            k0 = fb;
    }
    if (exact) {
        const double S = block_exact_row_sum<T>(p, rowc, m, ebuf, sm64);
        S_used = S;
        int fb = Kc;
        for (int i = tid; i < Kc; i += WIDE_THREADS)
            if (e_of(i) / S < thr && i < fb) fb = i;
        k0 = block_min_int(fb, smi);
    }
    int k = k0 < 2 ? 2 : k0;
    if (k > p.topk) k = p.topk;

    // ---- 2. E = sum_{i<k} e_i, order-free (exact limb sums, canonical step 6)
    const double E = block_mass(k, e_of, sm64);

    // ---- 3. q_i = rint(e_i/E*R), inclusive prefix over contiguous rank chunks, overfill trim
    const int cs = (k + WIDE_THREADS - 1) / WIDE_THREADS;
    const int i0 = min(k, tid * cs), i1 = min(k, i0 + cs);
    auto q_of = [&](int i) -> int64_t { return (int64_t)__builtin_rint((e_of(i) / E) * Rd); };
    // q of this thread's chunk computed once into registers when the chunk fits (k <= CQ * 1024, the usual
    // case): the prefix, overfill, selection and cum passes below re-read them instead of re-evaluating
    // exp_canon and re-loading the sorted keys each time
    constexpr int CQ = 8;
    const bool cached = cs <= CQ;
    int64_t qc[CQ];
#pragma unroll
    for (int j = 0; j < CQ; ++j) qc[j] = (cached && i0 + j < i1) ? q_of(i0 + j) : 0;
    auto for_chunk = [&](int iend, auto&& f) {  // f(rank, q) in rank order over [i0, iend); true = stop
        if (cached) {
#pragma unroll
            for (int j = 0; j < CQ; ++j)
                if (i0 + j < iend && f(i0 + j, qc[j])) return;
        } else {
            for (int i = i0; i < iend; ++i)
                if (f(i, q_of(i))) return;
        }
    };
    int64_t local = 0;
    for_chunk(i1, [&](int, int64_t q) {
        local += q;
        return false;
    });
    int64_t total;
    const int64_t pre = block_excl_scan(local, sml, total);
    int kp_l = k;
    {
        int64_t c = pre;
        for_chunk(i1, [&](int i, int64_t q) {
            c += q;
            if (c > (int64_t)R) {
                kp_l = i;
                return true;
            }
            return false;
        });
    }
    const int kp = block_min_int(kp_l, smi);
    // cum at rank kp-1 (its chunk owner recomputes the running prefix)
    auto cum_upto = [&](int i) -> int64_t {  // valid only for the owner of rank i
        int64_t c = pre;
        for_chunk(i + 1, [&](int, int64_t q) {
            c += q;
            return false;
        });
        return c;
    };
    if (kp - 1 >= i0 && kp - 1 < i1) cum_at[0] = cum_upto(kp - 1);
    __syncthreads();
    const int64_t shift = (int64_t)R - cum_at[0] + (int64_t)st.lo;

    // ---- selection
    int sel_l = 0x7FFFFFFF;
    uint32_t err = 0;
    if (!DECODE) {
        const uint64_t idx = payload_window(p, b, st.bit_pos);
        int64_t c = pre;
        for_chunk(min(i1, kp), [&](int i, int64_t q) {
            c += q;
            if ((uint64_t)(c + shift) > idx) {
                sel_l = i;
                return true;
            }
            return false;
        });
    } else {
        const int32_t tok = p.in_token[b];
        if (tok >= 0 && tok < p.V && !is_banned(p, tok)) {
            const uint64_t kt = wkey(Elem<T>::load1(rowc, tok), (uint32_t)tok);
            for (int i = i0; i < min(i1, kp); ++i)
                if (sk[i] == kt) {
                    sel_l = i;
                    break;
                }
        }
    }
    const int sel = block_min_int(sel_l, smi);
    if (sel == 0x7FFFFFFF) err = DECODE ? NS_ST_ERR_DIVERGE : NS_ST_ERR_RANGE;
    if (!(E > 0.0 && E <= 1.7976931348623157e308)) err = NS_ST_ERR_RANGE;  // non-finite logits: no valid CDF
    if (DECODE && err && p.ranked) {  // ranked kept ids for the host's BPE repair (arithmetic.py:300-342)
        int32_t* rk_out = p.ranked + (int64_t)b * p.ranked_stride;
        for (int i = tid; i < kp && i < p.ranked_stride; i += WIDE_THREADS) rk_out[i] = (int32_t)wkey_id(sk[i]);
        if (tid == 0 && kp < p.ranked_stride) rk_out[kp] = -1;
    }
    // statistics of an encode step (arithmetic.py:193-199): KL(q || p) over the k' kept entries
    double kl = 0.0;
    if (want_stats && !err) {
        const int64_t deficit = (int64_t)R - cum_at[0];
        for_chunk(min(i1, kp), [&](int i, int64_t pf) {
            if (i == 0) pf += deficit;
            const double qd = (double)pf / Rd;
            if (qd > 0.0) kl += qd * (log(qd) - (((double)wkey_val(sk[i]) - m) - rs.lse1));
            return false;
        });
    }
    if (want_stats) kl = block_sum(kl, sm64);
    if (!err) {
        if (sel - 1 >= i0 && sel - 1 < i1) cum_at[1] = cum_upto(sel - 1);
        if (sel >= i0 && sel < i1) cum_at[2] = cum_upto(sel);
        if (tid == 0) sel_key = sk[sel];
    }
    __syncthreads();
    if (tid != 0) return;
    if (err) {
        p.state[b].flags = st.flags | err | NS_ST_DONE;
        if (p.trace) {
            ns_step_trace tr = {k, kp, -1, -1, -1, exact ? 1 : 0, S_used};
            p.trace[b] = tr;
        }
        return;
    }
    wide_finish<DECODE>(p, b, st, k, kp, sel, exact, S_used, cum_at[1], cum_at[2], shift, sel_key, m, rs, kl,
                        want_stats);
}

// the streams wide_fast_kernel listed (todo[1 .. todo[0]]: more keys than its LDS holds, or a step it hands on),
// a grid-stride loop over the list so that the launch does not depend on how many there are
template <typename T, bool DECODE>
__global__ __launch_bounds__(WIDE_THREADS) void wide_cdf_kernel(StepParams p, const WideStat* ws,
                                                                const uint64_t* keys_sorted,
                                                                const unsigned int* count, int cap,
                                                                const unsigned int* todo) {
    const unsigned int nt = todo[0];
    for (unsigned int i = blockIdx.x; i < nt; i += gridDim.x) {
        wide_cdf_stream<T, DECODE>(p, ws, keys_sorted, count, cap, (int)todo[1 + i]);
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------ passes 3+4 in LDS
// The usual stream keeps a few thousand ids (3·N(0,1) logits at precision 16: 2-5k), far fewer than the
// device-wide sort is sized for.  One 512-thread workgroup per such stream (count <= FAST_NL) sorts its keys in
// LDS -- a counting sort on FAST_NB key-range buckets, then each key's rank inside its bucket by counting the
// larger bucket-mates (a bitonic sort instead when a bucket holds more than FAST_OCC_MAX keys) -- and runs the
// canonical tail on the sorted keys: the same arithmetic, in the same order, as wide_cdf_kernel.  Streams that
// need the exact row sum, the row-statistics fallback, the sampler, or hit an error are handed to
// wide_cdf_kernel (listed in todo) with their sorted keys written to keys_out; streams with more keys were
// sorted by the device-wide sort and are listed too.  Round 3-4: 53,248 B of LDS and <= 80 VGPRs, three
// workgroups per CU (measured 0.53 vs 0.58 ms per step with 8,192 keys / 3,840 buckets at two per CU, an older
// kernel); round 5: two per CU without the spill frame (NSG_FAST_WAVES_PER_SIMD below).
#ifndef NSG_SCAN_DIAG
#define NSG_SCAN_DIAG 0
#endif
#ifndef NSG_SCAN_VEC_BYTES
#define NSG_SCAN_VEC_BYTES 64  // row bytes per thread per group in the two sweeps (two groups in flight)
#endif
#ifndef NSG_SCAN_P1_KEEP
#define NSG_SCAN_P1_KEEP 1  // pass 1 loads with the default policy (0: non-temporal, for A/B timing)
#endif
constexpr int FAST_THREADS = 512;
constexpr int FAST_WAVES = FAST_THREADS / WAVE;
#ifndef NSG_FAST_NL
#define NSG_FAST_NL 6144  // round 5 (two workgroups per CU leave the LDS for it): 5,632 before
#endif
#ifndef NSG_FAST_NB
#define NSG_FAST_NB 2048
#endif
#ifndef NSG_FAST_WAVES_PER_SIMD
// launch-bounds occupancy target.  Round 5: 4 = two 512-thread workgroups per CU, 127 VGPRs and 36 B of scratch per
// lane, against 6 = three per CU at 80 VGPRs, whose ~200-byte spill frame per lane was 410 MB of HBM writes per
// launch (PMC 1.85x the algorithmic bytes -> 1.08x) -- and 3.5-4 % faster (profiles/r05/wide_occupancy_ab/)
#define NSG_FAST_WAVES_PER_SIMD 4
#endif
constexpr int FAST_NL = NSG_FAST_NL;               // keys of a stream sorted in LDS
constexpr int FAST_R = FAST_NL / FAST_THREADS;     // ranks per thread: rank i = r * FAST_THREADS + tid
constexpr int FAST_NB = NSG_FAST_NB;               // counting-sort buckets over [kmin, kmax]
constexpr uint32_t FAST_OCC_MAX = 48;              // fuller bucket -> bitonic sort

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int off) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, off);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), off);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ int wave_min_int(int v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = min(v, __shfl_xor(v, off));
    return v;
}

// the LDS path for one stream whose n <= FAST_NL collected keys sit at `kin` (global or LDS, any order): sort,
// then the canonical tail; every thread of the 512-thread block calls it
// the keys a thread loads: slot r of thread tid -- any partition of the stream's n keys over the block's slots
// (the counting sort below does not care which thread holds which key)
struct KeysFlat {  // one array (global memory or LDS): slot r of thread tid = key r * FAST_THREADS + tid
    const uint64_t* k;
    int n;
    __device__ __forceinline__ bool operator()(int r, uint64_t& key) const {
        const int i = r * FAST_THREADS + (int)threadIdx.x;
        key = i < n ? k[i] : 0ull;
        return i < n;
    }
};
// INX: the exact row sum (forced, unusable bound, or an ambiguous cutoff) is computed here by the block,
// instead of handing the stream to the list kernel (the one-pass kernel: ~1 % of stream-steps)
template <typename T, bool DECODE, bool INX = false, typename KeyAt>
__device__ __forceinline__ void fast_tail(const StepParams& p, const WideStat& w, WideStat* wsb, const int b,
                                          const int n, const KeyAt kin, uint64_t* keys_out, const int cap,
                                          unsigned int* todo, uint64_t* s_keys, uint64_t* s_aux) {
    uint32_t* s_cnt = (uint32_t*)s_aux;
    const int tid = (int)threadIdx.x, lane = tid & (WAVE - 1), wv = tid / WAVE;
    // ---- load (unsorted, as collected) + key range; every key is in registers before the first LDS write
    uint64_t kr[FAST_R];
    uint32_t vm = 0u;  // bit r: slot r holds a key
    uint64_t kmax = 0ull, kmin = ~0ull;
#pragma unroll
    for (int r = 0; r < FAST_R; ++r) {
        if (kin(r, kr[r])) {
            vm |= 1u << r;
            kmax = kr[r] > kmax ? kr[r] : kmax;
            kmin = kr[r] < kmin ? kr[r] : kmin;
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const uint64_t a = shfl_xor_u64(kmax, off), c = shfl_xor_u64(kmin, off);
        kmax = a > kmax ? a : kmax;
        kmin = c < kmin ? c : kmin;
    }
    if (lane == 0) {
        s_aux[wv] = kmax;
        s_aux[FAST_WAVES + wv] = kmin;
    }
    __syncthreads();
    uint64_t hi = s_aux[0], lo = s_aux[FAST_WAVES];
#pragma unroll
    for (int i = 1; i < FAST_WAVES; ++i) {
        hi = s_aux[i] > hi ? s_aux[i] : hi;
        lo = s_aux[FAST_WAVES + i] < lo ? s_aux[FAST_WAVES + i] : lo;
    }
    __syncthreads();
    for (int i = tid; i < FAST_NB; i += FAST_THREADS) s_cnt[i] = 0u;
    __syncthreads();
    // ---- counting sort: bucket 0 = the largest keys (monotone: a larger key never gets a later bucket)
    const double bscale = (double)FAST_NB / ((double)(hi - lo) + 1.0);
    uint32_t bs[FAST_R];  // bucket << 16 | slot inside the bucket
#pragma unroll
    for (int r = 0; r < FAST_R; ++r) {
        bs[r] = 0u;
        if ((vm >> r) & 1u) {
            const uint32_t bk = min((uint32_t)((double)(hi - kr[r]) * bscale), (uint32_t)(FAST_NB - 1));
            bs[r] = (bk << 16) | atomicAdd(&s_cnt[bk], 1u);
        }
    }
    __syncthreads();
    uint32_t* scr = (uint32_t*)s_keys;  // wave totals (s_keys is free until the scatter)
    uint32_t occ = 0u;
    {
        constexpr int PER = (FAST_NB + FAST_THREADS - 1) / FAST_THREADS;  // 8 buckets per thread
        const int c0 = tid * PER;
        uint32_t loc[PER], sum = 0u, mx = 0u;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            loc[j] = c0 + j < FAST_NB ? s_cnt[c0 + j] : 0u;
            sum += loc[j];
            mx = max(mx, loc[j]);
        }
        const uint32_t inc = wave_incl_scan_u32(sum);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off));
        if (lane == WAVE - 1) scr[wv] = inc;
        if (lane == 0) scr[FAST_WAVES + wv] = mx;
        __syncthreads();
        uint32_t run = inc - sum;
#pragma unroll
        for (int i = 0; i < FAST_WAVES; ++i) {
            if (i < wv) run += scr[i];
            occ = max(occ, scr[FAST_WAVES + i]);
        }
#pragma unroll
        for (int j = 0; j < PER; ++j)
            if (c0 + j < FAST_NB) {
                s_cnt[c0 + j] = run;
                run += loc[j];
            }
    }
    __syncthreads();
    const bool bitonic = occ > FAST_OCC_MAX;
    if (bitonic && tid == 0 && p.counters) atomicAdd(&p.counters[4 * (b & (NS_COUNTER_SHARDS - 1)) + 3], 1ull);
    int P2 = 1;
    while (P2 < n) P2 <<= 1;
#pragma unroll
    for (int r = 0; r < FAST_R; ++r)
        if ((vm >> r) & 1u) s_keys[s_cnt[bs[r] >> 16] + (bs[r] & 0xFFFFu)] = kr[r];
    __syncthreads();
    if (!bitonic) {
        // rank = bucket start + larger keys in the bucket (keys are distinct: ids are)
#pragma unroll
        for (int r = 0; r < FAST_R; ++r) {
            if ((vm >> r) & 1u) {
                const uint32_t bk = bs[r] >> 16;
                const uint32_t s0 = s_cnt[bk], s1 = bk + 1 < (uint32_t)FAST_NB ? s_cnt[bk + 1] : (uint32_t)n;
                uint32_t c = s0;
                for (uint32_t j = s0; j < s1; ++j) c += s_keys[j] > kr[r] ? 1u : 0u;
                bs[r] = c;
            }
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < FAST_R; ++r)
            if ((vm >> r) & 1u) s_keys[bs[r]] = kr[r];
        __syncthreads();
    } else {
        // bitonic network in its one-direction form (every compare-exchange puts the larger key at the lower
        // index: a mirror stage, then half-cleaners), over P2 = next power of two >= n positions of which only
        // [0, n) exist: a pair whose upper index is >= n pairs a real key with a virtual minimum, already in
        // order, so it is skipped and nothing is stored beyond n (P2 may exceed the LDS array)
        for (int size = 2; size <= P2; size <<= 1) {
            const int half = size >> 1;
            for (int t = tid; t < P2 / 2; t += FAST_THREADS) {
                const int base = (t / half) * size, off = t % half;
                const int i = base + off, j = base + size - 1 - off;
                if (j < n) {
                    const uint64_t a = s_keys[i], c = s_keys[j];
                    if (a < c) {
                        s_keys[i] = c;
                        s_keys[j] = a;
                    }
                }
            }
            __syncthreads();
            for (int stride = half >> 1; stride > 0; stride >>= 1) {
                for (int t = tid; t < P2 / 2; t += FAST_THREADS) {
                    const int i = 2 * t - (t & (stride - 1)), j = i + stride;
                    if (j < n) {
                        const uint64_t a = s_keys[i], c = s_keys[j];
                        if (a < c) {
                            s_keys[i] = c;
                            s_keys[j] = a;
                        }
                    }
                }
                __syncthreads();
            }
        }
    }
    // ---- sorted keys of this thread's ranks into registers; s_keys becomes the e_i array
    NSG_STAMP(p, b, tid, 5);
    uint64_t ks[FAST_R];
#pragma unroll
    for (int r = 0; r < FAST_R; ++r) {
        const int i = r * FAST_THREADS + tid;
        ks[r] = i < n ? s_keys[i] : 0ull;
    }
    const uint64_t top = s_keys[0];
    __syncthreads();
#if NSG_SCAN_DIAG == 3  // passes 1 and 2 and the LDS sort only
    if (tid == 0) atomicExch((unsigned int*)&keys_out[(int64_t)b * cap], (unsigned int)ks[0]);  // keep ks live
    return;
#endif
    auto defer = [&]() __attribute__((always_inline)) {  // hand the stream to wide_cdf_kernel with its keys in rank order
        uint64_t* ko = keys_out + (int64_t)b * cap;
#pragma unroll
        for (int r = 0; r < FAST_R; ++r) {
            const int i = r * FAST_THREADS + tid;
            if (i < n) ko[i] = ks[r];
        }
        if (tid == 0) todo[1 + atomicAdd(&todo[0], 1u)] = (unsigned int)b;
    };
    const ns_stream_state st = p.state[b];
    const double m = (double)wkey_val(top);
    const bool want_stats = !DECODE && p.stats != nullptr;
    RowStats rs{0.0, 0.0, 0.0};
    if ((!DECODE && p.sample) || (w.exact && !INX) ||
        (want_stats && !row_stats_from_stream(w.S_r, w.B_r, w.U_r, w.r, m, p.inv_temp, rs))) {
        defer();
        return;
    }
    const int Kc = min(n, p.K);
    const uint64_t R = st.hi - st.lo;
    const double Rd = (double)R;
    const double thr = 1.0 / Rd;
    double* s_e = (double*)s_keys;
    bool exact = w.exact != 0;
    double S_used = w.S_fast;
    // ---- 1. cutoff k0 (the fast-sum interval decides it, or the stream needs the exact sum)
    int fb = Kc, fa = Kc;
    if (!exact) {
        const double inv_lo = 1.0 / (w.S_lo * (1.0 - 1.0e-15));
        const double inv_hi = 1.0 / (w.S_hi * (1.0 + 1.0e-15));
#pragma unroll
        for (int r = 0; r < FAST_R; ++r) {
            const int i = r * FAST_THREADS + tid;
            if (i < Kc) {
                const double e = exp_canon(((double)wkey_val(ks[r]) - m) * p.inv_temp);
                s_e[i] = e;
                const bool below = e * inv_lo < thr;
                const bool above = e * inv_hi >= thr;
                if (below) fb = min(fb, i);
                if (!below && !above) fa = min(fa, i);
            }
        }
    }
    int* s_i = (int*)(s_aux + 16);
    fb = wave_min_int(fb);
    fa = wave_min_int(fa);
    if (lane == 0) {
        s_i[wv] = fb;
        s_i[FAST_WAVES + wv] = fa;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < FAST_WAVES; ++i) {
        fb = min(fb, s_i[i]);
        fa = min(fa, s_i[FAST_WAVES + i]);
    }
    if (INX && (exact || fa < fb)) {
        // the canonical exact row sum by this block (s_keys is scratch: e_i are recomputed from the registers)
        __syncthreads();
        const char* rowc = (const char*)p.logits + (int64_t)b * p.ld * (int64_t)sizeof(T);
        const double S = block_exact_row_sum<T, FAST_THREADS, 4096>(p, rowc, m, (double*)s_keys, (double*)(s_aux + 512));
        exact = true;
        S_used = S;
        fb = Kc;
#pragma unroll
        for (int r = 0; r < FAST_R; ++r) {
            const int i = r * FAST_THREADS + tid;
            if (i < Kc) {
                const double e = exp_canon(((double)wkey_val(ks[r]) - m) * p.inv_temp);
                s_e[i] = e;
                if (e / S < thr) fb = min(fb, i);
            }
        }
        fb = wave_min_int(fb);
        if (lane == 0) s_i[wv] = fb;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < FAST_WAVES; ++i) fb = min(fb, s_i[i]);
        fa = Kc;
    }
    NSG_STAMP(p, b, tid, 6);
#if NSG_SCAN_DIAG == 4  // timing diagnostics: up to the cutoff
    if (tid == 0) atomicExch((unsigned int*)&keys_out[(int64_t)b * cap], (unsigned int)(fb + fa));
    return;
#endif
    int k = fb < 2 ? 2 : fb;
    if (k > p.topk) k = p.topk;
    // ambiguous cutoff (the exact row sum: measured cheaper in the list kernel than in this one, whose
    // workgroup slots are the row stream's) or a degenerate row: wide_cdf_kernel
    if (fa < fb || k > Kc) {
        // an ambiguous cutoff is marked exact, so wide_cdf_kernel goes straight to the exact row sum (it would
        // find the same ambiguity first)
        if (fa < fb && tid == 0) wsb->exact = 1u;
        defer();
        return;
    }
    // ---- 2. E = sum_{i<k} e_i, order-free (exact limb sums, canonical step 6)
    double* s_d = (double*)(s_aux + 32);
    const double E = block_mass<FAST_THREADS>(k, [&](int i) { return s_e[i]; }, s_d);
    // ---- 3. q_i = rint(e_i/E*R); inclusive prefix in rank order (wave scans + per-round wave totals)
    const int nr = (k + FAST_THREADS - 1) / FAST_THREADS;
    int64_t* s_tot = (int64_t*)(s_aux + 64);  // [FAST_R][FAST_WAVES]
    int64_t cum[FAST_R];
#pragma unroll
    for (int r = 0; r < FAST_R; ++r) {
        cum[r] = 0;
        if (r < nr) {
            const int i = r * FAST_THREADS + tid;
            const int64_t q = i < k ? (int64_t)__builtin_rint((s_e[i] / E) * Rd) : 0;
            cum[r] = wave_incl_scan(q, lane);
            if (lane == WAVE - 1) s_tot[r * FAST_WAVES + wv] = cum[r];
        }
    }
    __syncthreads();
    {
        int64_t carry = 0;
#pragma unroll
        for (int r = 0; r < FAST_R; ++r)
            if (r < nr) {
                int64_t before = 0, all = 0;
#pragma unroll
                for (int j = 0; j < FAST_WAVES; ++j) {
                    const int64_t t = s_tot[r * FAST_WAVES + j];
                    if (j < wv) before += t;
                    all += t;
                }
                cum[r] += carry + before;
                carry += all;
            }
    }
    // overfill: kp = first rank whose cum exceeds R
    int kp = k;
#pragma unroll
    for (int r = 0; r < FAST_R; ++r) {
        const int i = r * FAST_THREADS + tid;
        if (r < nr && i < k && cum[r] > (int64_t)R) kp = min(kp, i);
    }
    int* s_j = (int*)(s_aux + 256);
    kp = wave_min_int(kp);
    if (lane == 0) s_j[wv] = kp;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < FAST_WAVES; ++i) kp = min(kp, s_j[i]);
    int64_t* s_c = (int64_t*)(s_aux + 272);  // [0] cum(kp-1), [1] cum(sel-1), [2] cum(sel), [3] key(sel)
    auto publish = [&](int rank, int slot, bool key) __attribute__((always_inline)) {  // owner of `rank` writes its cum (or key) to s_c[slot]
        if (rank >= 0 && rank % FAST_THREADS == tid) {
            // masked sum, not `if (r == rr)`: the compiler folds that into an indexed load, which puts the
            // register arrays in scratch memory
            const int rr = rank / FAST_THREADS;
            int64_t v = 0;
#pragma unroll
            for (int r = 0; r < FAST_R; ++r) v |= (key ? (int64_t)ks[r] : cum[r]) & -(int64_t)(r == rr);
            s_c[slot] = v;
        }
    };
    publish(kp - 1, 0, false);
    __syncthreads();
    const int64_t cum_kp = s_c[0];
    NSG_STAMP(p, b, tid, 7);
    const int64_t shift = (int64_t)R - cum_kp + (int64_t)st.lo;
    // ---- selection
    int sel = 0x7FFFFFFF;
    if (!DECODE) {
        const uint64_t idx = payload_window(p, b, st.bit_pos);
#pragma unroll
        for (int r = 0; r < FAST_R; ++r) {
            const int i = r * FAST_THREADS + tid;
            if (r < nr && i < kp && (uint64_t)(cum[r] + shift) > idx) sel = min(sel, i);
        }
    } else {
        const int32_t tok = p.in_token[b];
        if (tok >= 0 && tok < p.V && !is_banned(p, tok)) {
            const char* rowc = (const char*)p.logits + (int64_t)b * p.ld * (int64_t)sizeof(T);
            const uint64_t kt = wkey(Elem<T>::load1(rowc, tok), (uint32_t)tok);
#pragma unroll
            for (int r = 0; r < FAST_R; ++r) {
                const int i = r * FAST_THREADS + tid;
                if (i < kp && ks[r] == kt) sel = min(sel, i);
            }
        }
    }
    int* s_k = (int*)(s_aux + 288);
    sel = wave_min_int(sel);
    if (lane == 0) s_k[wv] = sel;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < FAST_WAVES; ++i) sel = min(sel, s_k[i]);
    if (sel == 0x7FFFFFFF || !(E > 0.0 && E <= 1.7976931348623157e308)) {  // range / divergence error or
        // non-finite logits: wide_cdf_kernel reports it (and the ranked export)
        defer();
        return;
    }
    publish(sel - 1, 1, false);
    publish(sel, 2, false);
    publish(sel, 3, true);
    // statistics of an encode step (arithmetic.py:193-199): KL(q || p) over the k' kept entries
    double kl = 0.0;
    if (want_stats) {
        const int64_t deficit = (int64_t)R - cum_kp;
#pragma unroll
        for (int r = 0; r < FAST_R; ++r) {
            const int i = r * FAST_THREADS + tid;
            if (r < nr && i < kp) {
                int64_t pf = (int64_t)__builtin_rint((s_e[i] / E) * Rd);
                if (i == 0) pf += deficit;
                const double qd = (double)pf / Rd;
                if (qd > 0.0) kl += qd * (log(qd) - (((double)wkey_val(ks[r]) - m) - rs.lse1));
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) kl += __shfl_xor(kl, off);
        if (lane == 0) s_d[8 + wv] = kl;
    }
    __syncthreads();
    if (tid != 0) return;
    if (want_stats) {
        kl = 0.0;
        for (int i = 0; i < FAST_WAVES; ++i) kl += s_d[8 + i];
    }
    wide_finish<DECODE>(p, b, st, k, kp, sel, exact, S_used, s_c[1], s_c[2], shift, (uint64_t)s_c[3], m, rs, kl,
                        want_stats);
    NSG_STAMP(p, b, tid, 8);
    NSG_STAMP_RT(p, b, tid, 10);
}


// ------------------------------------------------------------------------------------------ fused wide step
// One 512-thread workgroup per stream does passes 1 and 2 and, for the usual stream, the whole step:
//   pass 1: stream the row once (default cache policy) -> max, second max, the proven fast-sum interval
//           (fp32 groups of W terms, as wide_stats_kernel: the same bound)
//   pass 2: stream it again -- three workgroups per CU keep ~768 rows (~155 MB fp32) in flight, within the
//           256 MiB Infinity Cache, so the re-read can be served there (a non-temporal pass 1 measured 4 % slower
//           overall) -- collecting the ids that can clear the cutoff into LDS
//   then fast_tail (LDS sort + canonical tail).  More than FAST_NL keys: pass 3 writes them to keys_in for the
//   device-wide sort and the stream is listed for wide_cdf_kernel.
__device__ __forceinline__ float uni_f32(float v) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ __forceinline__ double uni_f64(double v) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(u >> 32));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

template <typename T, bool DECODE>
__global__ __launch_bounds__(FAST_THREADS, NSG_FAST_WAVES_PER_SIMD) void wide_scan_kernel(StepParams p, WideStat* ws, uint64_t* keys_in,
                                                                   uint64_t* keys_out, unsigned int* count, int cap,
                                                                   unsigned int* todo) {
    __shared__ uint64_t s_keys[FAST_NL];
    __shared__ uint64_t s_aux[FAST_NB / 2];
    constexpr int W = Elem<T>::W;
    constexpr int G = NSG_SCAN_VEC_BYTES / (4 * W);  // 16-B vectors per thread per block row group
    constexpr int TS = FAST_THREADS * W;      // ids per block-wide vector row
    const int b = blockIdx.x, tid = (int)threadIdx.x, lane = tid & (WAVE - 1), wv = tid / WAVE;
    const ns_stream_state st = p.state[b];
    bool active = !(st.flags & NS_ST_DONE);
    if (!DECODE && !p.sample && active && st.bit_pos >= p.nbits[b]) {
        if (tid == 0 && !(p.flags & NS_STEP_FINISH_SENT)) p.state[b].flags = st.flags | NS_ST_DONE;
        active = false;
    }
    if (DECODE && p.active && !p.active[b]) active = false;
    if (!active) {
        if (tid == 0) {
            ws[b].active = 0;
            count[b] = 0;
        }
        return;
    }
    const int V = p.V;
    const char* rowc = (const char*)p.logits + (int64_t)b * p.ld * (int64_t)sizeof(T);
    const RowReader rd(rowc, (uint32_t)(p.ld * (int64_t)sizeof(T)));
    const int nvec = (V + W - 1) / W;
    const int nsup = (nvec + G * FAST_THREADS - 1) / (G * FAST_THREADS);
    // x[g][.] = block-row (s*G + g) of this thread; ids >= V and banned ids -> `fill` (pass 1: -inf, which adds
    // nothing to the sums; pass 2: NaN, which no threshold collects -- a real -inf logit is a valid id and is
    // collected when the threshold is -inf, as in wide_collect_kernel)
    auto fetch = [&](int sI, uint4 (&raw)[G], bool keep) __attribute__((always_inline)) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int v = (sI * G + g) * FAST_THREADS + tid;
            raw[g] = keep ? rd.vec_keep(v) : rd.vec(v);
        }
    };
    auto prep = [&](int sI, const uint4 (&raw)[G], float (&x)[G][W], int& bi, int& next_ban,
                    float fill) __attribute__((always_inline)) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            Elem<T>::unpack(raw[g], x[g]);
            const int j0 = ((sI * G + g) * FAST_THREADS + tid) * W;
#pragma unroll
            for (int q = 0; q < W; ++q)
                if (j0 + q >= V) x[g][q] = fill;
            while (next_ban < (sI * G + g + 1) * TS) {
#pragma unroll
                for (int q = 0; q < W; ++q)
                    if (j0 + q == next_ban) x[g][q] = fill;
                ++bi;
                next_ban = bi < p.nbanned ? p.banned[bi] : 0x7FFFFFFF;
            }
        }
    };
    // one sweep over the row: consume(sI, x) for every block row in order, the loads of block row sI + 1 in
    // flight while block row sI is consumed (two register buffers, no copies between them)
    auto sweep = [&](bool keep, float fill, auto&& consume) __attribute__((always_inline)) {
        int bi = 0, next_ban = p.nbanned > 0 ? p.banned[0] : 0x7FFFFFFF;
        uint4 ra[G], rb[G];
        fetch(0, ra, keep);
        for (int sI = 0; sI < nsup; sI += 2) {
            if (sI + 1 < nsup) fetch(sI + 1, rb, keep);
            {
                float x[G][W];
                prep(sI, ra, x, bi, next_ban, fill);
                consume(sI, x);
            }
            if (sI + 1 < nsup) {
                if (sI + 2 < nsup) fetch(sI + 2, ra, keep);
                float x[G][W];
                prep(sI + 1, rb, x, bi, next_ban, fill);
                consume(sI + 1, x);
            }
        }
    };
    // ---- pass 1
    float r = 0.0f, m1 = -__builtin_inff(), m2 = -__builtin_inff();
    double acc64 = 0.0, b64 = 0.0, u64 = 0.0;
    const bool stats = p.stats != nullptr;
    sweep(NSG_SCAN_P1_KEEP != 0, -__builtin_inff(), [&](int sI, float (&x)[G][W]) __attribute__((always_inline)) {
        if (sI == 0) {  // reference r = max of the first block rows (any finite reference is valid)
            float mx = -__builtin_inff();
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int q = 0; q < W; ++q) mx = fmaxf(mx, x[g][q]);
            mx = wave_max(mx);
            float* s_f = (float*)(s_aux + 8);
            if (lane == 0) s_f[wv] = mx;
            __syncthreads();
            r = s_f[0];
#pragma unroll
            for (int i = 1; i < FAST_WAVES; ++i) r = fmaxf(r, s_f[i]);
            if (r == -__builtin_inff()) r = 0.0f;
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            float a = 0.0f, bb = 0.0f, uu = 0.0f;
#pragma unroll
            for (int q = 0; q < W; ++q) {
                const float dx = fmaxf(x[g][q] - r, -3.0e38f);
                const float e = __builtin_amdgcn_exp2f(dx * p.c32);
                a += e;
                if (stats) {
                    bb += e * dx;
                    uu += __builtin_amdgcn_exp2f(dx * L2E_F);
                }
                m2 = fmaxf(m2, fminf(m1, x[g][q]));
                m1 = fmaxf(m1, x[g][q]);
            }
            acc64 += (double)a;
            b64 += (double)bb;
            u64 += (double)uu;
        }
    });
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const float o1 = __shfl_xor(m1, off), o2 = __shfl_xor(m2, off);
        m2 = fmaxf(fminf(m1, o1), fmaxf(m2, o2));
        m1 = fmaxf(m1, o1);
    }
    acc64 = wave_sum_butterfly(acc64);
    b64 = wave_sum_butterfly(b64);
    u64 = wave_sum_butterfly(u64);
    {
        double* s_d = (double*)(s_aux + 16);  // [3][FAST_WAVES]
        float* s_f = (float*)(s_aux + 48);    // [2][FAST_WAVES]
        if (lane == 0) {
            s_d[wv] = acc64;
            s_d[FAST_WAVES + wv] = b64;
            s_d[2 * FAST_WAVES + wv] = u64;
            s_f[wv] = m1;
            s_f[FAST_WAVES + wv] = m2;
        }
        __syncthreads();
        acc64 = b64 = u64 = 0.0;
        m1 = m2 = -__builtin_inff();
#pragma unroll
        for (int i = 0; i < FAST_WAVES; ++i) {
            acc64 += s_d[i];
            b64 += s_d[FAST_WAVES + i];
            u64 += s_d[2 * FAST_WAVES + i];
            const float o1 = s_f[i], o2 = s_f[FAST_WAVES + i];
            m2 = fmaxf(fminf(m1, o1), fmaxf(m2, o2));
            m1 = fmaxf(m1, o1);
        }
    }
    // block-uniform from here on: into scalar registers (the LDS tail needs the vector registers)
    acc64 = uni_f64(acc64);
    b64 = uni_f64(b64);
    u64 = uni_f64(u64);
    m1 = uni_f32(m1);
    m2 = uni_f32(m2);
    WideStat w;
    {
        double Sf = 0.0, S_lo = 0.0, S_hi = 0.0;
        const bool ok = fast_sum_interval(acc64, r, (double)(m1 + 0.0f), p.c32, p.inv_temp, W, Sf, S_lo, S_hi);
        w.m = m1;
        w.m2 = m2;
        w.r = r;
        w.active = 1;
        w.S_lo = S_lo;
        w.S_hi = S_hi;
        w.S_fast = Sf;
        w.exact = (ok && !(p.flags & NS_STEP_FORCE_EXACT_SUM)) ? 0u : 1u;
        w.pad = 0;
        w.S_r = acc64;
        w.B_r = b64;
        w.U_r = u64;
        w.S_lo = uni_f64(w.S_lo);
        w.S_hi = uni_f64(w.S_hi);
        w.S_fast = uni_f64(w.S_fast);
        w.exact = (uint32_t)__builtin_amdgcn_readfirstlane((int)w.exact);
    }
    if (tid == 0) ws[b] = w;
#if NSG_SCAN_DIAG == 1  // timing diagnostics (tools/wide_timing.py on a tools/build_variant.sh build): pass 1 only
    if (tid == 0) count[b] = 0u;
    return;
#endif
    // ---- collection threshold (as wide_collect_kernel)
    float xt;
    {
        const double thr = 1.0 / (double)(st.hi - st.lo);
        const double temp = 1.0 / p.inv_temp;
        if (p.sample) {
            const double t = (double)w.m - temp * 41.58883083359672;
            xt = (float)(t - 1.0e-4 * (1.0 + fabs((double)w.m) + temp * 41.58883083359672));
        } else if (w.exact) {
            xt = -__builtin_inff();
        } else {
            const double L = log(w.S_lo * thr);
            const double t = (double)w.m + temp * L;
            xt = (float)(t - 1.0e-4 * (1.0 + fabs((double)w.m) + fabs(temp * L)));
        }
        xt = uni_f32(fminf(xt, w.m2));  // at least the top two ids (k >= 2)
    }
    // ---- pass 2 (and pass 3 into global memory when the keys overflow the LDS)
    uint32_t* s_ctr = (uint32_t*)(s_aux + FAST_NB / 2 - 1);
    if (tid == 0) s_ctr[0] = 0u;
    __syncthreads();
    auto collect = [&](bool to_global) __attribute__((always_inline)) {
        uint64_t* kout = keys_in + (int64_t)b * cap;
        sweep(false, __builtin_nanf(""), [&](int sI, float (&x)[G][W]) __attribute__((always_inline)) {
            uint32_t tot = 0;
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int q = 0; q < W; ++q) tot += (uint32_t)popc64(ballot(x[g][q] >= xt));
            if (tot == 0u) return;  // wave-uniform
            uint32_t base = 0u;
            if (lane == 0) base = atomicAdd(s_ctr, tot);
            base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
            uint32_t off = 0u;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const int j0 = ((sI * G + g) * FAST_THREADS + tid) * W;
#pragma unroll
                for (int q = 0; q < W; ++q) {
                    const uint64_t mk = ballot(x[g][q] >= xt);  // recomputed: cheaper than holding G*W masks
                    const uint32_t pos = base + off + (uint32_t)lanes_below(mk);
                    if ((mk >> lane) & 1ull) {
                        const uint64_t key = wkey(x[g][q], (uint32_t)(j0 + q));
                        if (to_global) {
                            if (pos < (uint32_t)cap) kout[pos] = key;  // n <= V - nbanned <= cap
                        } else if (pos < (uint32_t)FAST_NL) {
                            s_keys[pos] = key;
                        }
                    }
                    off += (uint32_t)popc64(mk);
                }
            }
        });
    };
    collect(false);
    __syncthreads();
    const int n = (int)s_ctr[0];
#if NSG_SCAN_DIAG == 2  // passes 1 and 2 only
    if (tid == 0) count[b] = 0u;
    return;
#endif
    if (n <= FAST_NL) {
        if (tid == 0) count[b] = (unsigned int)n;
        fast_tail<T, DECODE>(p, w, &ws[b], b, n, KeysFlat{s_keys, n}, keys_out, cap, todo, s_keys, s_aux);
        return;
    }
    __syncthreads();
    if (tid == 0) s_ctr[0] = 0u;
    __syncthreads();
    collect(true);
    if (tid == 0) {
        count[b] = (unsigned int)n;
        todo[1 + atomicAdd(&todo[0], 1u)] = (unsigned int)b;
    }
}

// ------------------------------------------------------------------------------------------ one-pass wide step
// (round 3) The row is streamed ONCE.  wide_scan_kernel needed two sweeps because the collection threshold
// x_t = r + T ln(S_r / R) (an id below it has e_i < S/R: below the cutoff for certain) depends on the row sum S,
// known only after the first sweep.  But any partial sum is a lower bound of S, so a threshold computed from the
// ids seen so far is a valid (lower, i.e. collect-more) threshold, and it only rises as the sweep goes on:
//   * each of the 8 waves takes a contiguous slice of the row; its last NSW tiles (8 x NSW x 1 KiB = 4,096 ids,
//     a stratified sample) are read first; their max is the reference r and their sum the first threshold;
//   * the wave streams the rest of its slice (non-temporal 16-B loads, a ring of NR tiles refilled in place),
//     accumulating the fast sum (fp32 per tile, float64 across tiles), e * |arg| for the data-dependent bound,
//     the lane's top two values, and appending the ids at or above its threshold to its own LDS buffer
//     (704 keys; when full, compacted to the current threshold -- ids below it are below the final one too);
//   * after every ring group the wave publishes its partial sum and re-reads the others' (plain LDS words:
//     each is a partial sum, so whatever subset is read is a lower bound), and raises its threshold;
//   * ids that can be among the top two are kept too (k >= 2): a wave's threshold is min(x_t, its running
//     second max), which never exceeds the row's second max when that id arrives.
// At the end the buffers are filtered to x >= min(x_t(final interval), m2) -- exactly a prefix of the ranking --
// merged into one LDS array and handed to fast_tail.  A wave whose buffer overflows even after compaction makes
// the stream take the old path: one more block sweep collects into global memory (sorted in LDS by fast_tail
// when it fits, else by the device-wide sort and the list kernel).
#ifndef NSG_WIDE_ONEPASS
#define NSG_WIDE_ONEPASS 1
#endif
#ifndef NSG_WIDE_SPLIT
#define NSG_WIDE_SPLIT 0  // 1: row stream and tail in two kernels (wide_onepass_kernel + wide_tail_kernel)
#endif
#ifndef NSG_TAIL_PRIO
#define NSG_TAIL_PRIO 0  // s_setprio level of the one-pass kernel after its row stream (0: off)
#endif
#ifndef NSG_OP_RING
#define NSG_OP_RING 4
#endif
constexpr int OP_CAPW = FAST_NL / FAST_WAVES;  // keys per wave buffer

__device__ __forceinline__ float wave_sum_f32(float v) {
    v += __uint_as_float(xor_lane_u32<32>(__float_as_uint(v)));
    v += __uint_as_float(xor_lane_u32<16>(__float_as_uint(v)));
    v += __uint_as_float(xor_lane_u32<8>(__float_as_uint(v)));
    v += __uint_as_float(xor_lane_u32<4>(__float_as_uint(v)));
    v += __uint_as_float(xor_lane_u32<2>(__float_as_uint(v)));
    v += __uint_as_float(xor_lane_u32<1>(__float_as_uint(v)));
    return v;
}
// wave top two of the lanes' (m1, m2): every lane ends with the wave's (m1, m2)
__device__ __forceinline__ void wave_top2(float& m1, float& m2) {
    auto step = [&](float o1, float o2) __attribute__((always_inline)) {
        m2 = fmaxf(fminf(m1, o1), fmaxf(m2, o2));
        m1 = fmaxf(m1, o1);
    };
    step(__uint_as_float(xor_lane_u32<32>(__float_as_uint(m1))), __uint_as_float(xor_lane_u32<32>(__float_as_uint(m2))));
    step(__uint_as_float(xor_lane_u32<16>(__float_as_uint(m1))), __uint_as_float(xor_lane_u32<16>(__float_as_uint(m2))));
    step(__uint_as_float(xor_lane_u32<8>(__float_as_uint(m1))), __uint_as_float(xor_lane_u32<8>(__float_as_uint(m2))));
    step(__uint_as_float(xor_lane_u32<4>(__float_as_uint(m1))), __uint_as_float(xor_lane_u32<4>(__float_as_uint(m2))));
    step(__uint_as_float(xor_lane_u32<2>(__float_as_uint(m1))), __uint_as_float(xor_lane_u32<2>(__float_as_uint(m2))));
    step(__uint_as_float(xor_lane_u32<1>(__float_as_uint(m1))), __uint_as_float(xor_lane_u32<1>(__float_as_uint(m2))));
}

// raw buffer entries of the one-pass kernel: value bits << 32 | id (the order transform waits for the tail)
__device__ __forceinline__ uint64_t op_raw(float x, uint32_t j) { return ((uint64_t)__float_as_uint(x) << 32) | j; }
__device__ __forceinline__ float op_raw_val(uint64_t e) { return __uint_as_float((uint32_t)(e >> 32)); }
__device__ __forceinline__ uint64_t op_raw_key(uint64_t e) { return wkey(op_raw_val(e), (uint32_t)e); }
// keep the entries of a wave buffer whose value is >= t, in place and in order
__device__ __forceinline__ int wave_compact(uint64_t* wbuf, int cnt, float t) {
    const int lane = (int)(threadIdx.x & (WAVE - 1));
    int nc = 0;
    for (int base = 0; base < cnt; base += WAVE) {
        const int i = base + lane;
        const uint64_t k = i < cnt ? wbuf[i] : 0ull;
        const bool keep = i < cnt && op_raw_val(k) >= t;
        const uint64_t km = ballot(keep);
        if (keep) wbuf[nc + lanes_below(km)] = k;
        nc += popc64(km);
    }
    return __builtin_amdgcn_readfirstlane(nc);
}

// ---- sort-free tail (round 3) -------------------------------------------------------------------------------
// The CDF needs the kept keys' q_i in rank order only where a cumulative sum is SEARCHED (the overfill trim,
// the selection, the received token's interval), and E no longer needs any order (canonical step 6).  So the
// usual stream is finished without sorting its ~4,000 kept keys:
//   1. every thread: its keys' exps and kept flags (not provably below the cutoff); wave sums of the limb mass,
//      the kept count, the key range, an ambiguity flag -> one barrier -> E, k
//   2. q_i and a 512-bucket histogram (monotone in the key: bucket order = rank order) of counts and q sums
//      (LDS atomics) -> exclusive prefix per bucket (one bucket per thread, wave scans) -> the overfill bucket
//   3. the kept keys scattered in bucket order (unordered inside a bucket)
//   4. wave 0 ranks the few keys of the searched buckets among themselves (<= 64 each: lane-to-lane loop) and
//      finishes the step: overfill trim, selection (encode) or the received token's rank (decode)
// Anything else -- an ambiguous cutoff, k outside [2, topk], a bucket with more than 64 keys, a decode token that is
// not kept or sits in the overfill bucket, statistics, the sampler -- returns false BEFORE s_keys is touched, and
// the stream takes fast_tail (sort) as before.  Same integers: the kept set, E and every q_i are the canonical
// step's; the searches give the first rank whose cumulative sum crosses the target, as the rank-order scans do.
#ifndef NSG_NOSORT
#define NSG_NOSORT 0  // sort-free tail (measured slower, A/B: DESIGN.md)
#endif
constexpr int NS_NB = FAST_THREADS;  // buckets (one per thread in the scan)

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const uint64_t o = shfl_xor_u64(v, off);
        v = o < v ? o : v;
    }
    return v;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const uint64_t o = shfl_xor_u64(v, off);
        v = o > v ? o : v;
    }
    return v;
}
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

struct KeysWave {  // slot r of a thread: entry r * 64 + lane of its wave's raw LDS buffer
    const uint64_t* wbuf;
    int mine;
    __device__ __forceinline__ bool operator()(int r, uint64_t& key) const {
        const int j = r * WAVE + (int)(threadIdx.x & (WAVE - 1));
        key = j < mine ? op_raw_key(wbuf[j]) : 0ull;
        return j < mine;
    }
};

// own function (not inlined): its register demand stays out of the row-stream loop's allocation
template <typename T, bool DECODE, typename KeyAt>
__device__ __noinline__ bool nosort_tail(const StepParams& p, const WideStat* wsb, const int b, const KeyAt kin,
                                         uint64_t* s_keys, uint64_t* s_aux) {
    const WideStat w = *wsb;
    const int tid = (int)threadIdx.x, lane = tid & (WAVE - 1), wv = tid / WAVE;
    uint64_t* qb = s_aux;                       // [NS_NB] bucket q sums, then their exclusive prefix
    uint32_t* cb = (uint32_t*)(s_aux + NS_NB);  // [NS_NB] bucket counts, then their exclusive prefix
    uint64_t* pw = s_aux + NS_NB + NS_NB / 2;   // 256 words of per-wave partials
    const ns_stream_state st = p.state[b];
    const uint64_t R = st.hi - st.lo;
    const double Rd = (double)R, thr = 1.0 / Rd;
    const double inv_lo = 1.0 / (w.S_lo * (1.0 - 1.0e-15)), inv_hi = 1.0 / (w.S_hi * (1.0 + 1.0e-15));
    const double m = (double)w.m;  // the row max = the largest collected key's value
    // ---- 1. exps, kept flags, limb mass, key range (keys re-read from LDS in every phase and exps recomputed
    // in step 2: register arrays of all slots would spill at the 80-VGPR occupancy budget)
    auto e_of = [&](uint64_t k) __attribute__((always_inline)) -> double {
        return exp_canon(((double)wkey_val(k) - m) * p.inv_temp);
    };
    uint32_t km = 0u;
    Mass ms{0.0, 0.0, 0.0, 0.0};
    uint64_t kmin = ~0ull, kmax = 0ull;
    uint32_t nk = 0u;
    bool amb = false;
#pragma unroll
    for (int r = 0; r < FAST_R; ++r) {
        uint64_t k;
        if (!kin(r, k)) continue;
        kmax = k > kmax ? k : kmax;
        const double e = e_of(k);
        if (e * inv_lo < thr) continue;  // provably below the cutoff
        amb |= !(e * inv_hi >= thr);     // neither provably below nor above: the exact sum decides
        km |= 1u << r;
        ++nk;
        kmin = k < kmin ? k : kmin;
        mass_add(ms, e);
    }
    mass_wave_sum(ms);
    kmin = wave_min_u64(kmin);
    kmax = wave_max_u64(kmax);
    nk = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan_u32(nk), WAVE - 1);
    const bool wamb = ballot(amb) != 0ull;
    if (lane == 0) {
        pw[8 * wv + 0] = __builtin_bit_cast(uint64_t, ms.a);
        pw[8 * wv + 1] = __builtin_bit_cast(uint64_t, ms.b);
        pw[8 * wv + 2] = __builtin_bit_cast(uint64_t, ms.c);
        pw[8 * wv + 3] = __builtin_bit_cast(uint64_t, ms.d);
        pw[8 * wv + 4] = kmin;
        pw[8 * wv + 5] = kmax;
        pw[8 * wv + 6] = (uint64_t)nk | ((uint64_t)(wamb ? 1u : 0u) << 32);
    }
    __syncthreads();
    Mass tot{0.0, 0.0, 0.0, 0.0};
    uint64_t kmin_a = ~0ull, kmax_a = 0ull;
    int k0 = 0;
    bool amb_a = false;
#pragma unroll
    for (int i = 0; i < FAST_WAVES; ++i) {
        tot.a += __builtin_bit_cast(double, pw[8 * i + 0]);
        tot.b += __builtin_bit_cast(double, pw[8 * i + 1]);
        tot.c += __builtin_bit_cast(double, pw[8 * i + 2]);
        tot.d += __builtin_bit_cast(double, pw[8 * i + 3]);
        kmin_a = pw[8 * i + 4] < kmin_a ? pw[8 * i + 4] : kmin_a;
        kmax_a = pw[8 * i + 5] > kmax_a ? pw[8 * i + 5] : kmax_a;
        k0 += (int)(uint32_t)pw[8 * i + 6];
        amb_a |= (pw[8 * i + 6] >> 32) != 0ull;
    }
    // decode: the received token must be a kept key (else fast_tail reports the divergence + ranked export)
    uint64_t kt = 0ull;
    if (DECODE) {
        const int32_t tok = p.in_token[b];
        if (tok >= 0 && tok < p.V && !is_banned(p, tok)) {
            const char* rowc = (const char*)p.logits + (int64_t)b * p.ld * (int64_t)sizeof(T);
            kt = wkey(Elem<T>::load1(rowc, tok), (uint32_t)tok);
        }
    }
    if (amb_a || k0 < 2 || k0 > p.topk || (DECODE && !(kt >= kmin_a && kt <= kmax_a))) return false;
    const double E = mass_value(tot);
    NSG_STAMP(p, b, tid, 5);
    // ---- 2. q and the bucket histogram (bucket 0 = the largest keys; monotone, so bucket order = rank order)
    qb[tid] = 0ull;
    cb[tid] = 0u;
    __syncthreads();
    const double bscale = (double)NS_NB / ((double)(kmax_a - kmin_a) + 1.0);
    auto bucket_of = [&](uint64_t k) __attribute__((always_inline)) -> uint32_t {
        return min((uint32_t)((double)(kmax_a - k) * bscale), (uint32_t)(NS_NB - 1));
    };
    uint32_t bs[FAST_R];
#pragma unroll
    for (int r = 0; r < FAST_R; ++r) {
        bs[r] = 0u;
        if ((km >> r) & 1u) {
            uint64_t k;
            kin(r, k);
            const int64_t q = (int64_t)__builtin_rint((e_of(k) / E) * Rd);
            const uint32_t bk = bucket_of(k);
            bs[r] = (bk << 16) | atomicAdd(&cb[bk], 1u);
            atomicAdd((unsigned long long*)&qb[bk], (unsigned long long)q);
        }
    }
    __syncthreads();
    // ---- 3. exclusive prefixes (thread t owns bucket t), the largest bucket, the overfill bucket
    const uint32_t c = cb[tid];
    const int64_t qv = (int64_t)qb[tid];
    const uint32_t ci = wave_incl_scan_u32(c);
    const int64_t qi = wave_incl_scan(qv, lane);
    uint32_t occ = c;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) occ = max(occ, (uint32_t)__shfl_xor((int)occ, off));
    if (lane == WAVE - 1) {
        pw[64 + wv] = (uint64_t)qi;
        pw[72 + wv] = (uint64_t)ci | ((uint64_t)occ << 32);
    }
    __syncthreads();
    int64_t qbefore = 0, Q = 0;
    uint32_t cbefore = 0u, maxocc = 0u;
#pragma unroll
    for (int i = 0; i < FAST_WAVES; ++i) {
        const int64_t tq = (int64_t)pw[64 + i];
        const uint32_t tc = (uint32_t)pw[72 + i];
        if (i < wv) {
            qbefore += tq;
            cbefore += tc;
        }
        Q += tq;
        maxocc = max(maxocc, (uint32_t)(pw[72 + i] >> 32));
    }
    if (maxocc > (uint32_t)WAVE) return false;  // a crowded bucket (skewed row): the sort path
    NSG_STAMP(p, b, tid, 6);
    const int64_t QP = qbefore + qi - qv;        // exclusive prefix of bucket tid
    const uint32_t CP = cbefore + ci - c;
    // overfill bucket: the first whose inclusive prefix exceeds R (NS_NB: none)
    int ovf = (Q > (int64_t)R && QP + qv > (int64_t)R) ? tid : NS_NB;
    ovf = wave_min_int(ovf);
    // the decode token's bucket must lie before the overfill bucket (else the sort path checks it)
    const int bt = DECODE ? (int)bucket_of(kt) : 0;
    __syncthreads();  // every thread has read its bucket's count and sum
    qb[tid] = (uint64_t)QP;
    cb[tid] = CP;
    if (lane == 0) pw[80 + wv] = (uint64_t)(uint32_t)ovf;
    __syncthreads();
    int b_ov = NS_NB;
#pragma unroll
    for (int i = 0; i < FAST_WAVES; ++i) b_ov = min(b_ov, (int)(uint32_t)pw[80 + i]);
    if (DECODE && bt >= b_ov) return false;
    // ---- 4. kept keys in bucket order: every thread holds its keys in registers before the first write
    uint64_t kr[FAST_R];
#pragma unroll
    for (int r = 0; r < FAST_R; ++r) {
        kr[r] = 0ull;
        if ((km >> r) & 1u) kin(r, kr[r]);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < FAST_R; ++r)
        if ((km >> r) & 1u) s_keys[cb[bs[r] >> 16] + (bs[r] & 0xFFFFu)] = kr[r];
    __syncthreads();
    if (wv != 0) return true;
    NSG_STAMP(p, b, tid, 7);
    // ---- 5. wave 0: resolve the searched buckets and finish the step
    // member `lane` of bucket bk: its key, q, rank among the members, and cum = inclusive prefix at its rank
    auto resolve = [&](int bk, uint64_t& key, int64_t& q, int& rank, int64_t& cum, int& occ_b)
                       __attribute__((always_inline)) {
        const int c0 = (int)cb[bk], c1 = bk + 1 < NS_NB ? (int)cb[bk + 1] : k0;
        occ_b = c1 - c0;
        const bool valid = lane < occ_b;
        key = valid ? s_keys[c0 + lane] : 0ull;
        q = valid ? (int64_t)__builtin_rint((e_of(key) / E) * Rd) : 0;
        rank = 0;
        int64_t ge = 0;
        for (int o = 0; o < occ_b; ++o) {
            const uint64_t ko = readlane_u64(key, o);
            const int64_t qo = (int64_t)readlane_u64((uint64_t)q, o);
            rank += ko > key ? 1 : 0;
            ge += ko >= key ? qo : 0;
        }
        cum = (int64_t)qb[bk] + ge;
    };
    int kp = k0;
    int64_t cumkp = Q;  // cum(kp - 1)
    int kp_local = WAVE;
    if (b_ov < NS_NB) {
        uint64_t key;
        int64_t q, cum;
        int rank, occ_b;
        resolve(b_ov, key, q, rank, cum, occ_b);
        const bool over = lane < occ_b && cum > (int64_t)R;
        kp_local = wave_min_int(over ? rank : WAVE);
        kp = (int)cb[b_ov] + kp_local;
        // cum(kp - 1): the member ranked kp_local - 1, or the prefix before the bucket
        const bool prev = lane < occ_b && rank == kp_local - 1;
        const uint64_t mp = ballot(prev);
        cumkp = mp ? (int64_t)readlane_u64((uint64_t)cum, __builtin_ctzll(mp)) : (int64_t)qb[b_ov];
    }
    const int64_t shift = (int64_t)R - cumkp + (int64_t)st.lo;
    int sel = -1;
    int64_t cum_m1 = 0, cum_sel = 0;
    uint64_t sel_key = 0ull;
    if (!DECODE) {
        const uint64_t idx = payload_window(p, b, st.bit_pos);
        // first bucket (<= b_ov) whose inclusive cum + shift exceeds idx; 8 buckets per lane
        int bs_l = NS_NB;
#pragma unroll
        for (int j = 0; j < NS_NB / WAVE; ++j) {
            const int bk = lane * (NS_NB / WAVE) + j;
            if (bk > b_ov) break;
            const int64_t incl = bk == b_ov ? cumkp : (bk + 1 < NS_NB ? (int64_t)qb[bk + 1] : Q);
            if ((uint64_t)(incl + shift) > idx) {
                bs_l = bk;
                break;
            }
        }
        const int bsel = wave_min_int(bs_l);
        if (bsel < NS_NB) {
            uint64_t key;
            int64_t q, cum;
            int rank, occ_b;
            resolve(bsel, key, q, rank, cum, occ_b);
            const bool hit = lane < occ_b && (bsel != b_ov || rank < kp_local) && (uint64_t)(cum + shift) > idx;
            const int rl = wave_min_int(hit ? rank : WAVE);
            const uint64_t mh = ballot(hit && rank == rl);
            if (mh) {
                const int src = __builtin_ctzll(mh);
                sel = (int)cb[bsel] + rl;
                cum_sel = (int64_t)readlane_u64((uint64_t)cum, src);
                cum_m1 = cum_sel - (int64_t)readlane_u64((uint64_t)q, src);
                sel_key = readlane_u64(key, src);
            }
        }
    } else {
        uint64_t key;
        int64_t q, cum;
        int rank, occ_b;
        resolve(bt, key, q, rank, cum, occ_b);
        const uint64_t mh = ballot(lane < occ_b && key == kt);
        if (mh) {
            const int src = __builtin_ctzll(mh);
            sel = (int)cb[bt] + __builtin_amdgcn_readlane(rank, src);
            cum_sel = (int64_t)readlane_u64((uint64_t)cum, src);
            cum_m1 = cum_sel - (int64_t)readlane_u64((uint64_t)q, src);
            sel_key = kt;
        }
    }
    if (lane != 0) return true;
    if (sel < 0) {  // encode: no interval above the payload index (decode cannot get here: the token is kept)
        p.state[b].flags = st.flags | (DECODE ? NS_ST_ERR_DIVERGE : NS_ST_ERR_RANGE) | NS_ST_DONE;
        if (p.trace) {
            ns_step_trace tr = {k0, kp, -1, -1, -1, 0, w.S_fast};
            p.trace[b] = tr;
        }
        return true;
    }
    const RowStats rs{0.0, 0.0, 0.0};
    wide_finish<DECODE>(p, b, st, k0, kp, sel, false, w.S_fast, sel > 0 ? cum_m1 : 0, cum_sel, shift, sel_key, m, rs,
                        0.0, false);
    NSG_STAMP(p, b, tid, 8);
    NSG_STAMP_RT(p, b, tid, 10);
    return true;
}

template <typename T, bool DECODE>
__global__ __launch_bounds__(FAST_THREADS, NSG_FAST_WAVES_PER_SIMD) void wide_onepass_kernel(
    StepParams p, WideStat* ws, uint64_t* keys_in, uint64_t* keys_out, unsigned int* count, int cap,
    unsigned int* todo) {
    __shared__ uint64_t s_keys[FAST_NL];
    __shared__ uint64_t s_aux[FAST_NB / 2];
    constexpr int W = Elem<T>::W;
    constexpr int TS = WAVE * W;             // ids per wave tile (1 KiB)
    constexpr int NSW = (W == 4) ? 2 : 1;    // sample tiles per wave: 8 x NSW x TS = 4,096 ids
    constexpr int NR = NSG_OP_RING;
    const int b = blockIdx.x, tid = (int)threadIdx.x, lane = tid & (WAVE - 1);
    const int wv = __builtin_amdgcn_readfirstlane(tid / WAVE);
    const ns_stream_state st = p.state[b];
    bool active = !(st.flags & NS_ST_DONE);
    if (!DECODE && !p.sample && active && st.bit_pos >= p.nbits[b]) {
        if (tid == 0 && !(p.flags & NS_STEP_FINISH_SENT)) p.state[b].flags = st.flags | NS_ST_DONE;
        active = false;
    }
    if (DECODE && p.active && !p.active[b]) active = false;
    if (!active) {
        if (tid == 0) {
            ws[b].active = 0;
            count[b] = 0;
        }
        return;
    }
    const int V = p.V;
    const char* rowc = (const char*)p.logits + (int64_t)b * p.ld * (int64_t)sizeof(T);
    const RowReader rd(rowc, (uint32_t)(p.ld * (int64_t)sizeof(T)));
    const int ntiles = (V + TS - 1) / TS;
    const int per = (ntiles + FAST_WAVES - 1) / FAST_WAVES;
    NSG_STAMP_RT(p, b, tid, 9);
    NSG_STAMP(p, b, tid, 0);
    const int s0 = min(ntiles, wv * per), s1 = min(ntiles, s0 + per);
    const int ns = min(NSW, s1 - s0);  // sample tiles: the last ns tiles of the slice
    const int se = s1 - ns;            // streamed tiles [s0, se)
    uint64_t* wbuf = s_keys + wv * OP_CAPW;
    // LDS scratch (s_aux, 64-bit words): [0,4) published partial sums (f32), [8,12) wave maxima (f32),
    // [16,48) per-wave double sums, [48,52) counts, [52,56) running thresholds, [60] sweep counter
    volatile float* s_part = (volatile float*)(s_aux + 0);
    float* s_m1 = (float*)(s_aux + 8);
    double* s_d = (double*)(s_aux + 16);
    int* s_n = (int*)(s_aux + 48);
    float* s_xt = (float*)(s_aux + 52);
    const bool stats = p.stats != nullptr;
    const double temp = 1.0 / p.inv_temp;
    const float tempf = (float)temp;
    const double Rd = (double)(st.hi - st.lo);
    const float lnthr = (float)(-log(Rd));  // ln(1/R)

    // x of tile t: out-of-row and banned ids -> -1e30 (no sum, below every real max), and bit q of `mb` set (never
    // collected: a real -inf logit IS collected when the threshold is -inf).  Bans are walked with a per-wave pointer
    // (`bi`, `next_ban`: the first ban at or after the tiles still to come), so the per-tile test is one scalar
    // compare; tiles must be visited in increasing order between resets of the pointer.
    int bi = 0, next_ban = 0x7FFFFFFF;
    auto ban_reset = [&](int t) __attribute__((always_inline)) {
        bi = 0;
        while (bi < p.nbanned && p.banned[bi] < t * TS) ++bi;
        next_ban = bi < p.nbanned ? p.banned[bi] : 0x7FFFFFFF;
    };
    auto load_x = [&](int t, const uint4& raw, float (&x)[W], uint32_t& mb) __attribute__((always_inline)) {
        Elem<T>::unpack(raw, x);
        mb = 0u;
        const int j0 = t * TS + lane * W;
        if ((t + 1) * TS > V) {
#pragma unroll
            for (int q = 0; q < W; ++q)
                if (j0 + q >= V) {
                    x[q] = -1.0e30f;
                    mb |= 1u << q;
                }
        }
        while (next_ban < (t + 1) * TS) {  // wave-uniform, at most nbanned times per slice
            const int d = next_ban - j0;
            if (d >= 0 && d < W) {
#pragma unroll
                for (int q = 0; q < W; ++q)
                    if (q == d) {
                        x[q] = -1.0e30f;
                        mb |= 1u << q;
                    }
            }
            ++bi;
            next_ban = bi < p.nbanned ? p.banned[bi] : 0x7FFFFFFF;
        }
    };
    float r = 0.0f, nrc = 0.0f;  // reference and -fl(r * c32)
    float m1 = -__builtin_inff();
    double accS = 0.0, accT = 0.0, accB = 0.0, accU = 0.0;
    float accSf = 0.0f;
    // one tile's fast-sum terms: e = 2^fma(x, c32, -r c32) in packed pairs, sum e and sum e*t (the bound's B_t),
    // flushed into float64 per tile (W terms per fp32 partial); the lane max with v_max3.  Masked ids are -1e30
    // (t finite, e = 0, e*t = 0); a real -inf logit makes B_t NaN, i.e. the bound unusable (exact row sum).
    auto sum_tile = [&](const float (&x)[W]) __attribute__((always_inline)) {
        typedef float f2 __attribute__((ext_vector_type(2)));
        const f2 c2 = {p.c32, p.c32}, n2 = {nrc, nrc};
        f2 a2 = {0.0f, 0.0f}, b2 = {0.0f, 0.0f};
#pragma unroll
        for (int q = 0; q < W; q += 2) {
            const f2 x2 = {x[q], x[q + 1]};
            const f2 t = __builtin_elementwise_fma(x2, c2, n2);
            const f2 e2 = {__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
            a2 += e2;
            b2 = __builtin_elementwise_fma(e2, t, b2);
            m1 = __builtin_fmaxf(__builtin_fmaxf(m1, x[q]), x[q + 1]);  // v_max3_f32
        }
        const float a = a2.x + a2.y;
        accS += (double)a;
        accT += (double)(b2.x + b2.y);
        accSf += a;
        if (stats) {  // sum e*(x-r) and the untempered sum: the statistics, not the bound
            float bb = 0.0f, uu = 0.0f;
#pragma unroll
            for (int q = 0; q < W; ++q) {
                const float dx = fmaxf(x[q] - r, -3.0e38f);
                const float e = __builtin_amdgcn_exp2f(dx * p.c32);
                bb += e * dx;
                uu += __builtin_amdgcn_exp2f(dx * L2E_F);
            }
            accB += (double)bb;
            accU += (double)uu;
        }
    };
    int cnt = 0;          // keys in this wave's buffer (wave-uniform)
    bool ovf = false;     // the buffer overflowed even after compaction (wave-uniform)
    float t_wave = -__builtin_inff();  // candidate threshold (wave-uniform)
    auto compact = [&]() __attribute__((always_inline)) { cnt = wave_compact(wbuf, cnt, t_wave); };
    // appends: each lane's passing values go to consecutive slots (lane order, then value order inside the
    // lane): a per-lane count, one wave scan (DPP), predicated raw writes -- no per-value ballot/mbcnt
    auto append_tile = [&](int t, const float (&x)[W], uint32_t mb) __attribute__((always_inline)) {
#if defined(NSG_OP_NOAPPEND)  // timing diagnostics: streaming and sums only
        return;
#endif
        uint32_t c = 0u;
#pragma unroll
        for (int q = 0; q < W; ++q) c += (x[q] >= t_wave) ? 1u : 0u;
        if (mb) {  // masked values (tail tile / banned ids) never pass: recount without them (rare)
            c = 0u;
#pragma unroll
            for (int q = 0; q < W; ++q) c += (x[q] >= t_wave && !((mb >> q) & 1u)) ? 1u : 0u;
        }
        const uint32_t incl = wave_incl_scan_u32(c);
        const int tot = __builtin_amdgcn_readlane((int)incl, WAVE - 1);
        if (tot == 0 || ovf) return;
        if (cnt + tot > OP_CAPW) {
            compact();
            if (cnt + tot > OP_CAPW) {
                ovf = true;
                return;
            }
        }
        uint32_t pos = (uint32_t)cnt + incl - c;
        const uint32_t j0 = (uint32_t)(t * TS + lane * W);
#pragma unroll
        for (int q = 0; q < W; ++q)
            if (x[q] >= t_wave && !((mb >> q) & 1u)) wbuf[pos++] = op_raw(x[q], j0 + q);
        cnt += tot;
    };
    // threshold from a lower bound S_part of the row sum against r (fp32; 2^-10 of slack covers every rounding
    // of the partial sum by orders of magnitude, and the widening every rounding of the threshold)
    auto threshold = [&](float s_part, float mx) __attribute__((always_inline)) -> float {
        if (p.sample) {  // sampler support e_i >= 2^-60 of the max: any running max is a lower bound of m
            const float t = mx - tempf * 41.58883083359672f;
            return t - 1.0e-4f * (1.0f + fabsf(mx) + tempf * 41.58883083359672f);
        }
        if (!(s_part > 0.0f && s_part < 3.0e38f)) return -__builtin_inff();
        const float L = __builtin_amdgcn_logf(s_part * 0.9990234375f) * 0.6931471805599453f + lnthr;
        const float t = r + tempf * L;
        return t - 1.0e-4f * (1.0f + fabsf(r) + fabsf(tempf * L));
    };
    float xt_run = -__builtin_inff();

    // ---- sample tiles first (and the first ring tiles in flight behind them)
    uint4 smp[NSW];
#pragma unroll
    for (int i = 0; i < NSW; ++i)
        if (i < ns) smp[i] = rd.vec((se + i) * WAVE + lane);
    uint4 ring[NR];
#pragma unroll
    for (int j = 0; j < NR; ++j)
        if (s0 + j < se) ring[j] = rd.vec((s0 + j) * WAVE + lane);
    float xs[NSW][W];
    uint32_t mbs[NSW];
    float smax = -__builtin_inff();
    ban_reset(se);
#pragma unroll
    for (int i = 0; i < NSW; ++i) {
        mbs[i] = ~0u;
#pragma unroll
        for (int q = 0; q < W; ++q) xs[i][q] = -1.0e30f;
        if (i < ns) {
            load_x(se + i, smp[i], xs[i], mbs[i]);
#pragma unroll
            for (int q = 0; q < W; ++q) smax = fmaxf(smax, xs[i][q]);
        }
    }
    smax = wave_max(smax);
    if (lane == 0) s_m1[wv] = smax;
    __syncthreads();
    r = s_m1[0];
#pragma unroll
    for (int i = 1; i < FAST_WAVES; ++i) r = fmaxf(r, s_m1[i]);
    if (!(r > -1.0e29f)) r = 0.0f;  // no valid id in the sample
    r = uni_f32(r);
    nrc = uni_f32(-(r * p.c32));
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NSW; ++i)
        if (i < ns) sum_tile(xs[i]);
    {
        const float ws0 = wave_sum_f32(accSf);
        if (lane == 0) s_part[wv] = ws0;
        __syncthreads();
        float tot = 0.0f;
#pragma unroll
        for (int i = 0; i < FAST_WAVES; ++i) tot += s_part[i];
        xt_run = uni_f32(threshold(tot, r));
        t_wave = xt_run;
    }
#pragma unroll
    for (int i = 0; i < NSW; ++i)
        if (i < ns) append_tile(se + i, xs[i], mbs[i]);
    NSG_STAMP(p, b, tid, 1);

    // ---- stream the rest of the slice; the threshold rises every UPD tiles (16 values per lane)
    constexpr int UPD = 16 / W;
    static_assert(NR % UPD == 0, "ring a multiple of the update interval");
    ban_reset(s0);
    for (int base = s0; base < se; base += NR) {
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            const int t = base + j;
            if (t < se) {
                const uint4 v = ring[j];
                if (t + NR < se) ring[j] = rd.vec((t + NR) * WAVE + lane);
                float x[W];
                uint32_t mb;
                load_x(t, v, x, mb);
                sum_tile(x);
                append_tile(t, x, mb);
            }
#if !defined(NSG_OP_NOUPDATE)
            if ((j + 1) % UPD == 0 && t < se) {
                // publish this wave's partial sum, read the others' (each a partial sum: whatever is read is a
                // lower bound of the row sum), raise the threshold
                const float wsum = wave_sum_f32(accSf);
                if (lane == 0) s_part[wv] = wsum;
                float tot = 0.0f;
#pragma unroll
                for (int i = 0; i < FAST_WAVES; ++i) tot += s_part[i];
                xt_run = uni_f32(fmaxf(xt_run, threshold(tot, p.sample ? wave_max(m1) : r)));
                t_wave = xt_run;
            }
#endif
        }
    }
#if defined(NSG_OP_DIAG) && NSG_OP_DIAG == 1  // register-pressure / timing diagnostics: streaming only
    if (lane == 0) s_part[wv] = (float)accS + accSf + (float)accT + m1 + (float)cnt;
    if (tid == 0) count[b] = 0u;
    return;
#endif
    NSG_STAMP(p, b, tid, 2);
#if NSG_TAIL_PRIO
    // the rest of the step is a latency-bound chain of block reductions, barriers and fp64 work, sharing its SIMDs
    // with the row streams of the other resident workgroups: give it issue priority
    __builtin_amdgcn_s_setprio(NSG_TAIL_PRIO);
#endif

    // ---- the row's statistics
    accS = wave_sum_butterfly(accS);
    accT = wave_sum_butterfly(accT);
    if (stats) {
        accB = wave_sum_butterfly(accB);
        accU = wave_sum_butterfly(accU);
    }
    m1 = wave_max(m1);
    __syncthreads();  // every wave is past its last read of s_part
    if (lane == 0) {
        s_d[wv] = accS;
        s_d[FAST_WAVES + wv] = accT;
        s_d[2 * FAST_WAVES + wv] = accB;
        s_d[3 * FAST_WAVES + wv] = accU;
        s_m1[wv] = m1;
        s_n[wv] = ovf ? -1 : cnt;
        s_xt[wv] = xt_run;
    }
    __syncthreads();
    double S_r = 0.0, T_r = 0.0, B_r = 0.0, U_r = 0.0;
    float bm1 = -__builtin_inff(), xt_all = -__builtin_inff();
    bool any_ovf = false;
#pragma unroll
    for (int i = 0; i < FAST_WAVES; ++i) {
        S_r += s_d[i];
        T_r += s_d[FAST_WAVES + i];
        B_r += s_d[2 * FAST_WAVES + i];
        U_r += s_d[3 * FAST_WAVES + i];
        bm1 = fmaxf(bm1, s_m1[i]);
        xt_all = fmaxf(xt_all, s_xt[i]);  // every wave collected all ids >= its own final threshold
        any_ovf |= s_n[i] < 0;
    }
    if (!(bm1 > -1.0e29f)) bm1 = -__builtin_inff();
    WideStat w;
    {
        double Sf = 0.0, S_lo = 0.0, S_hi = 0.0;
        const bool ok = fast_sum_interval_dd(uni_f64(S_r), uni_f64(T_r), r, (double)(bm1 + 0.0f), p.c32, p.inv_temp,
                                             W, Sf, S_lo, S_hi);
        w.m = uni_f32(bm1);
        w.m2 = -__builtin_inff();  // not tracked (k >= 2 is checked below)
        w.r = r;
        w.active = 1;
        w.S_lo = uni_f64(S_lo);
        w.S_hi = uni_f64(S_hi);
        w.S_fast = uni_f64(Sf);
        w.exact = (uint32_t)__builtin_amdgcn_readfirstlane((ok && !(p.flags & NS_STEP_FORCE_EXACT_SUM)) ? 0 : 1);
        w.pad = 0;
        w.S_r = uni_f64(S_r);
        w.B_r = uni_f64(B_r);
        w.U_r = uni_f64(U_r);
        // the final collection threshold (as wide_collect_kernel), never below what every wave collected
        float xt = -__builtin_inff();
        const double thr = 1.0 / Rd;
        if (p.sample) {
            const double t = (double)w.m - temp * 41.58883083359672;
            xt = (float)(t - 1.0e-4 * (1.0 + fabs((double)w.m) + temp * 41.58883083359672));
        } else if (ok) {
            const double L = log(S_lo * thr);
            const double t = (double)w.m + temp * L;
            xt = (float)(t - 1.0e-4 * (1.0 + fabs((double)w.m) + fabs(temp * L)));
        }
        xt_all = uni_f32(fmaxf(xt, xt_all));  // ids >= it: a prefix of the ranking, all collected
    }
    if (tid == 0) ws[b] = w;
    __syncthreads();
    NSG_STAMP(p, b, tid, 3);
    // the row's second largest valid value (a block rescan of the row; block-uniform result)
    auto top2_second = [&]() __attribute__((always_inline)) -> float {
        float l1 = -__builtin_inff(), l2 = -__builtin_inff();
        ban_reset(wv);
        for (int t0 = 0; t0 < ntiles; t0 += FAST_WAVES) {
            const int t = t0 + wv;
            if (t < ntiles) {
                float x[W];
                uint32_t mb;
                load_x(t, rd.vec(t * WAVE + lane), x, mb);
#pragma unroll
                for (int q = 0; q < W; ++q) {
                    const float v = ((mb >> q) & 1u) ? -__builtin_inff() : x[q];
                    l2 = fmaxf(l2, fminf(l1, v));
                    l1 = fmaxf(l1, v);
                }
            }
        }
        wave_top2(l1, l2);
        __syncthreads();
        if (lane == 0) {
            s_m1[wv] = l1;
            s_xt[wv] = l2;
        }
        __syncthreads();
        float b1 = -__builtin_inff(), b2 = -__builtin_inff();
#pragma unroll
        for (int i = 0; i < FAST_WAVES; ++i) {
            b2 = fmaxf(fminf(b1, s_m1[i]), fmaxf(b2, s_xt[i]));
            b1 = fmaxf(b1, s_m1[i]);
        }
        __syncthreads();
        return uni_f32(b2);
    };
    // one block sweep collecting the valid ids with x >= thr into this stream's global key segment; the count
    uint32_t* s_ctr = (uint32_t*)(s_aux + 60);
    uint64_t* kout = keys_in + (int64_t)b * cap;
    auto sweep_global = [&](float thr) __attribute__((always_inline)) -> uint32_t {
        __syncthreads();
        if (tid == 0) s_ctr[0] = 0u;
        __syncthreads();
        ban_reset(wv);
        for (int t0 = 0; t0 < ntiles; t0 += FAST_WAVES) {
            const int t = t0 + wv;
            if (t < ntiles) {
                float x[W];
                uint32_t mb;
                load_x(t, rd.vec(t * WAVE + lane), x, mb);
                uint32_t tot = 0;
#pragma unroll
                for (int q = 0; q < W; ++q) tot += (uint32_t)popc64(ballot(x[q] >= thr && !((mb >> q) & 1u)));
                if (tot) {
                    uint32_t bs = 0u;
                    if (lane == 0) bs = atomicAdd(s_ctr, tot);
                    bs = (uint32_t)__builtin_amdgcn_readfirstlane((int)bs);
                    const int j0 = t * TS + lane * W;
#pragma unroll
                    for (int q = 0; q < W; ++q) {
                        const bool take = x[q] >= thr && !((mb >> q) & 1u);
                        const uint64_t mk = ballot(take);
                        const uint32_t pos = bs + (uint32_t)lanes_below(mk);
                        if (take && pos < (uint32_t)cap) kout[pos] = wkey(x[q], (uint32_t)(j0 + q));
                        bs += (uint32_t)popc64(mk);
                    }
                }
            }
        }
        __syncthreads();
        const uint32_t got = min(s_ctr[0], (uint32_t)cap);
        __syncthreads();
        return (uint32_t)__builtin_amdgcn_readfirstlane((int)got);
    };

    int n = 0;
    [[maybe_unused]] int n_before = 0;  // wave w's offset in the segment (split form only)
    bool from_lds = false;
    if (!any_ovf) {
        // ---- each wave filters its buffer to x >= xt_all in place; fast_tail reads the kept keys of its own
        // wave's buffer (slot r of a thread = entry r * 64 + lane; every key in registers before it writes LDS)
        t_wave = xt_all;
        compact();
        if (lane == 0) s_n[wv] = cnt;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < FAST_WAVES; ++i) {
            if (i < wv) n_before += s_n[i];
            n += s_n[i];
        }
        __syncthreads();
        from_lds = n >= 2 || n >= V - p.nbanned;
        // fewer than two ids clear the threshold (a peaked row: k >= 2 needs the second largest, which the
        // running threshold may have skipped): collect down to it with a sweep (rare)
        if (!from_lds) xt_all = uni_f32(fminf(xt_all, top2_second()));
    }
    if (!from_lds) {
        // ---- a buffer overflowed (or the top two are needed): one block sweep collects x >= xt_all into the
        // stream's global key segment; the LDS sort takes it from there when it fits, else the device-wide sort
        // (ws.pad marks it for wide_offsets_kernel) and the list kernel
        uint32_t got = sweep_global(xt_all);
        if (got < 2u && (int)got < V - p.nbanned) {  // overflowed AND peaked: the top two are below the threshold
            xt_all = uni_f32(fminf(xt_all, top2_second()));
            got = sweep_global(xt_all);
        }
        if (tid == 0 && p.counters) atomicAdd(&p.counters[4 * (b & (NS_COUNTER_SHARDS - 1)) + 1], 1ull);
        if (got > (uint32_t)FAST_NL) {
            if (tid == 0) {
                count[b] = got;
                ws[b].pad = 1u;
                todo[1 + atomicAdd(&todo[0], 1u)] = (unsigned int)b;
            }
            return;
        }
        n = (int)got;
    }
    if (tid == 0) count[b] = (unsigned int)n;
    static_assert(FAST_R * WAVE == OP_CAPW, "one slot per buffer entry");
    NSG_STAMP(p, b, tid, 4);
#if NSG_WIDE_SPLIT
    // split form: the kept keys go to the stream's global segment (wave w's after those of waves < w) and
    // wide_tail_kernel finishes the step, so this kernel carries no tail code (registers: the row stream only)
    if (from_lds && n <= FAST_NL) {
        for (int i = lane; i < cnt; i += WAVE) kout[n_before + i] = op_raw_key(wbuf[i]);
    }
    return;
#endif
    const int mine = cnt;
    auto at = [&](int rr, uint64_t& key) __attribute__((always_inline)) -> bool {
        if (from_lds) {  // block-uniform
            const int j = rr * WAVE + lane;
            key = j < mine ? op_raw_key(wbuf[j]) : 0ull;
            return j < mine;
        }
        const int i = rr * FAST_THREADS + tid;
        key = i < n ? kout[i] : 0ull;
        return i < n;
    };
#if NSG_NOSORT
    if (from_lds && !(!DECODE && p.sample) && !w.exact && !(!DECODE && p.stats != nullptr)) {
        if (nosort_tail<T, DECODE>(p, &ws[b], b, KeysWave{wbuf, mine}, s_keys, s_aux)) return;
        __syncthreads();  // the partials area of s_aux is rewritten by fast_tail
    }
#endif
    fast_tail<T, DECODE, true>(p, w, &ws[b], b, n, at, keys_out, cap, todo, s_keys, s_aux);
}

// ------------------------------------------------------------------------------------------ split-form tail
// (round 3) The tail of the one-pass step as its own kernel: one 512-thread workgroup per stream reads the kept
// keys wide_onepass_kernel wrote to the stream's segment and runs the sort-free tail, or the LDS sort tail
// (fast_tail, exact row sum included) when the sort-free one does not apply.  Streams the one-pass kernel
// handed to the device-wide sort (ws.pad) and inactive streams are skipped.  Without the row stream in the
// same kernel the tail keeps its registers (no spills at the 80-VGPR budget of three workgroups per CU) and
// never holds a row-stream slot.
#ifndef NSG_TAIL_WAVES_PER_SIMD
#define NSG_TAIL_WAVES_PER_SIMD 4  // 128 VGPRs: the tail's per-slot register arrays fit without spilling
#endif
template <typename T, bool DECODE>
__global__ __launch_bounds__(FAST_THREADS, NSG_TAIL_WAVES_PER_SIMD) void wide_tail_kernel(
    StepParams p, WideStat* ws, const uint64_t* keys_in, uint64_t* keys_out, const unsigned int* count, int cap,
    unsigned int* todo) {
    __shared__ uint64_t s_keys[FAST_NL];
    __shared__ uint64_t s_aux[FAST_NB / 2];
    const int b = blockIdx.x;
    const WideStat w = ws[b];
    if (!w.active || w.pad) return;
    NSG_STAMP(p, b, (int)threadIdx.x, 11);
    const int n = (int)count[b];
    const KeysFlat kin{keys_in + (int64_t)b * cap, n};
#if NSG_NOSORT
    if (!(!DECODE && p.sample) && !w.exact && !(!DECODE && p.stats != nullptr)) {
        if (nosort_tail<T, DECODE>(p, &ws[b], b, kin, s_keys, s_aux)) return;
        __syncthreads();  // the partials area of s_aux is rewritten by fast_tail
    }
#endif
    fast_tail<T, DECODE, true>(p, w, &ws[b], b, n, kin, keys_out, cap, todo, s_keys, s_aux);
}

// ------------------------------------------------------------------------------------------ wide step, round 4
// The wide step as two kernels sized for occupancy rather than one workgroup per stream:
//   wide_stream_kernel  one WAVE per stream (four streams per 256-thread workgroup, like the single-pass coder):
//                       streams the row once with a 4-tile load ring, keeps the fast sum, the max and the
//                       running collection threshold x_t = r + T ln(S_part / R) (any partial sum is a lower bound
//                       of S, so x_t only rises), appends ids at or above it to an 8 KiB LDS buffer, compacts the
//                       buffer to the current threshold when full and flushes it to the stream's global segment
//                       (values and ids as two arrays) when it stays more than half full.  At the end: the proven
//                       fast-sum interval (WideStat) and the final threshold xt; segment entries below xt are stale.
//   wide_wtail_kernel   one 256-thread workgroup per stream, no key array: each pass streams the segment's values
//                       again (L2 / Infinity Cache); pass A: exps, the cutoff (the kept set is x >= vk), the
//                       order-free limb mass E; pass C: q_i and a 256-bucket histogram (bucket order = rank order)
//                       of counts and q sums; one prefix per bucket; the members of the searched buckets (overfill,
//                       selection, the decode token) gathered into LDS and ranked against each other.
// Anything else -- an ambiguous cutoff or unusable bound (exact sum), k outside [2, topk], a crowded bucket, a
// decode token that is not kept, an encode range error -- is handed, untouched, to the
// device sort + wide_cdf_kernel (the list path) with its collected keys.  Statistics and the sampler keep the
// one-pass kernel (host dispatch).
constexpr int WS_WAVES = 4;                    // streams per stream-kernel workgroup
constexpr int WS_CW = 1024;                    // LDS buffer entries per wave (8 KiB)
#ifndef NSG_WS_NK
#define NSG_WS_NK 4  // sample tiles (1,024 fp32 / 2,048 fp16 ids); 8 spill (the unpacked tiles stay live)
#endif
#ifndef NSG_WS_NR
#define NSG_WS_NR 4
#endif
constexpr int WV_CW = 4096;                    // wave-per-stream step: LDS buffer entries (32 KiB)
constexpr int WT_THREADS = 256;                // tail workgroup
constexpr int WT_WAVES = WT_THREADS / WAVE;
constexpr int WT_U = 4;                        // segment values in flight per tail thread
constexpr int WT_LV = 8192;                    // segment values staged in LDS (32 KiB)
constexpr int WT_NB = WT_THREADS;              // buckets (one per thread in the prefix)
constexpr int WT_GM = 256;                     // members of one gathered bucket

__device__ __forceinline__ float* seg_vals(uint64_t* keys, int b, int cap) { return (float*)(keys + (int64_t)b * cap); }
// the id of segment entry i: 16-bit words when the vocabulary fits (V <= 65,536), else 32-bit
__device__ __forceinline__ uint32_t seg_id(const uint32_t* gj, int i, bool id16) {
    return id16 ? (uint32_t)((const uint16_t*)gj)[i] : gj[i];
}
__device__ __forceinline__ uint32_t* seg_ids(uint64_t* keys, int b, int cap) {
    return (uint32_t*)(keys + (int64_t)b * cap) + cap;
}

// The sort-free tail of one stream by ONE wave, from the candidates in its LDS buffer (wbuf[0, n): raw entries,
// all at or above the final threshold xt): the arithmetic of wide_wtail_kernel with wave-level reductions.  The
// step is finished here (state, token / bits) and the stream marked inactive for the later kernels, or handed to
// the hand-off list (keys to keys_out, pad) for an ambiguous cutoff, k outside [2, topk], a crowded bucket, a decode
// token that is not kept, or an encode range error.
template <typename T, bool DECODE>
__device__ __forceinline__ void wave_tail(const StepParams& p, WideStat* wsb, WideStat w, int b,
                                          const ns_stream_state& st, const uint64_t* wbuf, int n, uint64_t* keys_out,
                                          unsigned int* count, int cap, unsigned int* todo) {
    __shared__ uint32_t t_cnt[WT_NB];  // bucket counts, then their exclusive prefix
    __shared__ uint64_t t_q[WT_NB];    // bucket q sums, then their exclusive prefix
    __shared__ uint64_t t_mem[WT_GM];  // gathered members: keys
    __shared__ int64_t t_memq[WT_GM];  //   and q
    __shared__ uint32_t t_ctr;
    const int lane = (int)(threadIdx.x & (WAVE - 1));
    auto defer = [&](bool exact) __attribute__((always_inline)) {
        uint64_t* ko = keys_out + (int64_t)b * cap;
        for (int i = lane; i < n; i += WAVE) ko[i] = op_raw_key(wbuf[i]);
        if (lane == 0) {
            w.pad = 1u;
            if (exact) w.exact = 1u;
            w.nraw = 0u;
            *wsb = w;
            count[b] = (unsigned int)n;
            todo[1 + atomicAdd(&todo[0], 1u)] = (unsigned int)b;
        }
    };
    const uint64_t R = st.hi - st.lo;
    const double Rd = (double)R, thr = 1.0 / Rd;
    const double inv_lo = 1.0 / (w.S_lo * (1.0 - 1.0e-15)), inv_hi = 1.0 / (w.S_hi * (1.0 + 1.0e-15));
    const double m = (double)w.m;
    // ---- A: exps, cutoff (kept <=> x >= vk), order-free limb mass
    Mass ms{0.0, 0.0, 0.0, 0.0};
    uint32_t nk = 0u;
    bool amb = false;
    float vk = __builtin_inff();
    for (int i = lane; i < n; i += WAVE) {
        const float xv = op_raw_val(wbuf[i]);
        const double e = exp_canon(((double)xv - m) * p.inv_temp);
        if (e * inv_lo < thr) continue;
        amb |= !(e * inv_hi >= thr);
        ++nk;
        vk = fminf(vk, xv);
        mass_add(ms, e);
    }
    mass_wave_sum(ms);
    const int k0 = __builtin_amdgcn_readlane((int)wave_incl_scan_u32(nk), WAVE - 1);
    const bool amb_a = ballot(amb) != 0ull;
    vk = -wave_max(-vk);
    const double E = mass_value(ms);
    float xtok = -__builtin_inff();
    uint64_t kt = 0ull;
    bool tok_ok = true;
    if (DECODE) {
        const int32_t tok = p.in_token[b];
        tok_ok = tok >= 0 && tok < p.V && !is_banned(p, tok);
        if (tok_ok) {
            const char* rowc = (const char*)p.logits + (int64_t)b * p.ld * (int64_t)sizeof(T);
            xtok = Elem<T>::load1(rowc, tok);
            kt = wkey(xtok, (uint32_t)tok);
            tok_ok = xtok >= vk;
        }
    }
    if (amb_a || k0 < 2 || k0 > p.topk || k0 > p.K || !tok_ok || !(E > 0.0 && E <= 1.7976931348623157e308)) {
        defer(amb_a);
        return;
    }
    // ---- C: q and the bucket histogram over [vk, m]
    const float fm = w.m;
    const float bscale = fm > vk ? (float)WT_NB / (fm - vk) : 0.0f;
    auto bucket_of = [&](float v) __attribute__((always_inline)) -> uint32_t {
        return min((uint32_t)((fm - v) * bscale), (uint32_t)(WT_NB - 1));
    };
    auto q_of = [&](float v) __attribute__((always_inline)) -> int64_t {
        return (int64_t)__builtin_rint((exp_canon(((double)v - m) * p.inv_temp) / E) * Rd);
    };
    for (int j = lane; j < WT_NB; j += WAVE) {
        t_cnt[j] = 0u;
        t_q[j] = 0ull;
    }
    lds_fence();
    for (int i = lane; i < n; i += WAVE) {
        const float xv = op_raw_val(wbuf[i]);
        if (!(xv >= vk)) continue;
        const uint32_t bk = bucket_of(xv);
        atomicAdd(&t_cnt[bk], 1u);
        atomicAdd((unsigned long long*)&t_q[bk], (unsigned long long)q_of(xv));
    }
    lds_fence();
    // ---- prefixes: lane owns buckets 4 lane .. 4 lane + 3; the overfill bucket
    constexpr int BPL = WT_NB / WAVE;
    uint32_t cb[BPL];
    int64_t qb[BPL];
    uint32_t csum = 0u;
    int64_t qsum = 0;
#pragma unroll
    for (int j = 0; j < BPL; ++j) {
        cb[j] = t_cnt[BPL * lane + j];
        qb[j] = (int64_t)t_q[BPL * lane + j];
        csum += cb[j];
        qsum += qb[j];
    }
    const uint32_t cincl = wave_incl_scan_u32(csum);
    const int64_t qincl = wave_incl_scan(qsum, lane);
    const int64_t Q = (int64_t)readlane_u64((uint64_t)qincl, WAVE - 1);
    uint32_t cp = cincl - csum;
    int64_t qp = qincl - qsum;
    int ovf = WT_NB;
#pragma unroll
    for (int j = 0; j < BPL; ++j) {
        t_cnt[BPL * lane + j] = cp;
        t_q[BPL * lane + j] = (uint64_t)qp;
        if (Q > (int64_t)R && qp + qb[j] > (int64_t)R && ovf == WT_NB) ovf = BPL * lane + j;
        cp += cb[j];
        qp += qb[j];
    }
    const int b_ov = wave_min_int(ovf);
    lds_fence();
    auto incl_of = [&](int bk) __attribute__((always_inline)) -> int64_t {
        return bk + 1 < WT_NB ? (int64_t)t_q[bk + 1] : Q;
    };
    auto gather = [&](int bk) __attribute__((always_inline)) -> int {
        if (lane == 0) t_ctr = 0u;
        lds_fence();
        for (int i = lane; i < n; i += WAVE) {
            const uint64_t e = wbuf[i];
            const float xv = op_raw_val(e);
            if (!(xv >= vk) || (int)bucket_of(xv) != bk) continue;
            const uint32_t at = atomicAdd(&t_ctr, 1u);
            if (at < (uint32_t)WT_GM) {
                t_mem[at] = op_raw_key(e);
                t_memq[at] = q_of(xv);
            }
        }
        lds_fence();
        return (int)__builtin_amdgcn_readfirstlane((int)t_ctr);
    };
    struct Mem {
        uint64_t key[WT_GM / WAVE];
        int64_t q[WT_GM / WAVE], cum[WT_GM / WAVE];
        int rank[WT_GM / WAVE];
    };
    auto resolve = [&](int bk, int nm, Mem& mm) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < WT_GM / WAVE; ++j) {
            const int i = lane + WAVE * j;
            mm.key[j] = i < nm ? t_mem[i] : 0ull;
            mm.q[j] = i < nm ? t_memq[i] : 0;
            mm.rank[j] = 0;
            mm.cum[j] = 0;
        }
        for (int o = 0; o < nm; ++o) {
            const uint64_t ko = t_mem[o];
            const int64_t qo = t_memq[o];
#pragma unroll
            for (int j = 0; j < WT_GM / WAVE; ++j) {
                mm.rank[j] += ko > mm.key[j] ? 1 : 0;
                mm.cum[j] += ko >= mm.key[j] ? qo : 0;
            }
        }
        const int64_t base = (int64_t)t_q[bk];
#pragma unroll
        for (int j = 0; j < WT_GM / WAVE; ++j) mm.cum[j] += base;
    };
    auto crowded = [&]() __attribute__((always_inline)) {
        if (lane == 0 && p.counters) atomicAdd(&p.counters[4 * (b & (NS_COUNTER_SHARDS - 1)) + 3], 1ull);
        defer(false);
    };
    // ---- overfill: kp = first rank whose cum exceeds R
    int kp = k0, kp_local = WT_GM + 1, nm_ov = -1;
    int64_t cumkp = Q;
    if (b_ov < WT_NB) {
        nm_ov = gather(b_ov);
        if (nm_ov > WT_GM) {
            crowded();
            return;
        }
        Mem mm;
        resolve(b_ov, nm_ov, mm);
        int kl = WT_GM + 1;
#pragma unroll
        for (int j = 0; j < WT_GM / WAVE; ++j)
            if (lane + WAVE * j < nm_ov && mm.cum[j] > (int64_t)R) kl = min(kl, mm.rank[j]);
        kl = wave_min_int(kl);
        int64_t cprev = (int64_t)t_q[b_ov];
#pragma unroll
        for (int j = 0; j < WT_GM / WAVE; ++j) {
            const uint64_t mp = ballot(lane + WAVE * j < nm_ov && mm.rank[j] == kl - 1);
            if (mp) cprev = (int64_t)readlane_u64((uint64_t)mm.cum[j], __builtin_ctzll(mp));
        }
        kp_local = kl;
        kp = (int)t_cnt[b_ov] + kl;
        cumkp = cprev;
    }
    const int64_t shift = (int64_t)R - cumkp + (int64_t)st.lo;
    // ---- the searched bucket
    uint64_t idx = 0ull;
    int bsel;
    if (!DECODE) {
        idx = payload_window(p, b, st.bit_pos);
        int bl = WT_NB;
#pragma unroll
        for (int j = 0; j < BPL; ++j) {
            const int bk = BPL * lane + j;
            if (bk <= b_ov && bl == WT_NB) {
                const int64_t inc = bk == b_ov ? cumkp : incl_of(bk);
                if ((uint64_t)(inc + shift) > idx) bl = bk;
            }
        }
        bsel = wave_min_int(bl);
    } else {
        bsel = (int)bucket_of(xtok);
    }
    if (bsel >= WT_NB || bsel > b_ov) {
        defer(false);
        return;
    }
    const int nm = bsel == b_ov ? nm_ov : gather(bsel);
    if (nm > WT_GM) {
        crowded();
        return;
    }
    Mem mm;
    resolve(bsel, nm, mm);
    int rl = WT_GM + 1;
#pragma unroll
    for (int j = 0; j < WT_GM / WAVE; ++j) {
        const bool valid = lane + WAVE * j < nm && (bsel != b_ov || mm.rank[j] < kp_local);
        const bool hit = DECODE ? (valid && mm.key[j] == kt) : (valid && (uint64_t)(mm.cum[j] + shift) > idx);
        if (hit) rl = min(rl, mm.rank[j]);
    }
    rl = wave_min_int(rl);
    if (rl > WT_GM) {
        defer(false);
        return;
    }
    int64_t cum_sel = 0, q_sel = 0;
    uint64_t key_sel = 0ull;
#pragma unroll
    for (int j = 0; j < WT_GM / WAVE; ++j) {
        const uint64_t mh = ballot(lane + WAVE * j < nm && mm.rank[j] == rl);
        if (mh) {
            const int src = __builtin_ctzll(mh);
            cum_sel = (int64_t)readlane_u64((uint64_t)mm.cum[j], src);
            q_sel = (int64_t)readlane_u64((uint64_t)mm.q[j], src);
            key_sel = readlane_u64(mm.key[j], src);
        }
    }
    if (lane == 0) {
        const int sel = (int)t_cnt[bsel] + rl;
        const RowStats rs{0.0, 0.0, 0.0};
        wide_finish<DECODE>(p, b, st, k0, kp, sel, false, w.S_fast, sel > 0 ? cum_sel - q_sel : 0, cum_sel, shift,
                            key_sel, m, rs, 0.0, false);
        w.active = 0u;  // finished: the tail kernel, the hand-off list and the device sort skip it
        w.nraw = 0u;
        *wsb = w;
        count[b] = 0u;
    }
    NSG_STAMP(p, b, lane, 8);
    NSG_STAMP_RT(p, b, lane, 10);
}

// NWV waves (streams) per workgroup, CW buffer entries per wave, NR tiles in flight per wave.  INTAIL (the
// wave-per-stream step, wide_wave_kernel below): a wave whose candidates stayed in its buffer finishes the step
// itself (wave_tail); the others leave their segment to wide_wtail_kernel.
template <typename T, bool DECODE, int NWV, int CW, int NR, bool INTAIL>
__device__ __forceinline__ void wide_stream_body(const StepParams& p, WideStat* ws, uint64_t* keys_in,
                                                 uint64_t* keys_out, unsigned int* count, int cap,
                                                 unsigned int* todo, uint64_t (*s_buf)[CW]) {
    constexpr int W = Elem<T>::W;
    constexpr int TS = WAVE * W;
    constexpr int WS_NK = NSG_WS_NK;  // sample tiles (in registers during the prologue, skipped by the stream)
    constexpr int WS_CW = CW;
    const int lane = (int)(threadIdx.x & (WAVE - 1));
    const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x / WAVE);
    const int b = __builtin_amdgcn_readfirstlane((int)blockIdx.x * NWV + wv);
    if (b >= p.B) return;
    const ns_stream_state st = p.state[b];
    bool active = !(st.flags & NS_ST_DONE);
    if (!DECODE && active && st.bit_pos >= p.nbits[b]) {
        if (lane == 0 && !(p.flags & NS_STEP_FINISH_SENT)) p.state[b].flags = st.flags | NS_ST_DONE;
        active = false;
    }
    if (DECODE && p.active && !p.active[b]) active = false;
    if (!active) {
        if (lane == 0) {
            ws[b].active = 0;
            count[b] = 0;
        }
        return;
    }
    NSG_STAMP_RT(p, b, lane, 9);
    NSG_STAMP(p, b, lane, 0);
    const int V = p.V;
    const char* rowc = (const char*)p.logits + (int64_t)b * p.ld * (int64_t)sizeof(T);
    const RowReader rd(rowc, (uint32_t)(p.ld * (int64_t)sizeof(T)));
    const int ntiles = (V + TS - 1) / TS;
    const double temp = 1.0 / p.inv_temp;
    const float tempf = (float)temp;
    const double Rd = (double)(st.hi - st.lo);
    const float lnthr = (float)(-log(Rd));
    uint64_t* wbuf = s_buf[wv];
    float* gv = seg_vals(keys_in, b, cap);
    uint32_t* gj = seg_ids(keys_in, b, cap);
    uint16_t* gj16 = (uint16_t*)gj;
    const bool id16 = V <= 65536;  // ids as 16-bit words: 6 bytes per segment entry

    // masked ids (past the row, banned): -1e30 and bit q of mb (never collected), bans walked in tile order
    int bi = 0, next_ban = 0x7FFFFFFF;
    auto ban_reset = [&]() __attribute__((always_inline)) {
        bi = 0;
        next_ban = p.nbanned > 0 ? p.banned[0] : 0x7FFFFFFF;
    };
    auto load_x = [&](int t, const uint4& raw, float (&x)[W], uint32_t& mb) __attribute__((always_inline)) {
        Elem<T>::unpack(raw, x);
        mb = 0u;
        const int j0 = t * TS + lane * W;
        if ((t + 1) * TS > V) {
#pragma unroll
            for (int q = 0; q < W; ++q)
                if (j0 + q >= V) {
                    x[q] = -1.0e30f;
                    mb |= 1u << q;
                }
        }
        while (next_ban < t * TS) {  // bans of skipped tiles
            ++bi;
            next_ban = bi < p.nbanned ? p.banned[bi] : 0x7FFFFFFF;
        }
        while (next_ban < (t + 1) * TS) {
            const int d = next_ban - j0;
            if (d >= 0 && d < W) {
#pragma unroll
                for (int q = 0; q < W; ++q)
                    if (q == d) {
                        x[q] = -1.0e30f;
                        mb |= 1u << q;
                    }
            }
            ++bi;
            next_ban = bi < p.nbanned ? p.banned[bi] : 0x7FFFFFFF;
        }
    };
    float r = 0.0f, nrc = 0.0f;
    float m1 = -__builtin_inff();
    double accS = 0.0, accT = 0.0;
    float accSf = 0.0f;
    auto sum_tile = [&](const float (&x)[W]) __attribute__((always_inline)) {
        typedef float f2 __attribute__((ext_vector_type(2)));
        const f2 c2 = {p.c32, p.c32}, n2 = {nrc, nrc};
        f2 a2 = {0.0f, 0.0f}, b2 = {0.0f, 0.0f};
#pragma unroll
        for (int q = 0; q < W; q += 2) {
            const f2 x2 = {x[q], x[q + 1]};
            const f2 t = __builtin_elementwise_fma(x2, c2, n2);
            const f2 e2 = {__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
            a2 += e2;
            b2 = __builtin_elementwise_fma(e2, t, b2);
            m1 = __builtin_fmaxf(__builtin_fmaxf(m1, x[q]), x[q + 1]);
        }
        const float a = a2.x + a2.y;
        accS += (double)a;
        accT += (double)(b2.x + b2.y);
        accSf += a;
    };
    int cnt = 0;       // entries in the LDS buffer (wave-uniform)
    uint32_t gcnt = 0;  // entries flushed to the segment
    float t_wave = -__builtin_inff();
    auto flush = [&]() __attribute__((always_inline)) {
        for (int i = lane; i < cnt; i += WAVE) {
            const uint64_t e = wbuf[i];
            gv[gcnt + i] = op_raw_val(e);
            if (id16)
                gj16[gcnt + i] = (uint16_t)e;
            else
                gj[gcnt + i] = (uint32_t)e;
        }
        gcnt += (uint32_t)cnt;
        cnt = 0;
    };
    auto append_tile = [&](int t, const float (&x)[W], uint32_t mb) __attribute__((always_inline)) {
#ifdef NSG_WS_NOAPPEND
        return;
#endif
        uint32_t c = 0u;
#pragma unroll
        for (int q = 0; q < W; ++q) c += (x[q] >= t_wave && !((mb >> q) & 1u)) ? 1u : 0u;
        const uint32_t incl = wave_incl_scan_u32(c);
        const int tot = __builtin_amdgcn_readlane((int)incl, WAVE - 1);
        if (tot == 0) return;
        if (cnt + tot > WS_CW) {
            cnt = wave_compact(wbuf, cnt, t_wave);
            if (cnt + tot > WS_CW || 2 * cnt > WS_CW) flush();
        }
        uint32_t pos = (uint32_t)cnt + incl - c;
        const uint32_t j0 = (uint32_t)(t * TS + lane * W);
#pragma unroll
        for (int q = 0; q < W; ++q)
            if (x[q] >= t_wave && !((mb >> q) & 1u)) wbuf[pos++] = op_raw(x[q], j0 + q);
        cnt += tot;
    };
    auto threshold = [&](float s_part) __attribute__((always_inline)) -> float {
        if (!(s_part > 0.0f && s_part < 3.0e38f)) return -__builtin_inff();
        const float L = __builtin_amdgcn_logf(s_part * 0.9990234375f) * 0.6931471805599453f + lnthr;
        const float t = r + tempf * L;
        return t - 1.0e-4f * (1.0f + fabsf(r) + fabsf(tempf * L));
    };

    // ---- sample: WS_NK whole tiles spread over the row (tile s*space + space-1) give r and the first threshold;
    // the ring's first tiles are in flight behind them.  Small rows (fewer than 2*WS_NK tiles): r = max of tile 0.
    const bool spec = ntiles >= 2 * WS_NK;
    const int space = spec ? ntiles / WS_NK : 1;
    const int nstream = spec ? ntiles - WS_NK : ntiles;
    int lt = 0, lc = spec ? space - 1 : 0x7FFFFFFF, sleft = spec ? WS_NK : 0;
    auto next_tile = [&]() __attribute__((always_inline)) -> int {
        const int t = lt++;
        if (--lc == 0) {
            ++lt;
            lc = --sleft > 0 ? space - 1 : 0x7FFFFFFF;
        }
        return t;
    };
    uint4 smp[WS_NK];
    if (spec) {
#pragma unroll
        for (int s = 0; s < WS_NK; ++s) smp[s] = rd.vec((s * space + space - 1) * WAVE + lane);
    }
    uint4 ring[NR];
    int rt[NR];
#pragma unroll
    for (int d = 0; d < NR; ++d) {
        rt[d] = next_tile();
        ring[d] = rd.vec(rt[d] * WAVE + lane);
    }
    float xt_run = -__builtin_inff();
    if (spec) {
        float smax = -__builtin_inff();
        ban_reset();
#pragma unroll
        for (int s = 0; s < WS_NK; ++s) {
            float x[W];
            uint32_t mb;
            load_x(s * space + space - 1, smp[s], x, mb);
#pragma unroll
            for (int q = 0; q < W; ++q) smax = fmaxf(smax, x[q]);
        }
        r = wave_max(smax);
        if (!(r > -1.0e29f)) r = 0.0f;
        nrc = -(r * p.c32);
        ban_reset();
#pragma unroll
        for (int s = 0; s < WS_NK; ++s) {
            float x[W];
            uint32_t mb;
            load_x(s * space + space - 1, smp[s], x, mb);
            sum_tile(x);
        }
        xt_run = threshold(wave_sum_f32(accSf));
        t_wave = xt_run;
        ban_reset();
#pragma unroll
        for (int s = 0; s < WS_NK; ++s) {
            float x[W];
            uint32_t mb;
            load_x(s * space + space - 1, smp[s], x, mb);
            append_tile(s * space + space - 1, x, mb);
        }
    } else {
        float x[W];
        uint32_t mb;
        ban_reset();
        load_x(0, ring[0], x, mb);
        float mx = x[0];
#pragma unroll
        for (int q = 1; q < W; ++q) mx = fmaxf(mx, x[q]);
        r = wave_max(mx);
        if (!(r > -1.0e29f)) r = 0.0f;
        nrc = -(r * p.c32);
    }
    NSG_STAMP(p, b, lane, 1);

    // ---- the stream: ring groups of NR tiles; the threshold rises once per group
    ban_reset();
    int pos = 0;
    for (; pos + NR <= nstream; pos += NR) {
        // one tile at a time (its slot refilled as soon as it is unpacked): a single tile's values are live
#pragma unroll
        for (int d = 0; d < NR; ++d) {
            const int jt = rt[d];
            float x[W];
            uint32_t mb;
            load_x(jt, ring[d], x, mb);
            rt[d] = next_tile();
            ring[d] = rd.vec(rt[d] * WAVE + lane);
            sum_tile(x);
            append_tile(jt, x, mb);
        }
        xt_run = fmaxf(xt_run, threshold(wave_sum_f32(accSf)));
        t_wave = xt_run;
    }
#pragma unroll
    for (int d = 0; d < NR; ++d) {
        if (pos + d < nstream) {
            float x[W];
            uint32_t mb;
            load_x(rt[d], ring[d], x, mb);
            sum_tile(x);
            append_tile(rt[d], x, mb);
        }
    }
    NSG_STAMP(p, b, lane, 2);

    // ---- the proven interval, the final threshold, the buffer filtered to it and flushed
    accS = wave_sum_butterfly(accS);
    accT = wave_sum_butterfly(accT);
    float bm1 = wave_max(m1);
    if (!(bm1 > -1.0e29f)) bm1 = -__builtin_inff();
    WideStat w;
    double Sf = 0.0, S_lo = 0.0, S_hi = 0.0;
    const bool ok = fast_sum_interval_dd(accS, accT, r, (double)(bm1 + 0.0f), p.c32, p.inv_temp, W, Sf, S_lo, S_hi);
    w.m = bm1;
    w.m2 = -__builtin_inff();
    w.r = r;
    w.active = 1;
    w.S_lo = S_lo;
    w.S_hi = S_hi;
    w.S_fast = Sf;
    w.exact = (ok && !(p.flags & NS_STEP_FORCE_EXACT_SUM)) ? 0u : 1u;
    w.pad = 0;
    w.S_r = accS;
    w.B_r = 0.0;
    w.U_r = 0.0;
    float xt = -__builtin_inff();
    if (ok) {
        const double L = log(S_lo / Rd);
        const double t = (double)w.m + temp * L;
        xt = (float)(t - 1.0e-4 * (1.0 + fabs((double)w.m) + fabs(temp * L)));
    }
    xt = fmaxf(xt, xt_run);
    t_wave = xt;
    cnt = wave_compact(wbuf, cnt, t_wave);
    w.xt = xt;
    if constexpr (INTAIL) {
        // every candidate is still in the buffer: this wave finishes the step (else the segment goes to the tail
        // kernel, which also takes the exact row sum and the sweep for a peaked row)
        if (gcnt == 0 && !w.exact && cnt >= 2) {
            NSG_STAMP(p, b, lane, 3);
            wave_tail<T, DECODE>(p, &ws[b], w, b, st, wbuf, cnt, keys_out, count, cap, todo);
            return;
        }
    }
    flush();
    w.nraw = gcnt;
    if (lane == 0) {
        ws[b] = w;
        count[b] = gcnt;
    }
    NSG_STAMP(p, b, lane, 3);
}

template <typename T, bool DECODE>
__global__ __launch_bounds__(WS_WAVES* WAVE, 4) void wide_stream_kernel(StepParams p, WideStat* ws, uint64_t* keys_in,
                                                                        unsigned int* count, int cap,
                                                                        unsigned int* todo, unsigned int* todo2) {
    __shared__ uint64_t s_buf[WS_WAVES][WS_CW];
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // the step's two work lists start empty (no memset launches)
        todo[0] = 0u;
        todo2[0] = 0u;
    }
    wide_stream_body<T, DECODE, WS_WAVES, WS_CW, NSG_WS_NR, false>(p, ws, keys_in, nullptr, count, cap, todo, s_buf);
}

// the wave-per-stream step: one 64-thread workgroup per stream, a WV_CW-entry LDS buffer (its ~4,000 kept ids
// stay on chip), a WV_NR-tile load ring (one wave per SIMD: the ring is what keeps bytes in flight), the tail in
// the same wave
#ifndef NSG_WV_NR
#define NSG_WV_NR 12
#endif
template <typename T, bool DECODE>
__global__ __launch_bounds__(WAVE, 1) void wide_wave_kernel(StepParams p, WideStat* ws, uint64_t* keys_in,
                                                            uint64_t* keys_out, unsigned int* count, int cap,
                                                            unsigned int* todo, unsigned int* todo2) {
    __shared__ uint64_t s_buf[1][WV_CW];
    if (blockIdx.x == 0 && threadIdx.x == 0) todo2[0] = 0u;  // the hand-off kernel's list (todo: memset before)
    wide_stream_body<T, DECODE, 1, WV_CW, NSG_WV_NR, true>(p, ws, keys_in, keys_out, count, cap, todo, s_buf);
}

// the list path for one stream of the tail kernel: its collected keys (x >= xt) go to keys_out (unsorted) for the
// device sort; exact: the list kernel computes the exact row sum.  Fewer than two keys (a peaked row whose second
// largest value is below the running threshold): the row is swept again for x >= min(xt, second largest).
template <typename T>
__device__ void wtail_defer(const StepParams& p, WideStat* wsb, int b, const float* gv, const uint32_t* gj, int n,
                            float xt, uint64_t* keys_out, unsigned int* count, int cap, unsigned int* todo, bool exact,
                            uint32_t* s_ctr, float* s_top) {
    const int tid = (int)threadIdx.x, lane = tid & (WAVE - 1), wv = tid / WAVE;
    uint64_t* ko = keys_out + (int64_t)b * cap;
    __syncthreads();
    if (tid == 0) *s_ctr = 0u;
    __syncthreads();
    for (int i = tid; i < n; i += WT_THREADS) {
        const float v = gv[i];
        if (v >= xt) ko[atomicAdd(s_ctr, 1u)] = wkey(v, seg_id(gj, i, p.V <= 65536));
    }
    __syncthreads();
    uint32_t got = *s_ctr;
    if (got < 2u && (int)got < p.V - p.nbanned) {
        // the row's two largest valid values, then every valid id at or above the second one (block sweeps)
        constexpr int W = Elem<T>::W;
        const char* rowc = (const char*)p.logits + (int64_t)b * p.ld * (int64_t)sizeof(T);
        const RowReader rd(rowc, (uint32_t)(p.ld * (int64_t)sizeof(T)));
        const int nvec = (p.V + W - 1) / W;
        float l1 = -__builtin_inff(), l2 = -__builtin_inff();
        for (int v = tid; v < nvec; v += WT_THREADS) {
            float x[W];
            Elem<T>::unpack(rd.vec(v), x);
#pragma unroll
            for (int q = 0; q < W; ++q) {
                const int j = v * W + q;
                const float y = (j < p.V && !is_banned(p, j)) ? x[q] : -__builtin_inff();
                l2 = fmaxf(l2, fminf(l1, y));
                l1 = fmaxf(l1, y);
            }
        }
        wave_top2(l1, l2);
        if (lane == 0) {
            s_top[2 * wv] = l1;
            s_top[2 * wv + 1] = l2;
        }
        __syncthreads();
        float b1 = -__builtin_inff(), b2 = -__builtin_inff();
#pragma unroll
        for (int i = 0; i < WT_WAVES; ++i) {
            b2 = fmaxf(fminf(b1, s_top[2 * i]), fmaxf(b2, s_top[2 * i + 1]));
            b1 = fmaxf(b1, s_top[2 * i]);
        }
        const float thr = fminf(xt, b2);
        if (tid == 0) *s_ctr = 0u;
        __syncthreads();
        for (int v = tid; v < nvec; v += WT_THREADS) {
            float x[W];
            Elem<T>::unpack(rd.vec(v), x);
#pragma unroll
            for (int q = 0; q < W; ++q) {
                const int j = v * W + q;
                if (j < p.V && !is_banned(p, j) && x[q] >= thr) {
                    const uint32_t at = atomicAdd(s_ctr, 1u);
                    if (at < (uint32_t)cap) ko[at] = wkey(x[q], (uint32_t)j);
                }
            }
        }
        __syncthreads();
        got = min(*s_ctr, (uint32_t)cap);
        if (tid == 0 && p.counters) atomicAdd(&p.counters[4 * (b & (NS_COUNTER_SHARDS - 1)) + 1], 1ull);
    }
    if (tid == 0) {
        count[b] = got;
        wsb->pad = 1u;
        if (exact) wsb->exact = 1u;
        todo[1 + atomicAdd(&todo[0], 1u)] = (unsigned int)b;
    }
}

#ifndef NSG_WT_WAVES_PER_SIMD
#define NSG_WT_WAVES_PER_SIMD 4  // 40 KiB of LDS per workgroup: four per CU
#endif
template <typename T, bool DECODE>
__global__ __launch_bounds__(WT_THREADS, NSG_WT_WAVES_PER_SIMD) void wide_wtail_kernel(
    StepParams p, WideStat* ws, uint64_t* keys_in, uint64_t* keys_out, unsigned int* count, int cap,
    unsigned int* todo) {
    __shared__ uint32_t s_cnt[WT_NB];   // bucket counts, then their exclusive prefix
    __shared__ uint64_t s_q[WT_NB];     // bucket q sums, then their exclusive prefix
    __shared__ uint64_t s_mem[WT_GM];   // members of the searched bucket: keys
    __shared__ int64_t s_memq[WT_GM];   //   and q
    __shared__ double s_d[4 * WT_WAVES];
    __shared__ uint64_t s_w[8 * WT_WAVES];
    __shared__ uint32_t s_ctr[4];
    __shared__ float s_top[2 * WT_WAVES];
    __shared__ int64_t s_res[8];
    __shared__ float s_vals[WT_LV];
    const int b = blockIdx.x;
    WideStat* wsb = &ws[b];
    const WideStat w = *wsb;
    if (!w.active || w.pad) return;  // finished by the wave-per-stream step, or already on the hand-off list
    const int tid = (int)threadIdx.x, lane = tid & (WAVE - 1), wv = tid / WAVE;
    NSG_STAMP(p, b, tid, 11);
    float* gv = seg_vals(keys_in, b, cap);
    uint32_t* gj = seg_ids(keys_in, b, cap);
    const float xt = w.xt;
    int n = (int)w.nraw;
    const ns_stream_state st = p.state[b];
    if (w.exact) {
        wtail_defer<T>(p, wsb, b, gv, gj, n, xt, keys_out, count, cap, todo, true, s_ctr, s_top);
        return;
    }
    // the segment's values are read once into LDS (up to WT_LV of them; a longer segment -- a flat row -- is
    // streamed from global memory by every pass); stale entries (x < xt) are skipped by every pass
    const float* src = gv;
    if (n <= WT_LV) {
        for (int i = tid; i < n; i += WT_THREADS) s_vals[i] = gv[i];
        __syncthreads();
        src = s_vals;
    }
    auto for_each = [&](auto&& fn) __attribute__((always_inline)) {
        for (int i0 = tid; i0 < n; i0 += WT_U * WT_THREADS) {
            float xv[WT_U];
#pragma unroll
            for (int u = 0; u < WT_U; ++u) {
                const int i = i0 + u * WT_THREADS;
                xv[u] = i < n ? src[i] : -__builtin_inff();
            }
#pragma unroll
            for (int u = 0; u < WT_U; ++u)
                if (xv[u] >= xt) fn(xv[u], i0 + u * WT_THREADS);
        }
    };
    s_cnt[tid] = 0u;
    s_q[tid] = 0ull;
    const uint64_t R = st.hi - st.lo;
    const double Rd = (double)R, thr = 1.0 / Rd;
    const double inv_lo = 1.0 / (w.S_lo * (1.0 - 1.0e-15)), inv_hi = 1.0 / (w.S_hi * (1.0 + 1.0e-15));
    const double m = (double)w.m;
    // ---- A: exps, cutoff, limb mass (the kept set is x >= vk: e is monotone in x)
    Mass ms{0.0, 0.0, 0.0, 0.0};
    uint32_t nk = 0u;
    bool amb = false;
    float vk = __builtin_inff();
    for_each([&](float xv, int) __attribute__((always_inline)) {
        const double e = exp_canon(((double)xv - m) * p.inv_temp);
        if (e * inv_lo < thr) return;
        amb |= !(e * inv_hi >= thr);
        ++nk;
        vk = fminf(vk, xv);
        mass_add(ms, e);
    });
    mass_wave_sum(ms);
    {
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan_u32(nk), WAVE - 1);
        const float wvk = -wave_max(-vk);
        const bool wamb = ballot(amb) != 0ull;
        if (lane == 0) {
            s_d[4 * wv + 0] = ms.a;
            s_d[4 * wv + 1] = ms.b;
            s_d[4 * wv + 2] = ms.c;
            s_d[4 * wv + 3] = ms.d;
            s_w[wv] = (uint64_t)tot | ((uint64_t)(wamb ? 1u : 0u) << 32);
            s_top[wv] = wvk;
        }
    }
    __syncthreads();
    Mass tot{0.0, 0.0, 0.0, 0.0};
    int k0 = 0;
    bool amb_a = false;
    vk = __builtin_inff();
#pragma unroll
    for (int i = 0; i < WT_WAVES; ++i) {
        tot.a += s_d[4 * i + 0];
        tot.b += s_d[4 * i + 1];
        tot.c += s_d[4 * i + 2];
        tot.d += s_d[4 * i + 3];
        k0 += (int)(uint32_t)s_w[i];
        amb_a |= (s_w[i] >> 32) != 0ull;
        vk = fminf(vk, s_top[i]);
    }
    const double E = mass_value(tot);
    // decode: the received token must be kept (x >= vk), else the list path reports the divergence
    float xtok = -__builtin_inff();
    uint64_t kt = 0ull;
    bool tok_ok = true;
    if (DECODE) {
        const int32_t tok = p.in_token[b];
        tok_ok = tok >= 0 && tok < p.V && !is_banned(p, tok);
        if (tok_ok) {
            const char* rowc = (const char*)p.logits + (int64_t)b * p.ld * (int64_t)sizeof(T);
            xtok = Elem<T>::load1(rowc, tok);
            kt = wkey(xtok, (uint32_t)tok);
            tok_ok = xtok >= vk;
        }
    }
    if (amb_a || k0 < 2 || k0 > p.topk || k0 > p.K || !tok_ok || !(E > 0.0 && E <= 1.7976931348623157e308)) {
        wtail_defer<T>(p, wsb, b, gv, gj, n, xt, keys_out, count, cap, todo, amb_a, s_ctr, s_top);
        return;
    }
    NSG_STAMP(p, b, tid, 5);
    // ---- C: q_i and the bucket histogram over [vk, m] (linear in x: monotone, ties share a bucket)
    const float fm = w.m;
    const float bscale = fm > vk ? (float)WT_NB / (fm - vk) : 0.0f;
    auto bucket_of = [&](float v) __attribute__((always_inline)) -> uint32_t {
        return min((uint32_t)((fm - v) * bscale), (uint32_t)(WT_NB - 1));
    };
    for_each([&](float xv, int) __attribute__((always_inline)) {
        if (!(xv >= vk)) return;  // kept <=> x >= vk
        const double e = exp_canon(((double)xv - m) * p.inv_temp);
        const uint64_t q = (uint64_t)(int64_t)__builtin_rint((e / E) * Rd);
        const uint32_t bk = bucket_of(xv);
        atomicAdd(&s_cnt[bk], 1u);
        atomicAdd((unsigned long long*)&s_q[bk], (unsigned long long)q);
    });
    __syncthreads();
    // ---- prefixes (thread t owns bucket t), the overfill bucket
    const uint32_t c = s_cnt[tid];
    const int64_t qv = (int64_t)s_q[tid];
    const uint32_t ci = wave_incl_scan_u32(c);
    const int64_t qi = wave_incl_scan(qv, lane);
    if (lane == WAVE - 1) {
        s_w[8 + wv] = (uint64_t)qi;
        s_w[16 + wv] = (uint64_t)ci;
    }
    __syncthreads();
    int64_t qbefore = 0, Q = 0;
    uint32_t cbefore = 0u;
#pragma unroll
    for (int i = 0; i < WT_WAVES; ++i) {
        const int64_t tq = (int64_t)s_w[8 + i];
        if (i < wv) {
            qbefore += tq;
            cbefore += (uint32_t)s_w[16 + i];
        }
        Q += tq;
    }
    const int64_t QP = qbefore + qi - qv;
    const uint32_t CP = cbefore + ci - c;
    s_cnt[tid] = CP;  // own slot: read above by this thread only
    s_q[tid] = (uint64_t)QP;
    int ovf = (Q > (int64_t)R && QP + qv > (int64_t)R) ? tid : WT_NB;
    ovf = wave_min_int(ovf);
    if (lane == 0) s_w[24 + wv] = (uint64_t)(uint32_t)ovf;
    __syncthreads();
    int b_ov = WT_NB;
#pragma unroll
    for (int i = 0; i < WT_WAVES; ++i) b_ov = min(b_ov, (int)(uint32_t)s_w[24 + i]);
    NSG_STAMP(p, b, tid, 6);
    // inclusive prefix of bucket bk (the last bucket: Q)
    auto incl_of = [&](int bk) __attribute__((always_inline)) -> int64_t {
        return bk + 1 < WT_NB ? (int64_t)s_q[bk + 1] : Q;
    };
    // ---- gather the kept members of bucket `bk` (block-uniform) into s_mem / s_memq; returns their count
    auto gather = [&](int bk) __attribute__((always_inline)) -> int {
        if (tid == 0) s_ctr[0] = 0u;
        __syncthreads();
        for_each([&](float xv, int i) __attribute__((always_inline)) {
            if (!(xv >= vk) || (int)bucket_of(xv) != bk) return;
            const uint32_t at = atomicAdd(&s_ctr[0], 1u);
            if (at < (uint32_t)WT_GM) {
                const double e = exp_canon(((double)xv - m) * p.inv_temp);
                s_mem[at] = wkey(xv, seg_id(gj, i, p.V <= 65536));
                s_memq[at] = (int64_t)__builtin_rint((e / E) * Rd);
            }
        });
        __syncthreads();
        return (int)s_ctr[0];
    };
    // wave 0: member `lane + 64 j` of the gathered bucket: key, q, rank among the members, cum = inclusive prefix
    struct Mem {
        uint64_t key[WT_GM / WAVE];
        int64_t q[WT_GM / WAVE], cum[WT_GM / WAVE];
        int rank[WT_GM / WAVE];
    };
    auto resolve = [&](int bk, int nm, Mem& mm) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < WT_GM / WAVE; ++j) {
            const int i = lane + WAVE * j;
            mm.key[j] = i < nm ? s_mem[i] : 0ull;
            mm.q[j] = i < nm ? s_memq[i] : 0;
            mm.rank[j] = 0;
            mm.cum[j] = 0;
        }
        for (int o = 0; o < nm; ++o) {
            const uint64_t ko = s_mem[o];
            const int64_t qo = s_memq[o];
#pragma unroll
            for (int j = 0; j < WT_GM / WAVE; ++j) {
                mm.rank[j] += ko > mm.key[j] ? 1 : 0;
                mm.cum[j] += ko >= mm.key[j] ? qo : 0;
            }
        }
#pragma unroll
        for (int j = 0; j < WT_GM / WAVE; ++j) mm.cum[j] += (int64_t)s_q[bk];
    };
    // ---- overfill: kp = first rank whose cum exceeds R (b_ov == WT_NB: none, kp = k0)
    int kp = k0, kp_local = WT_GM + 1;
    int64_t cumkp = Q;
    if (b_ov < WT_NB) {
        const int nm = gather(b_ov);
        if (nm > WT_GM) {  // a crowded bucket (ties, skewed rows): counted like the LDS sort's bitonic fallback
            if (tid == 0 && p.counters) atomicAdd(&p.counters[4 * (b & (NS_COUNTER_SHARDS - 1)) + 3], 1ull);
            wtail_defer<T>(p, wsb, b, gv, gj, n, xt, keys_out, count, cap, todo, false, s_ctr, s_top);
            return;
        }
        if (wv == 0) {
            Mem mm;
            resolve(b_ov, nm, mm);
            int kl = WT_GM + 1;
#pragma unroll
            for (int j = 0; j < WT_GM / WAVE; ++j)
                if (lane + WAVE * j < nm && mm.cum[j] > (int64_t)R) kl = min(kl, mm.rank[j]);
            kl = wave_min_int(kl);
            int64_t cprev = (int64_t)s_q[b_ov];
#pragma unroll
            for (int j = 0; j < WT_GM / WAVE; ++j) {
                const uint64_t mp = ballot(lane + WAVE * j < nm && mm.rank[j] == kl - 1);
                if (mp) cprev = (int64_t)readlane_u64((uint64_t)mm.cum[j], __builtin_ctzll(mp));
            }
            if (lane == 0) {
                s_res[0] = kl;
                s_res[1] = cprev;
            }
        }
        __syncthreads();
        kp_local = (int)s_res[0];
        kp = (int)s_cnt[b_ov] + kp_local;
        cumkp = s_res[1];
    }
    const int64_t shift = (int64_t)R - cumkp + (int64_t)st.lo;
    // ---- the searched bucket: encode, the first bucket (<= b_ov) whose inclusive cum + shift exceeds the payload
    // index; decode, the token's bucket (it must lie before the overfill point)
    uint64_t idx = 0ull;
    int bsel;
    if (!DECODE) {
        if (wv == 0) {
            idx = payload_window(p, b, st.bit_pos);
            int bl = WT_NB;
#pragma unroll
            for (int j = 0; j < WT_NB / WAVE; ++j) {
                const int bk = lane * (WT_NB / WAVE) + j;
                if (bk <= b_ov && bk < WT_NB && bl == WT_NB) {
                    const int64_t inc = bk == b_ov ? cumkp : incl_of(bk);
                    if ((uint64_t)(inc + shift) > idx) bl = bk;
                }
            }
            bl = wave_min_int(bl);
            if (lane == 0) {
                s_res[2] = bl;
                s_res[3] = (int64_t)idx;
            }
        }
        __syncthreads();
        bsel = (int)s_res[2];
        idx = (uint64_t)s_res[3];
    } else {
        bsel = (int)bucket_of(xtok);
    }
    if (bsel >= WT_NB || bsel > b_ov) {  // encode range error, or a decode token past the overfill point
        wtail_defer<T>(p, wsb, b, gv, gj, n, xt, keys_out, count, cap, todo, false, s_ctr, s_top);
        return;
    }
    int nm = 0;
    if (bsel != b_ov) {
        nm = gather(bsel);
    } else {
        nm = (int)s_ctr[0];  // still gathered
    }
    if (nm > WT_GM) {
        if (tid == 0 && p.counters) atomicAdd(&p.counters[4 * (b & (NS_COUNTER_SHARDS - 1)) + 3], 1ull);
        wtail_defer<T>(p, wsb, b, gv, gj, n, xt, keys_out, count, cap, todo, false, s_ctr, s_top);
        return;
    }
    int found = 0;
    if (wv == 0) {
        Mem mm;
        resolve(bsel, nm, mm);
        int rl = WT_GM + 1;
#pragma unroll
        for (int j = 0; j < WT_GM / WAVE; ++j) {
            const bool valid = lane + WAVE * j < nm && (bsel != b_ov || mm.rank[j] < kp_local);
            const bool hit = DECODE ? (valid && mm.key[j] == kt) : (valid && (uint64_t)(mm.cum[j] + shift) > idx);
            if (hit) rl = min(rl, mm.rank[j]);
        }
        rl = wave_min_int(rl);
        int64_t cum_sel = 0, q_sel = 0;
        uint64_t key_sel = 0ull;
#pragma unroll
        for (int j = 0; j < WT_GM / WAVE; ++j) {
            const uint64_t mh = ballot(lane + WAVE * j < nm && mm.rank[j] == rl);
            if (mh) {
                const int src = __builtin_ctzll(mh);
                cum_sel = (int64_t)readlane_u64((uint64_t)mm.cum[j], src);
                q_sel = (int64_t)readlane_u64((uint64_t)mm.q[j], src);
                key_sel = readlane_u64(mm.key[j], src);
            }
        }
        found = rl <= WT_GM;
        if (found && lane == 0) {
            const int sel = (int)s_cnt[bsel] + rl;
            const RowStats rs{0.0, 0.0, 0.0};
            wide_finish<DECODE>(p, b, st, k0, kp, sel, false, w.S_fast, sel > 0 ? cum_sel - q_sel : 0, cum_sel, shift,
                                key_sel, m, rs, 0.0, false);
        }
        if (lane == 0) s_res[4] = found;
    }
    __syncthreads();
    if (!s_res[4]) wtail_defer<T>(p, wsb, b, gv, gj, n, xt, keys_out, count, cap, todo, false, s_ctr, s_top);
    NSG_STAMP(p, b, tid, 8);
    NSG_STAMP_RT(p, b, tid, 10);
}

// The streams the tail kernel handed on (todo): up to FAST_NL collected keys are sorted in LDS and finished by
// fast_tail (the exact row sum in the workgroup when needed); its own hand-offs (errors, non-finite rows) and the
// longer segments (flat rows: pad stays set, the device-wide sort) go on to wide_cdf_kernel through todo2.  A
// grid-stride loop over the list, so the launch does not depend on how many there are.
template <typename T, bool DECODE>
__global__ __launch_bounds__(FAST_THREADS) void wide_wlist_kernel(StepParams p, WideStat* ws, uint64_t* keys_in,
                                                                  uint64_t* keys_out, const unsigned int* count,
                                                                  int cap, const unsigned int* todo,
                                                                  unsigned int* todo2) {
    __shared__ uint64_t s_keys[FAST_NL];
    __shared__ uint64_t s_aux[FAST_NB / 2];
    const unsigned int nt = todo[0];
    for (unsigned int i = blockIdx.x; i < nt; i += gridDim.x) {
        const int b = (int)todo[1 + i];
        const int n = (int)count[b];
        if (n >= 2 && n <= FAST_NL) {
            const WideStat w = ws[b];
            __syncthreads();
            if (threadIdx.x == 0) ws[b].pad = 0u;  // sorted here, not by the device-wide sort
            fast_tail<T, DECODE, true>(p, w, &ws[b], b, n, KeysFlat{keys_out + (int64_t)b * cap, n}, keys_in, cap,
                                       todo2, s_keys, s_aux);
        } else if (threadIdx.x == 0) {
            todo2[1 + atomicAdd(&todo2[0], 1u)] = (unsigned int)b;
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------ rank coder
// src/neuralstego/codec/arithmetic.py:122-231 (encode_with_lm / decode_with_lm) with apply_quality /
// cap_bits_per_token (codec/quality.py:57-141).  Two row forms share the quality cut (R2), the capacity cap (R3) and
// the selection / emission (R4): wide_rank_kernel ranks the _ModelAdapter softmax of a logit row (canonical steps
// R1-R4 of oracle/nsg_oracle.c), wide_rank64_kernel a generic provider's own float64 ProbDist (P0-P5).

// R2: top_k, top_p (left-to-right cumsum over ranks [0, V), searchsorted 'left'), min_prob cut the support [0, n)
template <class PF>
__device__ int rank_quality_cut(const StepParams& p, int V, int n, PF&& pf, double* ebuf, int* smi, int& cut_sh,
                                double& acc_sh) {
    const int tid = threadIdx.x;
    if (p.rk_top_k > 0) n = min(n, p.rk_top_k);
    if (p.rk_top_p > 0.0) {
        if (tid == 0) {
            cut_sh = V;
            acc_sh = 0.0;
        }
        __syncthreads();
        for (int base = 0; base < V; base += WIDE_ROUND) {
            for (int i = tid; i < WIDE_ROUND; i += WIDE_THREADS) ebuf[i] = (base + i < V) ? pf(base + i) : 0.0;
            __syncthreads();
            if (tid == 0 && cut_sh == V) {
                double a = acc_sh;
                for (int i = 0; i < WIDE_ROUND && base + i < V; ++i) {
                    a += ebuf[i];
                    if (a >= p.rk_top_p) {
                        cut_sh = base + i;
                        break;
                    }
                }
                acc_sh = a;
            }
            __syncthreads();
            if (cut_sh != V) break;
        }
        n = min(n, min(cut_sh + 1, V));
        __syncthreads();
    }
    if (p.rk_min_prob >= 0.0) {
        int fm = V;
        for (int i = tid; i < V; i += WIDE_THREADS)
            if (i < fm && !(pf(i) >= p.rk_min_prob)) fm = i;
        n = min(n, block_min_int(fm, smi));
    }
    return n;
}

// R3: cap_per_token_bits -- entropy of the renormalised support; bisect tau on softmax(log(f+1e-12)/tau) over the
// universe of U ranks (float64, libm-equivalent log/exp: tolerance-level); returns the new support
template <class PF>
__device__ int rank_cap(const StepParams& p, int U, int n, PF&& pf, double* sm64, int* smi) {
    const int tid = threadIdx.x;
    if (!(p.rk_cap > 0 && n > 0)) return n;
    double fl = 0.0;
    for (int i = tid; i < n; i += WIDE_THREADS) fl += pf(i);
    const double F = block_sum(fl, sm64);
    double hl = 0.0;
    for (int i = tid; i < n; i += WIDE_THREADS) {
        const double f = pf(i) / F;
        if (f > 0.0) hl -= f * log2(f);
    }
    const double H = block_sum(hl, sm64);
    if (!(H > (double)p.rk_cap)) return n;
    const double lf0 = log(pf(0) / F + 1e-12);
    double low = 1e-6, high = 1.0;
    int n_target = n;
    for (int it = 0; it < 60; ++it) {
        const double mid = (low + high) / 2.0;
        const double mx = lf0 / mid;
        double sl = 0.0, tl = 0.0;
        int zl = U;
        for (int i = tid; i < U; i += WIDE_THREADS) {
            const double f = i < n ? pf(i) / F : 0.0;
            const double a = log(f + 1e-12) / mid - mx;
            const double c = exp(a);
            if (c > 0.0) {
                sl += c;
                tl += c * a;
            } else if (i < zl) {
                zl = i;
            }
        }
        const double s = block_sum(sl, sm64);
        const double t = block_sum(tl, sm64);
        const int nz = block_min_int(zl, smi);
        const double Hc = (log(s) - t / s) / 0.6931471805599453;  // entropy of c/s in bits
        if (Hc > (double)p.rk_cap) {
            high = mid;
        } else {
            low = mid;
            n_target = nz;
        }
    }
    return n_target;
}

// R4: capacity c = floor(log2 n); encode: the next c payload bits (MSB-first per byte, zero padded) select the
// rank, token = id_of(rank); decode: the received token's rank among the first 2^c (is_token(rank)), its first
// keep bits emitted.  Every thread of the block calls it.
template <bool DECODE, class IDF, class HITF>
__device__ void rank_emit(const StepParams& p, int b, const ns_stream_state& st, int n, double S, IDF&& id_of,
                          HITF&& is_token, int* smi) {
    const int tid = threadIdx.x;
    int c = 0;
    while (c < 30 && (1 << (c + 1)) <= n) ++c;
    if (c <= 0) {
        if (tid == 0) p.state[b].flags = st.flags | (DECODE ? NS_ST_ERR_DIVERGE : NS_ST_ERR_RANGE) | NS_ST_DONE;
        return;
    }
    if (!DECODE) {
        if (tid != 0) return;
        const int64_t nbits = p.nbits[b];
        const uint8_t* pl = p.payload + (int64_t)b * p.payload_stride;
        uint32_t idx = 0;
        int take = 0;
        for (int t = 0; t < c; ++t) {
            const int64_t bp = st.bit_pos + t;
            uint32_t bit = 0;
            if (bp < nbits) {
                bit = (pl[bp >> 3] >> (7 - (bp & 7))) & 1u;
                ++take;
            }
            idx = (idx << 1) | bit;
        }
        const int32_t token = id_of((int)idx);
        ns_stream_state ns = st;
        ns.bit_pos = st.bit_pos + take;
        ns.ntokens = st.ntokens + 1;
        if (ns.bit_pos >= nbits) ns.flags |= NS_ST_DONE;
        p.state[b] = ns;
        p.out_token[b] = token;
        if (p.hist && st.ntokens < p.hist_stride) p.hist[(int64_t)b * p.hist_stride + st.ntokens] = token;
        if (p.rk_cons && st.ntokens < p.hist_stride) p.rk_cons[(int64_t)b * p.hist_stride + st.ntokens] = take;
        if (p.trace) {
            ns_step_trace tr = {n, c, (int)idx, take, token, 0, S};
            p.trace[b] = tr;
        }
        return;
    }
    const int32_t tok = p.in_token[b];
    int found = 0x7FFFFFFF;
    for (int i = tid; i < (1 << c); i += WIDE_THREADS)
        if (is_token(i, tok)) found = min(found, i);
    const int idx = block_min_int(found, smi);
    if (tid != 0) return;
    if (idx == 0x7FFFFFFF) {
        p.state[b].flags = st.flags | NS_ST_ERR_DIVERGE | NS_ST_DONE;
        return;
    }
    const int keep = min(max(p.rk_keep[b], 0), c);
    uint8_t* ob = p.out_bits + (int64_t)b * p.out_stride;
    for (int t = 0; t < keep; ++t) {
        const int64_t bp = st.bit_pos + t;
        const uint8_t bitv = (uint8_t)((idx >> (c - 1 - t)) & 1);
        const uint8_t m = (uint8_t)(0x80u >> (bp & 7));
        ob[bp >> 3] = bitv ? (uint8_t)(ob[bp >> 3] | m) : (uint8_t)(ob[bp >> 3] & ~m);
    }
    ns_stream_state ns = st;
    ns.bit_pos = st.bit_pos + keep;
    ns.ntokens = st.ntokens + 1;
    p.state[b] = ns;
    if (p.trace) {
        ns_step_trace tr = {n, c, idx, keep, tok, 0, S};
        p.trace[b] = tr;
    }
}

// Logit rows (the _ModelAdapter softmax, lm/arithmetic.py:45-74): canonical steps R1-R4 of oracle/nsg_oracle.c.
// keys_sorted holds every id of the row in rank order.
template <typename T, bool DECODE>
__global__ __launch_bounds__(WIDE_THREADS) void wide_rank_kernel(StepParams p, const WideStat* ws,
                                                                 const uint64_t* keys_sorted,
                                                                 const unsigned int* count, int cap) {
    __shared__ double ebuf[WIDE_ROUND];
    __shared__ double sm64[64];
    __shared__ int smi[16];
    __shared__ int cut_sh;
    __shared__ double acc_sh;
    const int b = blockIdx.x;
    const WideStat w = ws[b];
    if (!w.active) return;
    const int tid = threadIdx.x;
    const ns_stream_state st = p.state[b];
    const uint64_t* sk = keys_sorted + (int64_t)b * cap;
    const int V = (int)count[b];
    const double temp = 1.0 / p.inv_temp;
    const double zmax = (double)wkey_val(sk[0]) / temp;
    auto e_of = [&](int i) -> double { return exp_canon((double)wkey_val(sk[i]) / temp - zmax); };

    // R1: S in the canonical rank order, p_i = e_i / S, n0 = #nonzero (a prefix)
    double acc = 0.0;
    for (int base = 0; base < V; base += WIDE_ROUND) {
        for (int i = tid; i < WIDE_ROUND; i += WIDE_THREADS) ebuf[i] = (base + i < V) ? e_of(base + i) : 0.0;
        __syncthreads();
        if (tid < 64)
            for (int i = tid; i < WIDE_ROUND && base + i < V; i += 64) acc += ebuf[i];
        __syncthreads();
    }
    if (tid < 64) sm64[tid] = acc;
    __syncthreads();
    const double S = block_canonical_butterfly(sm64);
    auto p_of = [&](int i) -> double { return e_of(i) / S; };
    int fz = V;
    for (int i = tid; i < V; i += WIDE_THREADS)
        if (i < fz && e_of(i) == 0.0) fz = i;
    int n = block_min_int(fz, smi);

    // R1c: crypto quality LM (crypto/quality.py:57-64): temperature on the probabilities,
    // q_i = exp(log(p_i + 1e-12)/T - max) normalised -- every id keeps mass unless exp underflows.
    // Monotone in p, so the rank order is unchanged; libm-equivalent log/exp (tolerance-level).
    const double Tq = p.rk_ptemp;
    const bool crypto = Tq > 0.0;
    double a0 = 0.0, Q = 1.0;
    if (crypto) {
        a0 = log(p_of(0) + 1e-12) / Tq;
        double ql = 0.0;
        int zq = V;
        for (int i = tid; i < V; i += WIDE_THREADS) {
            const double q = exp(log(p_of(i) + 1e-12) / Tq - a0);
            ql += q;
            if (q == 0.0 && i < zq) zq = i;
        }
        Q = block_sum(ql, sm64);
        n = block_min_int(zq, smi);
    }
    auto pf = [&](int i) -> double { return crypto ? exp(log(p_of(i) + 1e-12) / Tq - a0) / Q : p_of(i); };

    n = rank_quality_cut(p, V, n, pf, ebuf, smi, cut_sh, acc_sh);
    // next_token_probs (codec/distribution.py:107-142): the quality-filtered support renormalised, by id
    if (p.probs_out) {
        const bool filtered = p.rk_top_k > 0 || p.rk_top_p > 0.0 || p.rk_min_prob >= 0.0;
        const int keep = filtered ? n : V;
        double fl = 0.0;
        for (int i = tid; i < keep; i += WIDE_THREADS) fl += pf(i);
        const double F = block_sum(fl, sm64);
        double* out = p.probs_out + (int64_t)b * p.probs_stride;
        for (int j = tid; j < p.V; j += WIDE_THREADS) out[j] = 0.0;
        __syncthreads();
        for (int i = tid; i < keep; i += WIDE_THREADS) out[wkey_id(sk[i])] = pf(i) / F;
        return;
    }
    n = rank_cap(p, V, n, pf, sm64, smi);
    uint64_t kt = 0;  // decode: the received token's key
    if (DECODE) {
        const int32_t tok = p.in_token[b];
        const char* rowc = (const char*)p.logits + (int64_t)b * p.ld * (int64_t)sizeof(T);
        if (tok >= 0 && tok < p.V) kt = wkey(Elem<T>::load1(rowc, tok), (uint32_t)tok);
    }
    rank_emit<DECODE>(p, b, st, n, S, [&](int i) -> int32_t { return (int32_t)wkey_id(sk[i]); },
                      [&](int i, int32_t) -> bool { return kt != 0 && sk[i] == kt; }, smi);
}

// ---- numpy's float64 sum over f(0..n-1), restated exactly (or_np_sum): 8192-element chunks added left to right,
// each by numpy's pairwise_sum (leaves of <= 128 elements: 8 interleaved accumulators, < 8: a plain loop; larger
// ranges split at n/2 rounded down to a multiple of 8).  Leaves are summed in parallel, thread 0 walks the tree.
constexpr int NP_CHUNK = 8192;
constexpr int NP_MAX_LEAVES = 2048;  // 131072 entries: 16 chunks x 64 leaves

template <class F>
__device__ double np_leaf(int a, int len, F&& f) {
    if (len < 8) {
        double res = 0.0;
        for (int i = 0; i < len; ++i) res += f(a + i);
        return res;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = f(a + j);
    int i = 8;
    for (; i < len - (len % 8); i += 8)
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] += f(a + i + j);
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < len; ++i) res += f(a + i);
    return res;
}

template <class F>
__device__ double block_np_sum(int n, F&& f, double* lsum, int* lstart, int* llen, int* nleaf_sh) {
    const int tid = threadIdx.x;
    if (tid == 0) {  // leaves in depth-first, left-to-right order
        int nl = 0;
        for (int c0 = 0; c0 < n; c0 += NP_CHUNK) {
            int sa[32], sl[32], sp = 0;
            sa[0] = c0;
            sl[0] = min(NP_CHUNK, n - c0);
            sp = 1;
            while (sp > 0) {
                --sp;
                const int a = sa[sp], len = sl[sp];
                if (len <= 128) {
                    lstart[nl] = a;
                    llen[nl] = len;
                    ++nl;
                } else {
                    int n2 = len / 2;
                    n2 -= n2 % 8;
                    sa[sp] = a + n2;  // right half first on the stack: the left half is visited first
                    sl[sp] = len - n2;
                    sa[sp + 1] = a;
                    sl[sp + 1] = n2;
                    sp += 2;
                }
            }
        }
        *nleaf_sh = nl;
    }
    __syncthreads();
    const int nl = *nleaf_sh;
    for (int k = tid; k < nl; k += WIDE_THREADS) lsum[k] = np_leaf(lstart[k], llen[k], f);
    __syncthreads();
    double total = 0.0;
    if (tid == 0) {  // the same tree, combined bottom-up in the recursion's order
        int li = 0;
        for (int c0 = 0; c0 < n; c0 += NP_CHUNK) {
            int lenS[32], stS[32];
            double lS[32];
            int sp = 0;
            lenS[0] = min(NP_CHUNK, n - c0);
            stS[0] = 0;
            double ret = 0.0;
            bool done = false;
            while (!done) {
                const int L = lenS[sp];
                if (L <= 128) {
                    ret = lsum[li++];
                    bool descended = false;
                    while (sp > 0 && !descended) {  // return to the parents
                        --sp;
                        if (stS[sp] == 1) {  // left child done: keep it, descend right
                            lS[sp] = ret;
                            stS[sp] = 2;
                            int n2 = lenS[sp] / 2;
                            n2 -= n2 % 8;
                            lenS[sp + 1] = lenS[sp] - n2;
                            stS[sp + 1] = 0;
                            ++sp;
                            descended = true;
                        } else {
                            ret = lS[sp] + ret;
                        }
                    }
                    if (!descended) done = true;
                } else {
                    stS[sp] = 1;
                    int n2 = L / 2;
                    n2 -= n2 % 8;
                    lenS[sp + 1] = n2;
                    stS[sp + 1] = 0;
                    ++sp;
                }
            }
            total += ret;
        }
        lsum[0] = total;
    }
    __syncthreads();
    total = lsum[0];
    __syncthreads();
    return total;
}

__device__ __forceinline__ uint64_t prob_key(double v) {
    return v > 0.0 ? (uint64_t)__double_as_longlong(v) : 0ull;  // v <= 0 and NaN: never support, ranked last
}

// Generic provider rows (f64): per stream the activity check of the logit path, the entry count, and the keys
// (value bits) with their array positions for the device-wide pair sort.
template <bool DECODE>
__global__ void rank64_prep_kernel(StepParams p, WideStat* ws, unsigned int* count) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.B) return;
    const ns_stream_state st = p.state[b];
    bool active = !(st.flags & NS_ST_DONE);
    if (!DECODE && active && st.bit_pos >= p.nbits[b]) {
        p.state[b].flags = st.flags | NS_ST_DONE;
        active = false;
    }
    if (DECODE && p.active && !p.active[b]) active = false;
    int n = p.rk_count ? p.rk_count[b] : p.V;
    n = min(max(n, 0), p.V);
    WideStat w = {};
    w.active = (active && n > 0) ? 1u : 0u;
    ws[b] = w;
    count[b] = w.active ? (unsigned int)n : 0u;
}

__global__ __launch_bounds__(256) void rank64_collect_kernel(StepParams p, const WideStat* ws, uint64_t* keys,
                                                             uint32_t* vals, const unsigned int* count, int cap) {
    const int b = blockIdx.y;
    if (!ws[b].active) return;
    const int n = (int)count[b];
    const double* row = (const double*)p.logits + (int64_t)b * p.ld;
    for (int j = blockIdx.x * COLLECT_CHUNK + (int)threadIdx.x; j < min(n, (int)(blockIdx.x + 1) * COLLECT_CHUNK);
         j += 256) {
        keys[(int64_t)b * cap + j] = prob_key(row[j]);
        vals[(int64_t)b * cap + j] = (uint32_t)j;
    }
}

// Provider rows: canonical steps P0-P5 of oracle/nsg_oracle.c (or_rank_step64).  keys_sorted / pos_sorted: the
// row's entries in rank order (value bits desc, position asc: the pair sort is stable).
template <bool DECODE>
__global__ __launch_bounds__(WIDE_THREADS) void wide_rank64_kernel(StepParams p, const WideStat* ws,
                                                                   const uint64_t* keys_sorted,
                                                                   const uint32_t* pos_sorted,
                                                                   const unsigned int* count, int cap) {
    __shared__ double ebuf[WIDE_ROUND];  // also the pairwise leaf sums
    __shared__ int lstart[NP_MAX_LEAVES];
    __shared__ int llen[NP_MAX_LEAVES];
    __shared__ double sm64[64];
    __shared__ int smi[16];
    __shared__ int cut_sh, nleaf_sh;
    __shared__ double acc_sh;
    const int b = blockIdx.x;
    if (!ws[b].active) return;
    const int tid = threadIdx.x;
    const ns_stream_state st = p.state[b];
    const uint64_t* sk = keys_sorted + (int64_t)b * cap;
    const uint32_t* sp = pos_sorted + (int64_t)b * cap;
    const int N = (int)count[b];
    const double* row = (const double*)p.logits + (int64_t)b * p.ld;
    auto val = [&](int i) -> double { return __longlong_as_double((long long)sk[i]); };  // key 0 -> 0.0
    auto np_sum = [&](auto&& f) -> double { return block_np_sum(N, f, ebuf, lstart, llen, &nleaf_sh); };

    // P1: crypto policy: p = v / np.sum(v), then (unless isclose(T, 1)) tempered and renormalised
    const bool crypto = p.rk_crypto != 0;
    const double Tq = p.rk_ptemp;
    double tot = 1.0, a0 = 0.0, Q = 1.0;
    if (crypto) {
        tot = np_sum([&](int j) -> double { return row[j]; });
        if (Tq > 0.0) {
            a0 = log(val(0) / tot + 1e-12) / Tq;
            Q = np_sum([&](int j) -> double { return exp(log(row[j] / tot + 1e-12) / Tq - a0); });
        }
    }
    auto pf = [&](int i) -> double {  // rank order
        if (!crypto) return val(i);
        const double q = val(i) / tot;
        return Tq > 0.0 ? exp(log(q + 1e-12) / Tq - a0) / Q : q;
    };
    auto pfpos = [&](int j) -> double {  // array position order (the reference's arrays)
        if (!crypto) return row[j];
        const double q = row[j] / tot;
        return Tq > 0.0 ? exp(log(q + 1e-12) / Tq - a0) / Q : q;
    };
    // P2: support n = #{p > 0} (a prefix of the ranking), quality cut
    int fz = N;
    for (int i = tid; i < N; i += WIDE_THREADS)
        if (i < fz && !(pf(i) > 0.0)) fz = i;
    int n = block_min_int(fz, smi);
    n = rank_quality_cut(p, N, n, pf, ebuf, smi, cut_sh, acc_sh);
    // P3: apply_quality renormalises the kept values by np.sum over the array (zeros elsewhere); the support is
    // what stays > 0 (_rank_tokens' mask)
    const bool filtered = p.rk_top_k > 0 || p.rk_top_p > 0.0 || p.rk_min_prob >= 0.0;
    double F = 1.0, S_trace = crypto ? tot : 0.0;
    if ((crypto || filtered) && n > 0) {
        const uint64_t kth = sk[n - 1];
        const uint32_t pth = sp[n - 1];
        auto kept = [&](int j) -> bool {
            const uint64_t kj = prob_key(row[j]);
            return kj > kth || (kj == kth && (uint32_t)j <= pth);
        };
        F = np_sum([&](int j) -> double { return kept(j) ? pfpos(j) : 0.0; });
        S_trace = F;
        if (!(F > 0.0 && F <= 1.7976931348623157e308)) {  // QualityConfigError in the reference: range error
            n = 0;
        } else {
            int fz2 = n;
            for (int i = tid; i < n; i += WIDE_THREADS)
                if (i < fz2 && !(pf(i) / F > 0.0)) fz2 = i;
            n = block_min_int(fz2, smi);
        }
    }
    // P4: cap over the array's entries (a dict that went through apply_quality keeps only its positive entries)
    if (!crypto) {
        const int U = (p.rk_dict && filtered) ? n : N;
        n = rank_cap(p, U, n, [&](int i) -> double { return filtered ? pf(i) / F : pf(i); }, sm64, smi);
    }
    // P5: selection / emission; the token of rank i is the id of its array position
    auto id_of = [&](int i) -> int32_t {
        const uint32_t j = sp[i];
        return p.rk_idmap ? p.rk_idmap[(int64_t)b * p.rk_idmap_stride + j] : (int32_t)j;
    };
    rank_emit<DECODE>(p, b, st, n, S_trace, id_of, [&](int i, int32_t tok) -> bool { return id_of(i) == tok; },
                      smi);
}

}  // namespace nsg

// ------------------------------------------------------------------------------------------ host
int nsg_wide_alloc(ns_ctx* ctx) {
    NsgWide& w = ctx->wide;
    if (w.keys_in) return NS_OK;
    if (ctx->vocab > 0x1FFFF) return NS_ERR_UNSUPPORTED;
    w.cap = ctx->vocab;
    const size_t n = (size_t)ctx->max_batch * (size_t)w.cap;
    if (hipMalloc((void**)&w.keys_in, n * 8) != hipSuccess || hipMalloc((void**)&w.keys_out, n * 8) != hipSuccess ||
        hipMalloc((void**)&w.count, ctx->max_batch * sizeof(unsigned int)) != hipSuccess ||
        hipMalloc((void**)&w.begin, ctx->max_batch * sizeof(unsigned int)) != hipSuccess ||
        hipMalloc((void**)&w.end, ctx->max_batch * sizeof(unsigned int)) != hipSuccess ||
        hipMalloc((void**)&w.todo, 2 * (ctx->max_batch + 1) * sizeof(unsigned int)) != hipSuccess ||
        hipMalloc((void**)&w.stat, ctx->max_batch * sizeof(nsg::WideStat)) != hipSuccess)
        return NS_ERR_HIP;
    size_t bytes = 0;
    if (rocprim::segmented_radix_sort_keys_desc(nullptr, bytes, w.keys_in, w.keys_out, (unsigned int)n,
                                                (unsigned int)ctx->max_batch, w.begin, w.end, 0, 49) != hipSuccess)
        return NS_ERR_HIP;
    if (ctx->dtype == NS_DTYPE_F64) {  // provider rows: 64-bit value keys sorted with their array positions
        if (hipMalloc((void**)&w.vals_in, n * 4) != hipSuccess || hipMalloc((void**)&w.vals_out, n * 4) != hipSuccess)
            return NS_ERR_HIP;
        size_t pbytes = 0;
        if (rocprim::segmented_radix_sort_pairs_desc(nullptr, pbytes, w.keys_in, w.keys_out, w.vals_in, w.vals_out,
                                                     (unsigned int)n, (unsigned int)ctx->max_batch, w.begin, w.end,
                                                     0, 64) != hipSuccess)
            return NS_ERR_HIP;
        bytes = bytes > pbytes ? bytes : pbytes;
    }
    w.sort_tmp_bytes = bytes;
    if (hipMalloc(&w.sort_tmp, bytes ? bytes : 16) != hipSuccess) return NS_ERR_HIP;
    return NS_OK;
}

void nsg_wide_free(ns_ctx* ctx) {
    NsgWide& w = ctx->wide;
    for (void* ptr : {(void*)w.keys_in, (void*)w.keys_out, (void*)w.count, (void*)w.begin, (void*)w.end,
                      (void*)w.todo, (void*)w.stat, w.sort_tmp, (void*)w.vals_in, (void*)w.vals_out})
        if (ptr) (void)hipFree(ptr);
    w = NsgWide();
}

#ifndef NSG_WIDE_V2
#define NSG_WIDE_V2 0  // 1: stream + tail kernels (round-4 experiment, measured slower: DESIGN.md §4 wide path)
#endif
template <typename T, bool DECODE>
static bool wide_launch_t(ns_ctx* ctx, const nsg::StepParams& p, hipStream_t s) {
    NsgWide& w = ctx->wide;
    const int B = p.B;
    static const int v2 = [] {
        const char* e = getenv("NSG_WIDE_V2");
        return e ? atoi(e) : NSG_WIDE_V2;
    }();
    if (v2 && !p.sample && !p.stats) {
        // v2 = 1: stream kernel (wave per stream, 8 KiB buffers) + tail kernel; v2 = 2: wave per stream with the
        // tail in the same wave (32 KiB buffers), the tail kernel only for the streams whose buffer overflowed.
        // Only the streams the tails hand on are sorted and listed.
        unsigned int* todo2 = w.todo + ctx->max_batch + 1;
        if (v2 == 2) {
            if (hipMemsetAsync(w.todo, 0, sizeof(unsigned int), s) != hipSuccess) return false;
            hipLaunchKernelGGL((nsg::wide_wave_kernel<T, DECODE>), dim3(B), dim3(nsg::WAVE), 0, s, p, w.stat,
                               w.keys_in, w.keys_out, w.count, w.cap, w.todo, todo2);
        } else {
            hipLaunchKernelGGL((nsg::wide_stream_kernel<T, DECODE>), dim3((B + nsg::WS_WAVES - 1) / nsg::WS_WAVES),
                               dim3(nsg::WS_WAVES * nsg::WAVE), 0, s, p, w.stat, w.keys_in, w.count, w.cap, w.todo,
                               todo2);
        }
        hipLaunchKernelGGL((nsg::wide_wtail_kernel<T, DECODE>), dim3(B), dim3(nsg::WT_THREADS), 0, s, p, w.stat,
                           w.keys_in, w.keys_out, w.count, w.cap, w.todo);
        hipLaunchKernelGGL((nsg::wide_wlist_kernel<T, DECODE>), dim3(B < 512 ? B : 512), dim3(nsg::FAST_THREADS), 0, s,
                           p, w.stat, w.keys_in, w.keys_out, w.count, w.cap, w.todo, todo2);
        hipLaunchKernelGGL(nsg::wide_offsets_kernel, dim3((B + 255) / 256), dim3(256), 0, s, B, w.cap, w.stat,
                           w.count, w.begin, w.end, 0xFFFFFFFFu, nullptr);
        size_t bytes = w.sort_tmp_bytes;
        if (rocprim::segmented_radix_sort_keys_desc(w.sort_tmp, bytes, w.keys_out, w.keys_in,
                                                    (unsigned int)((size_t)B * w.cap), (unsigned int)B, w.begin,
                                                    w.end, 0, 49, s) != hipSuccess)
            return false;
        hipLaunchKernelGGL((nsg::wide_cdf_kernel<T, DECODE>), dim3(B < 256 ? B : 256), dim3(nsg::WIDE_THREADS), 0, s,
                           p, w.stat, w.keys_in, w.count, w.cap, todo2);
        return hipGetLastError() == hipSuccess;
    }
    if (hipMemsetAsync(w.todo, 0, sizeof(unsigned int), s) != hipSuccess) return false;
#if NSG_WIDE_ONEPASS
    hipLaunchKernelGGL((nsg::wide_onepass_kernel<T, DECODE>), dim3(B), dim3(nsg::FAST_THREADS), 0, s, p, w.stat,
                       w.keys_in, w.keys_out, w.count, w.cap, w.todo);
#if NSG_WIDE_SPLIT
    hipLaunchKernelGGL((nsg::wide_tail_kernel<T, DECODE>), dim3(B), dim3(nsg::FAST_THREADS), 0, s, p, w.stat,
                       w.keys_in, w.keys_out, w.count, w.cap, w.todo);
#endif
#else
    hipLaunchKernelGGL((nsg::wide_scan_kernel<T, DECODE>), dim3(B), dim3(nsg::FAST_THREADS), 0, s, p, w.stat,
                       w.keys_in, w.keys_out, w.count, w.cap, w.todo);
#endif
    hipLaunchKernelGGL(nsg::wide_offsets_kernel, dim3((B + 255) / 256), dim3(256), 0, s, B, w.cap, w.stat,
                       w.count, w.begin, w.end, (unsigned int)nsg::FAST_NL, nullptr);
    size_t bytes = w.sort_tmp_bytes;
    if (rocprim::segmented_radix_sort_keys_desc(w.sort_tmp, bytes, w.keys_in, w.keys_out,
                                                (unsigned int)((size_t)B * w.cap), (unsigned int)B, w.begin,
                                                w.end, 0, 49, s) != hipSuccess)
        return false;
    hipLaunchKernelGGL((nsg::wide_cdf_kernel<T, DECODE>), dim3(B < 256 ? B : 256), dim3(nsg::WIDE_THREADS), 0, s, p,
                       w.stat, w.keys_out, w.count, w.cap, w.todo);
    return hipGetLastError() == hipSuccess;
}

template <typename T, bool DECODE>
static bool rank_launch_t(ns_ctx* ctx, const nsg::StepParams& p, hipStream_t s) {
    NsgWide& w = ctx->wide;
    const int B = p.B;
    hipLaunchKernelGGL((nsg::wide_stats_kernel<T, DECODE>), dim3((B + nsg::WPB - 1) / nsg::WPB),
                       dim3(nsg::WPB * nsg::WAVE), 0, s, p, w.stat, w.count);
    const int nchunk = (p.V + nsg::COLLECT_CHUNK - 1) / nsg::COLLECT_CHUNK;
    hipLaunchKernelGGL((nsg::wide_collect_kernel<T>), dim3(nchunk, B), dim3(256), 0, s, p, w.stat, w.keys_in,
                       w.count, w.cap);
    hipLaunchKernelGGL(nsg::wide_offsets_kernel, dim3((B + 255) / 256), dim3(256), 0, s, B, w.cap, w.stat,
                       w.count, w.begin, w.end, 0u, nullptr);
    size_t bytes = w.sort_tmp_bytes;
    if (rocprim::segmented_radix_sort_keys_desc(w.sort_tmp, bytes, w.keys_in, w.keys_out,
                                                (unsigned int)((size_t)B * w.cap), (unsigned int)B, w.begin,
                                                w.end, 0, 49, s) != hipSuccess)
        return false;
    hipLaunchKernelGGL((nsg::wide_rank_kernel<T, DECODE>), dim3(B), dim3(nsg::WIDE_THREADS), 0, s, p, w.stat,
                       w.keys_out, w.count, w.cap);
    return hipGetLastError() == hipSuccess;
}

template <bool DECODE>
static bool rank64_launch_t(ns_ctx* ctx, const nsg::StepParams& p, hipStream_t s) {
    NsgWide& w = ctx->wide;
    const int B = p.B;
    hipLaunchKernelGGL(nsg::rank64_prep_kernel<DECODE>, dim3((B + 255) / 256), dim3(256), 0, s, p, w.stat, w.count);
    const int nchunk = (p.V + nsg::COLLECT_CHUNK - 1) / nsg::COLLECT_CHUNK;
    hipLaunchKernelGGL(nsg::rank64_collect_kernel, dim3(nchunk, B), dim3(256), 0, s, p, w.stat, w.keys_in, w.vals_in,
                       w.count, w.cap);
    hipLaunchKernelGGL(nsg::wide_offsets_kernel, dim3((B + 255) / 256), dim3(256), 0, s, B, w.cap, w.stat,
                       w.count, w.begin, w.end, 0u, nullptr);
    size_t bytes = w.sort_tmp_bytes;
    if (rocprim::segmented_radix_sort_pairs_desc(w.sort_tmp, bytes, w.keys_in, w.keys_out, w.vals_in, w.vals_out,
                                                 (unsigned int)((size_t)B * w.cap), (unsigned int)B, w.begin, w.end,
                                                 0, 64, s) != hipSuccess)
        return false;
    hipLaunchKernelGGL((nsg::wide_rank64_kernel<DECODE>), dim3(B), dim3(nsg::WIDE_THREADS), 0, s, p, w.stat,
                       w.keys_out, w.vals_out, w.count, w.cap);
    return hipGetLastError() == hipSuccess;
}

bool nsg_rank_launch(ns_ctx* ctx, const nsg::StepParams& p, bool decode, hipStream_t s) {
    if (ctx->dtype == NS_DTYPE_F64) return decode ? rank64_launch_t<true>(ctx, p, s) : rank64_launch_t<false>(ctx, p, s);
    if (ctx->dtype == NS_DTYPE_F16)
        return decode ? rank_launch_t<_Float16, true>(ctx, p, s) : rank_launch_t<_Float16, false>(ctx, p, s);
    return decode ? rank_launch_t<float, true>(ctx, p, s) : rank_launch_t<float, false>(ctx, p, s);
}

bool nsg_wide_launch(ns_ctx* ctx, const nsg::StepParams& p, bool decode, hipStream_t s) {
    if (ctx->dtype == NS_DTYPE_F16)
        return decode ? wide_launch_t<_Float16, true>(ctx, p, s) : wide_launch_t<_Float16, false>(ctx, p, s);
    return decode ? wide_launch_t<float, true>(ctx, p, s) : wide_launch_t<float, false>(ctx, p, s);
}

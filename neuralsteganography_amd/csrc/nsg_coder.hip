// nsg_coder.hip -- batched arithmetic-coding step for MI355X (gfx950 / CDNA4), C ABI in include/nsg_coder.h.
//
// One wavefront (64 lanes) owns one message stream per step.  The [B, ld] logit matrix is streamed from
// HBM once, 16 bytes per lane per load (global_load_dwordx4), several tiles in flight per wave.  While
// streaming, every wave keeps
//   * a float64 estimate of the softmax denominator (hardware v_exp_f32 on a fixed per-row reference,
//     fp32 partials flushed into a float64 accumulator per tile) with a rigorous error bound, and
//   * a candidate buffer in LDS of (value desc, id asc) keys above a running threshold; when it fills it
//     is compacted to the exact top-K by a ballot/popcount bisection (no sort).
// After the row, the top-K candidates are ranked (one LDS broadcast read per key), and the whole CDF
// step (canonical float64 exp, 1/R cutoff, rint, int64 prefix sum, overfill trim, interval update,
// bit consume / emit) runs across the wave's lanes with DPP/bpermute shuffles.
//
// Exactness contract: results are bit-identical to oracle/nsg_oracle.c (the canonical restatement of
// code_base/arithmetic.py).  Everything that feeds the emitted integers is computed in the canonical
// float64 order; the fast denominator is used only where its error bound proves the 1/R cutoff decision
// (arithmetic.py:140-142) cannot differ from the exact one -- otherwise the wave re-reads its row and
// computes the exact canonical sum (NS_ST_EXACT_SUM).
//
// Build (see __graft_entry__.build): hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>

#include "../../include/nsg_coder.h"

#pragma clang fp contract(off)

#include "nsg_common.h"
#include "nsg_host.h"
#include "nsg_host.h"

#ifndef NSG_SAMPLE
#define NSG_SAMPLE 64  // sample size / 64 ids: whole tiles spread over the row (16 fp32 / 8 fp16 tiles)
#endif
#ifndef NSG_FMA_ARG
#define NSG_FMA_ARG 1  // fast-sum exponent as one fma (x*c - r*c) with packed / two-chain fp32 sums
#endif
#ifndef NSG_ASM_APPEND
#define NSG_ASM_APPEND 0
#endif
#ifndef NSG_F16_NATIVE
#define NSG_F16_NATIVE 0  // 1: fp16 groups kept packed (fma_mix exponents, packed 16-bit integer pass tests, set-bit
                          // appends; round 5), 0: converted to fp32 first (A/B)
#endif
#ifndef NSG_SETBIT_APPEND
#define NSG_SETBIT_APPEND 2  // per-lane pass masks + a set-bit loop per tile: 0 never, 1 always, 2 fp16 rows only
#endif
#ifndef NSG_SLOT_APPEND
#define NSG_SLOT_APPEND 0  // per-slot ballot appends (offer_slots; A/B, round 5: f16 equal, f32 +2 %): 0 off, 1 all, 2 fp16
#endif
#ifndef NSG_DIAG_NOWRITE
#define NSG_DIAG_NOWRITE 0
#endif
#ifndef NSG_BUCKET_CAP
#define NSG_BUCKET_CAP 48  // largest bucket the bucket rank accepts (its fix-up loop runs that often)
#endif

namespace nsg {

typedef float f32x2 __attribute__((ext_vector_type(2)));

// Per-wave LDS scratch: 256+4 bucket counters/bases (u32), 64 gathered keys (u64), and a slow-path counter.
constexpr int SCR_U32 = 392;
constexpr int SCR_GATHER = 260;  // u32 offset of the gather area (8-byte aligned)
constexpr int SCR_SLOW = 391;    // selections that fell back to bisection / full counting (counters[3])

__device__ __forceinline__ void note_slow(uint32_t* scr, int lane) {
    if (lane == 0) scr[SCR_SLOW] += 1u;
}

// Keep exactly the top-K keys of keys[0..cnt) (cnt >= K).  Bisection on the value word, then on the id
// word among ties; counts by ballot+popcount.  Returns the K-th key.  (Fallback of compact_topk.)
__device__ __noinline__ uint64_t compact_bisect(uint64_t* keys, int cnt, int K, int lane) {
    constexpr int NSL = CAND / WAVE;
    uint64_t kr[NSL];
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
        const int i = s * WAVE + lane;
        kr[s] = (i < cnt) ? keys[i] : 0ull;  // real keys are > 0
    }
    const int nsl = (cnt + WAVE - 1) / WAVE;
    uint32_t v = 0;
    for (int bit = 31; bit >= 0; --bit) {
        const uint32_t cand = v | (1u << bit);
        int c = 0;
#pragma unroll
        for (int s = 0; s < NSL; ++s)
            if (s < nsl) c += popc64(ballot((uint32_t)(kr[s] >> 32) >= cand));
        if (c >= K) v = cand;
    }
    int c_gt = 0, c_eq = 0;
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
        if (s < nsl) {
            const uint32_t h = (uint32_t)(kr[s] >> 32);
            c_gt += popc64(ballot(h > v));
            c_eq += popc64(ballot(h == v));
        }
    }
    const int need = K - c_gt;
    uint32_t wlo = 0;
    if (c_eq > need) {
        for (int bit = 31; bit >= 0; --bit) {
            const uint32_t cand = wlo | (1u << bit);
            int c = 0;
#pragma unroll
            for (int s = 0; s < NSL; ++s)
                if (s < nsl) c += popc64(ballot((uint32_t)(kr[s] >> 32) == v && (uint32_t)kr[s] >= cand));
            if (c >= need) wlo = cand;
        }
    }
    const uint64_t kappa = ((uint64_t)v << 32) | wlo;
    lds_fence();
    int base = 0;
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
        if (s < nsl) {
            const bool keep = kr[s] >= kappa && kr[s] != 0ull;
            const uint64_t m = ballot(keep);
            if (keep) keys[base + lanes_below(m)] = kr[s];
            base += popc64(m);
        }
    }
    lds_fence();
    return kappa;
}

// Keep exactly the top-K keys of keys[0..cnt) (cnt >= K); returns the K-th key.  Histogram select: the
// value words are bucketed by a digit monotone in the value (256 linear buckets over [min, max], largest
// first, LDS ds_add), a scan finds the bucket holding the K-th key, only that bucket's keys are ranked
// exactly, and everything at or above the K-th key is kept.  Keys are re-read from LDS in every pass (few
// live registers: this is called from inside the streaming loop).  Falls back to bisection when every key
// has the same value word or the boundary bucket holds more than 64 keys.
__device__ __noinline__ uint64_t compact_topk(uint64_t* keys, uint32_t* scr, int cnt, int K, int lane) {
    constexpr int NB = 256;
    const int nsl = (cnt + WAVE - 1) / WAVE;
    uint32_t hmin = 0xFFFFFFFFu, hmax = 0u;
#pragma unroll 4
    for (int s = 0; s < nsl; ++s) {
        const int i = s * WAVE + lane;
        if (i < cnt) {
            const uint32_t h = (uint32_t)(keys[i] >> 32);
            hmin = min(hmin, h);
            hmax = max(hmax, h);
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        hmin = min(hmin, (uint32_t)__shfl_xor((int)hmin, off));
        hmax = max(hmax, (uint32_t)__shfl_xor((int)hmax, off));
    }
    hmin = __builtin_amdgcn_readfirstlane(hmin);
    hmax = __builtin_amdgcn_readfirstlane(hmax);
    if (hmax == hmin) {
        note_slow(scr, lane);
        return compact_bisect(keys, cnt, K, lane);
    }
    const float scale = __uint_as_float(
        __builtin_amdgcn_readfirstlane(__float_as_uint(255.99f / (float)(hmax - hmin))));  // wave-uniform
    // bucket of a key, largest values first (digit monotone in the value word; two roundings keep it < 256)
    auto bucket = [&](uint64_t k) -> uint32_t {
        return (uint32_t)(NB - 1) -
               min((uint32_t)((float)((uint32_t)(k >> 32) - hmin) * scale), (uint32_t)(NB - 1));
    };
    reinterpret_cast<uint4*>(scr)[lane] = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll 4
    for (int s = 0; s < nsl; ++s) {
        const int i = s * WAVE + lane;
        if (i < cnt) atomicAdd(&scr[bucket(keys[i])], 1u);
    }
    lds_fence();
    const uint4 c4 = reinterpret_cast<const uint4*>(scr)[lane];
    const uint32_t i1 = c4.x, i2 = i1 + c4.y, i3 = i2 + c4.z, i4 = i3 + c4.w;
    const uint32_t inc = wave_incl_scan_u32(i4);
    const uint32_t ex = inc - i4;
    // the bucket holding the K-th key: A < K <= A + C (exactly one, since cnt >= K)
    int hit = -1;
    uint32_t a_hit = 0u, c_hit = 0u;
    if (ex < (uint32_t)K && ex + c4.x >= (uint32_t)K) { hit = 0; a_hit = ex; c_hit = c4.x; }
    if (ex + i1 < (uint32_t)K && ex + i2 >= (uint32_t)K) { hit = 1; a_hit = ex + i1; c_hit = c4.y; }
    if (ex + i2 < (uint32_t)K && ex + i3 >= (uint32_t)K) { hit = 2; a_hit = ex + i2; c_hit = c4.z; }
    if (ex + i3 < (uint32_t)K && ex + i4 >= (uint32_t)K) { hit = 3; a_hit = ex + i3; c_hit = c4.w; }
    const int src = (int)__builtin_ctzll(ballot(hit >= 0));
    const uint32_t bstar = __builtin_amdgcn_readlane(4 * lane + hit, src);
    const uint32_t astar = __builtin_amdgcn_readlane(a_hit, src);
    const uint32_t hstar = __builtin_amdgcn_readlane(c_hit, src);
    if (hstar > (uint32_t)WAVE) {
        note_slow(scr, lane);
        return compact_bisect(keys, cnt, K, lane);
    }
    const int need = K - (int)astar;  // 1 <= need <= hstar
    uint64_t* g = reinterpret_cast<uint64_t*>(scr + SCR_GATHER);
    int gb = 0;
#pragma unroll 4
    for (int s = 0; s < nsl; ++s) {
        const int i = s * WAVE + lane;
        const uint64_t k = i < cnt ? keys[i] : 0ull;
        const bool in = k != 0ull && bucket(k) == bstar;
        const uint64_t m = ballot(in);
        if (in) g[gb + lanes_below(m)] = k;
        gb += popc64(m);
    }
    lds_fence();
    const uint64_t mine = lane < (int)hstar ? g[lane] : 0ull;
    int r = 0;
    for (uint32_t t = 0; t < hstar; ++t) r += g[t] > mine ? 1 : 0;  // LDS broadcast reads
    const uint64_t mk = ballot(lane < (int)hstar && r == need - 1);
    const uint64_t kappa = readlane64(mine, (int)__builtin_ctzll(mk));
    // in-place keep: slot s's keys are read before any write, and writes land below (s+1)*64
    int base = 0;
#pragma unroll 4
    for (int s = 0; s < nsl; ++s) {
        const int i = s * WAVE + lane;
        const uint64_t k = i < cnt ? keys[i] : 0ull;
        const bool keep = k >= kappa && k != 0ull;
        const uint64_t m = ballot(keep);
        if (keep) keys[base + lanes_below(m)] = k;
        base += popc64(m);
    }
    lds_fence();
    return kappa;
}

// buffer-resource row reader: one SRD per wave (uniform), range-checked 16-byte loads (0 beyond the row)
// Candidate buffer of one wave: keys of every element > thr seen so far (a superset of the running top-K).
// Appends store raw entries (value bits << 32 | id: no order transform on the streaming path); entries
// [0, conv) are canonical keys, [conv, cnt) raw, and to_keys() converts the raw tail before any read.
struct Cand {
    uint64_t* keys;
    uint32_t* scr;  // per-wave LDS scratch (SCR_U32)
    int cnt;
    int conv;
    int ncompact;
    float thr;       // element passes iff x > thr
    int nan;         // per lane: a NaN was appended by the packed fp16 test (the step then re-streams exactly)
    uint32_t tbits;  // wave-uniform: bits of the largest half <= thr (-0 taken as +0), for the packed fp16 test
};

__device__ __forceinline__ uint64_t raw_entry(float x, uint32_t j) {
    return ((uint64_t)__float_as_uint(x) << 32) | (uint64_t)j;
}

__device__ __forceinline__ void to_keys(Cand& c, int lane) {
    for (int i = c.conv + lane; i < c.cnt; i += WAVE) {
        const uint64_t r = c.keys[i];
        c.keys[i] = make_key(__uint_as_float((uint32_t)(r >> 32)), (uint32_t)r);
    }
    c.conv = c.cnt;
    lds_fence();
}

// A threshold t with x > t for every x whose value is >= v in key order (-inf stays -inf: never admitted).
// The next float below v, or -FLT_MIN around zero (+0 > -0 is false; denormals may flush).
__device__ __forceinline__ float thr_below(float v) {
    if (!(v > -__builtin_inff())) return v;
    const float t = unord32(ord32(v) - 1u);
    return t < v ? t : -1.17549435e-38f;
}

typedef _Float16 h2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h2v as_h2(uint32_t w) { return __builtin_bit_cast(h2v, w); }
__device__ __forceinline__ _Float16 half_below(float t) {  // the largest half <= t (t not NaN)
    _Float16 h = (_Float16)t;
    if ((float)h > t) {
        uint16_t u = __builtin_bit_cast(uint16_t, h);
        if (u == 0x0000u) u = 0x8001u;         // +0 -> -smallest denormal
        else if (u & 0x8000u) u = (uint16_t)(u + 1u);  // negative: one ulp further from zero
        else u = (uint16_t)(u - 1u);           // positive (incl. +inf -> max finite): one ulp toward zero
        h = __builtin_bit_cast(_Float16, u);
    }
    return h;
}
// c.thr and the packed fp16 test's threshold bits together (x > thr <=> x > the largest half <= thr, for halves;
// x > -0 <=> x > +0)
__device__ __forceinline__ void set_thr(Cand& c, float t) {
    c.thr = t;
    const uint32_t tb = (uint32_t)__builtin_bit_cast(uint16_t, half_below(t));
    c.tbits = __builtin_amdgcn_readfirstlane(tb == 0x8000u ? 0u : tb);
}
template <int W>
__device__ __forceinline__ void offer(Cand& c, const float (&x)[W], int j0, int K, int lane) {
    float mx = x[0];
#pragma unroll
    for (int q = 1; q < W; ++q) mx = fmaxf(mx, x[q]);
    if (!ballot(mx > c.thr)) return;
    uint64_t msk[W];
    int npt = 0;
#pragma unroll
    for (int q = 0; q < W; ++q) {
        msk[q] = ballot(x[q] > c.thr);
        npt += popc64(msk[q]);
    }
    if (c.cnt + npt > CAND) {  // cnt > CAND - TS >= K: keep the exact running top-K
        to_keys(c, lane);
        const uint64_t kappa = compact_topk(c.keys, c.scr, c.cnt, K, lane);
        ++c.ncompact;
        c.cnt = c.conv = K;
        // admit ties at the K-th value: the sample tiles are offered before the stream, so a later element can
        // carry a smaller id than the K-th key (a superset is always safe; the final selection is exact)
        set_thr(c, thr_below(key_val(kappa)));
        npt = 0;
#pragma unroll
        for (int q = 0; q < W; ++q) {
            msk[q] = ballot(x[q] > c.thr);
            npt += popc64(msk[q]);
        }
    }
    int base = c.cnt;
#pragma unroll
    for (int q = 0; q < W; ++q) {
        if (x[q] > c.thr) c.keys[base + lanes_below(msk[q])] = raw_entry(x[q], (uint32_t)(j0 + q));
        base += popc64(msk[q]);
    }
    c.cnt = base;
}

// exclusive prefix and total over the wave of a per-lane count n (0 <= n < 64): one ballot per bit plane
__device__ __forceinline__ void wave_excl_prefix(int n, int& excl, int& total) {
    excl = 0;
    total = 0;
#pragma unroll
    for (int bit = 0; bit < 6; ++bit) {
        const uint64_t m = ballot(((n >> bit) & 1) != 0);
        excl += lanes_below(m) << bit;
        total += popc64(m) << bit;
    }
}

// Per-slot appends of one tile (round 5): one v_cmp per value slot gives the slot's wave mask in SGPRs; the
// capacity check and the running base are scalar; only the slots that some lane passes (a scalar branch) compute
// a position (two mbcnt) and write, under exec = the slot's mask.  Every (tile, slot) in a 64-lane wave has a pass
// with probability ~1 - (1 - rate)^64, so a per-lane set-bit loop runs about once per tile whatever the rate; the
// slots cost ~4 VALU each only where they write (profiles/r05: appends were +30 us of the 121 us fp16 launch).
template <int W>
__device__ __forceinline__ void offer_slots(Cand& c, const float (&x)[W], int jl, int K, int lane) {
    uint64_t msk[W];
    int npt = 0;
#pragma unroll
    for (int q = 0; q < W; ++q) {
        msk[q] = ballot(x[q] > c.thr);
        npt += popc64(msk[q]);
    }
    if (npt == 0) return;
    if (c.cnt + npt > CAND) {  // the per-tile path compacts first (recomputing the tests at the raised threshold)
        offer<W>(c, x, jl, K, lane);
        return;
    }
    const uint32_t kb = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint64_t*)c.keys;
    int base = c.cnt;
#pragma unroll
    for (int q = 0; q < W; ++q) {
        if (msk[q] != 0ull) {  // wave-uniform
            const uint32_t pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(msk[q] >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)msk[q], (uint32_t)base));
            const uint64_t e = raw_entry(x[q], (uint32_t)(jl + q));
            uint64_t saved;
            // exec = the slot's passing lanes for the one write (LDS ops of a wave complete in order, so the
            // compiler's own lgkmcnt waits stay valid with this extra write in flight)
            asm volatile(
                "s_and_saveexec_b64 %0, %1\n\t"
                "ds_write_b64 %2, %3\n\t"
                "s_mov_b64 exec, %0"
                : "=&s"(saved)
                : "s"(msk[q]), "v"(kb + 8u * pos), "v"(e)
                : "memory");
            base += popc64(msk[q]);
        }
    }
    c.cnt = base;
}

// Group form of offer(): G tiles (G*W values per lane) share one reject test, one wave prefix and one
// capacity check; passing values are written with predicated stores at lane-private positions.  If the
// group does not fit, the per-tile path (which compacts as needed and always fits) takes over.  Tile d's
// value q of this lane has id tb[d] + lj + q: tb[d] the tile's first id (wave-uniform; the tiles of a group
// need not be adjacent), lj = lane * W.
template <int W, int G>
__device__ __forceinline__ void offer_group(Cand& c, const float (&x)[G][W], const int (&tb)[G], int lj, int K,
                                            int lane) {
    if constexpr (NSG_SLOT_APPEND == 1 || (NSG_SLOT_APPEND == 2 && W == 8)) {
#pragma unroll
        for (int d = 0; d < G; ++d) offer_slots<W>(c, x[d], tb[d] + lj, K, lane);
        return;
    }
    // set-bit appends: measured 1.6-2.2 % faster on fp16 rows, 2 % slower on fp32 rows (profiles/r04/coder_append_ab.jsonl)
    constexpr bool SETBIT = NSG_SETBIT_APPEND == 1 || (NSG_SETBIT_APPEND == 2 && W == 8);
    int n = 0;
    uint32_t pm[G];  // SETBIT, per tile: bit q = value q passes
    if constexpr (SETBIT) {
#pragma unroll
        for (int d = 0; d < G; ++d) {
            pm[d] = 0u;
#pragma unroll
            for (int q = 0; q < W; ++q) pm[d] |= (x[d][q] > c.thr) ? (1u << q) : 0u;
            n += __builtin_popcount(pm[d]);
        }
    } else {
#pragma unroll
        for (int d = 0; d < G; ++d)
#pragma unroll
            for (int q = 0; q < W; ++q) n += (x[d][q] > c.thr) ? 1 : 0;
    }
    int excl, total;
    wave_excl_prefix(n, excl, total);
    if (total == 0) return;
    if (c.cnt + total > CAND) {
#pragma unroll
        for (int d = 0; d < G; ++d) offer<W>(c, x[d], tb[d] + lj, K, lane);
        return;
    }
    int pos = c.cnt + excl;
#if NSG_DIAG_NOWRITE  // timing diagnostic only: count and prefix, no LDS writes, never compacts (wrong results)
    (void)pos;
    c.cnt = min(c.cnt + total, CAND / 2);
    return;
#endif
#if NSG_ASM_APPEND
    // branch-free appends: each slot's write is issued under exec = (lanes whose value passes); an empty mask
    // makes it a no-op.  LDS ops of a wave complete in order, so the compiler's own lgkmcnt waits stay valid.
    const uint32_t kb = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint64_t*)c.keys;
#pragma unroll
    for (int d = 0; d < G; ++d)
#pragma unroll
        for (int q = 0; q < W; ++q) {
            const bool pass = x[d][q] > c.thr;
            const uint64_t m = ballot(pass);
            const uint64_t e = raw_entry(x[d][q], (uint32_t)(tb[d] + lj + q));
            uint64_t saved;
            asm volatile(
                "s_and_saveexec_b64 %0, %1\n\t"
                "ds_write_b64 %2, %3\n\t"
                "s_mov_b64 exec, %0"
                : "=&s"(saved)
                : "s"(m), "v"(kb + 8u * (uint32_t)pos), "v"(e)
                : "memory");
            pos += pass ? 1 : 0;
        }
#else
    if constexpr (SETBIT) {
    // per tile, a wave-uniform loop over the lanes' set pass bits (as many rounds as the most passes any lane has
    // in the tile: usually one) instead of one predicated write per value slot; the value comes from the tile's W
    // registers through a select tree on the bit index
#pragma unroll
    for (int d = 0; d < G; ++d) {
        uint32_t m = pm[d];
        while (ballot(m != 0u)) {
            if (m) {
                const uint32_t q = (uint32_t)__builtin_ctz(m);
                m &= m - 1u;
                float sv[W];
#pragma unroll
                for (int i = 0; i < W; ++i) sv[i] = x[d][i];
#pragma unroll
                for (int k = 0; (1 << k) < W; ++k)
#pragma unroll
                    for (int i = 0; i < (W >> (k + 1)); ++i) sv[i] = ((q >> k) & 1u) ? sv[2 * i + 1] : sv[2 * i];
                c.keys[pos] = raw_entry(sv[0], (uint32_t)(tb[d] + lj) + q);
                ++pos;
            }
        }
    }
    } else {
#pragma unroll
    for (int d = 0; d < G; ++d)
#pragma unroll
        for (int q = 0; q < W; ++q)
            if (x[d][q] > c.thr) {
                c.keys[pos] = raw_entry(x[d][q], (uint32_t)(tb[d] + lj + q));
                ++pos;
            }
    }
#endif
    c.cnt += total;
}

// ---- fp16 rows kept packed (NSG_F16_NATIVE): the fast-sum exponent from the halves (the conversion folds into
// v_fma_mix), the candidate test as an fp16 compare against the largest half <= thr (x > thr <=> x > that half
// for every half x), and the passing values picked by a set-bit loop and converted one by one -- instead of
// converting all 32 values of a group to fp32 first.
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t sub_sat16x2(uint32_t a, uint32_t b) {  // v_pk_sub_i16 ... clamp
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(__builtin_bit_cast(s16x2, a),
                                                                      __builtin_bit_cast(s16x2, b)));
}
// Pass bits of one fp16 tile (8 halves of a lane, q = 2 * word + half) against t16 = the largest half <= thr, two
// halves per instruction, as 16-bit integers.  For t16 >= +0: x > t16 <=> int16(x) > int16(t16) (negative halves are
// negative integers, never above).  For t16 < 0: x > t16 <=> uint16(x) < uint16(t16) (x <= t means x negative with
// bits >= t's) <=> int16(x ^ 0x7FFF) > int16(t16 ^ 0x7FFF) (flip the sign bit to compare as int16, then complement
// to turn < into >).  So with XM = 0 or 0x7FFF per half: pass <=> sat(TT - (x ^ XM)) < 0, TT = t16 ^ XM -- the sign
// of one clamped v_pk_sub_i16 per two halves; v_perm gathers the eight sign bytes: bits 7, 15, 23, 31 are q = 0..3,
// bits 6, 14, 22, 30 are q = 4..7.  Exact for every half but positive NaNs, which pass here and are caught when
// appended (Cand::nan).
__device__ __forceinline__ uint32_t pass_bits_h(const uint4& v, uint32_t XM2, uint32_t TT2) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t sg[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) sg[i] = sub_sat16x2(TT2, w[i] ^ XM2);
    const uint32_t D = __builtin_amdgcn_perm(sg[1], sg[0], 0x07050301u);
    const uint32_t E = __builtin_amdgcn_perm(sg[3], sg[2], 0x07050301u);
    return (D & 0x80808080u) | ((E >> 1) & 0x40404040u);
}
template <int G>
__device__ __forceinline__ void offer_group_h(Cand& c, const uint4 (&raw)[G], const int (&tb)[G], int lj, int K,
                                              int lane) {
    const uint32_t XM2 = (c.tbits & 0x8000u) ? 0x7FFF7FFFu : 0u;  // wave-uniform (set_thr)
    const uint32_t TT2 = (c.tbits * 0x10001u) ^ XM2;
    uint32_t pm[G];
    int n = 0;
#pragma unroll
    for (int d = 0; d < G; ++d) {
        pm[d] = pass_bits_h(raw[d], XM2, TT2);
        n += __builtin_popcount(pm[d]);
    }
    int excl, total;
    wave_excl_prefix(n, excl, total);
    if (total == 0) return;
    if (c.cnt + total > CAND) {  // the per-tile path (compacts as needed) on fp32 values (NaN never passes there)
#pragma unroll
        for (int d = 0; d < G; ++d) {
            float x[8];
            Elem<_Float16>::unpack(raw[d], x);
            offer<8>(c, x, tb[d] + lj, K, lane);
        }
        return;
    }
    int pos = c.cnt + excl;
#pragma unroll
    for (int d = 0; d < G; ++d) {
        uint32_t m = pm[d];
        while (ballot(m != 0u)) {
            if (m) {
                const uint32_t bp = (uint32_t)__builtin_ctz(m);
                m &= m - 1u;
                const uint32_t q = (bp >> 3) + ((bp & 1u) ? 0u : 4u);
                const uint32_t wsel = (q & 4u) ? ((q & 2u) ? raw[d].w : raw[d].z) : ((q & 2u) ? raw[d].y : raw[d].x);
                const float v = Elem<_Float16>::h2f((q & 1u) ? (wsel >> 16) : (wsel & 0xFFFFu));
                c.nan |= (v != v) ? 1 : 0;
                c.keys[pos] = raw_entry(v, (uint32_t)(tb[d] + lj) + q);
                ++pos;
            }
        }
    }
    c.cnt += total;
}

// Rank the K unique keys held in sk[] (key i = s*64 + lane) and store keys[rank] = key (rank 0 = largest).
// Bucket pass: a digit monotone in the value word (256 linear buckets over [min, max] of the value words,
// largest first) and ds_add_rtn on LDS counters give every key a bucket and a slot in it; an exclusive scan
// turns counts into bucket bases; keys are scattered bucket-ordered and each key's rank is its bucket base
// plus the number of larger keys in its own bucket.  Returns false, having written nothing into keys[0..K),
// when the largest bucket holds more than `cap` keys (a skewed row): the caller ranks by full counting.
template <int NSK>
__device__ __forceinline__ bool bucket_rank(uint64_t* keys, uint32_t* base, const uint64_t (&sk)[NSK], int nsk, int K,
                                            int lane, int cap) {
    constexpr int NB = 256;
    uint32_t hmin = 0xFFFFFFFFu, hmax = 0u;
#pragma unroll
    for (int s = 0; s < NSK; ++s) {
        if (s < nsk && s * WAVE + lane < K) {
            const uint32_t h = (uint32_t)(sk[s] >> 32);
            hmin = min(hmin, h);
            hmax = max(hmax, h);
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        hmin = min(hmin, (uint32_t)__shfl_xor((int)hmin, off));
        hmax = max(hmax, (uint32_t)__shfl_xor((int)hmax, off));
    }
    // (float)(h - hmin) * scale is monotone in h and stays below 256 (two roundings of 255.99)
    const float scale = hmax > hmin ? 255.99f / (float)(hmax - hmin) : 0.0f;
    reinterpret_cast<uint4*>(base)[lane] = make_uint4(0u, 0u, 0u, 0u);
    if (lane == 0) base[NB] = 0u;
    lds_fence();
    uint32_t bk[NSK], slot[NSK];
#pragma unroll
    for (int s = 0; s < NSK; ++s) {
        bk[s] = 0u;
        slot[s] = 0u;
        if (s < nsk && s * WAVE + lane < K) {
            const uint32_t d = min((uint32_t)((float)((uint32_t)(sk[s] >> 32) - hmin) * scale), (uint32_t)(NB - 1));
            bk[s] = (uint32_t)(NB - 1) - d;
            slot[s] = atomicAdd(&base[bk[s]], 1u);
        }
    }
    lds_fence();
    const uint4 c4 = reinterpret_cast<const uint4*>(base)[lane];
    const uint32_t i1 = c4.x, i2 = i1 + c4.y, i3 = i2 + c4.z, i4 = i3 + c4.w;
    const uint32_t inc = wave_incl_scan_u32(i4);
    const uint32_t ex = inc - i4;
    reinterpret_cast<uint4*>(base)[lane] = make_uint4(ex, ex + i1, ex + i2, ex + i3);
    if (lane == 0) base[NB] = (uint32_t)K;
    lds_fence();
    uint32_t b0[NSK], b1[NSK];
    uint32_t biggest = 0u;
#pragma unroll
    for (int s = 0; s < NSK; ++s) {
        b0[s] = b1[s] = 0u;
        if (s < nsk && s * WAVE + lane < K) {
            b0[s] = base[bk[s]];
            b1[s] = base[bk[s] + 1];
            biggest = max(biggest, b1[s] - b0[s]);
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) biggest = max(biggest, (uint32_t)__shfl_xor((int)biggest, off));
    if (biggest > (uint32_t)cap) {
        note_slow(base, lane);
        return false;
    }
#pragma unroll
    for (int s = 0; s < NSK; ++s)
        if (b1[s] > b0[s]) keys[b0[s] + slot[s]] = sk[s];
    lds_fence();
    uint32_t rk[NSK];
#pragma unroll
    for (int s = 0; s < NSK; ++s) rk[s] = b0[s];
    for (uint32_t t = 0; t < biggest; ++t) {
#pragma unroll
        for (int s = 0; s < NSK; ++s) {
            const uint32_t idx = b0[s] + t;
            if (idx < b1[s]) rk[s] += keys[idx] > sk[s] ? 1u : 0u;
        }
    }
    lds_fence();
#pragma unroll
    for (int s = 0; s < NSK; ++s)
        if (b1[s] > b0[s]) keys[rk[s]] = sk[s];
    lds_fence();
    return true;
}

// -inf for ids >= V (last tile only) and for banned ids (sorted; `bi`/`next_ban` advance monotonically)
template <int W>
__device__ __forceinline__ void mask_tile(const StepParams& p, float (&x)[W], int tile, int ntiles, int j0,
                                          int& bi, int& next_ban) {
    constexpr int TS = WAVE * W;
    if (tile == ntiles - 1) {
#pragma unroll
        for (int q = 0; q < W; ++q)
            if (j0 + q >= p.V) x[q] = -__builtin_inff();
    }
    const int tile_end = (tile + 1) * TS;
    while (next_ban < tile_end) {  // wave-uniform, at most nbanned times per row
#pragma unroll
        for (int q = 0; q < W; ++q)
            if (j0 + q == next_ban) x[q] = -__builtin_inff();
        ++bi;
        next_ban = bi < p.nbanned ? p.banned[bi] : 0x7FFFFFFF;
    }
}

// Sampler tail (code_base/sample.py:28-46; canonical steps S2-S5 of oracle/nsg_oracle.c): the ranked top-K
// keys sk[] and their e_i are given.  Support k_s = leading ranks with e_i >= 2^-60; E canonical over it;
// integer CDF at 2^48; counter-based draw; the interval state is not touched.
template <int NSK>
__device__ __forceinline__ void sample_tail(const StepParams& p, int b, const ns_stream_state& st,
                                            const uint64_t (&sk)[NSK], const double (&e)[NSK], int nsk, int K,
                                            double m, const RowStats& rs, int lane, bool stats) {
    int ks = K;
#pragma unroll
    for (int s = 0; s < NSK; ++s) {
        if (s < nsk) {
            const int i = s * WAVE + lane;
            const uint64_t mb = ballot(i < K && e[s] < SAMPLE_SUPPORT);
            if (mb && ks == K) ks = s * WAVE + __builtin_ctzll(mb);
        }
    }
    double el = 0.0;
#pragma unroll
    for (int s = 0; s < NSK; ++s)
        if (s < nsk && s * WAVE + lane < ks) el += e[s];
    const double E = wave_sum_butterfly(el);
    int64_t cum[NSK];
    int64_t carry = 0;
#pragma unroll
    for (int s = 0; s < NSK; ++s) {
        const int i = s * WAVE + lane;
        const int64_t q = (s < nsk && i < ks) ? (int64_t)__builtin_rint((e[s] / E) * SAMPLE_SCALE) : 0;
        const int64_t c = (s < nsk) ? wave_incl_scan(q, lane) + carry : carry;
        cum[s] = c;
        if (s < nsk) carry = (int64_t)readlane64((uint64_t)c, WAVE - 1);
    }
    const uint64_t total = (uint64_t)carry;
    const uint64_t u = rand64(p.seed, p.stream_offset + b, st.ntokens);
    const uint64_t idx = __umul64hi(u, total);
    int sel = -1;
#pragma unroll
    for (int s = 0; s < NSK; ++s) {
        if (s < nsk) {
            const int i = s * WAVE + lane;
            const uint64_t ms = ballot(i < ks && (uint64_t)cum[s] > idx);
            if (ms && sel < 0) sel = s * WAVE + __builtin_ctzll(ms);
        }
    }
    uint64_t tk = 0;
#pragma unroll
    for (int s = 0; s < NSK; ++s)
        if (s == sel / WAVE) tk = readlane64(sk[s], sel % WAVE);
    const int32_t token = (int32_t)key_id(tk);
    double kl = 0.0, h = 0.0;
    if (stats) {
        const double logE = log(E);
#pragma unroll
        for (int s = 0; s < NSK; ++s) {
            if (s < nsk && s * WAVE + lane < ks) {
                const double xi = (double)key_val(sk[s]) - m;
                const double lq = xi * p.inv_temp - logE;
                const double q = e[s] / E;
                kl += q * (lq - (xi - rs.lse1));
                h += q * lq;
            }
        }
        kl = wave_sum_butterfly(kl);
        h = wave_sum_butterfly(h);
    }
    if (lane == 0) {
        ns_stream_state ns = st;
        ns.ntokens = st.ntokens + 1;
        p.state[b] = ns;
        p.out_token[b] = token;
        if (p.hist && st.ntokens < p.hist_stride) p.hist[(int64_t)b * p.hist_stride + st.ntokens] = token;
        if (p.trace) {
            ns_step_trace tr;
            tr.k = K;
            tr.kprime = ks;
            tr.sel = sel;
            tr.n = 0;
            tr.token = token;
            tr.exact = 0;
            tr.S = E;
            p.trace[b] = tr;
        }
        if (stats) {
            double* a = p.stats + 4 * (int64_t)b;
            a[0] += ((double)key_val(tk) - m) - rs.lse1;
            a[1] += kl / 0.69315;
            a[2] += -h / 0.69315;
            a[3] += 1.0;
        }
    }
}

// NSPLIT = 1: one wave per stream, WPB streams per workgroup.  NSPLIT > 1 (small batches, round 2): one workgroup
// of NSPLIT = NSAMP waves per stream; wave w streams the w-th slice of the row (its sample tile is the slice's
// last tile), the waves agree on r and the threshold through LDS, and wave 0 merges the candidate buffers and
// fast-sum partials and runs the tail alone.  The emitted integers are the same either way (the top-K keys are
// exact and the cutoff decision is proven; tested bit-exact against the oracle in both forms).
template <typename T, bool DECODE, int NSK, bool STATS, int NSPLIT = 1>
__global__ __launch_bounds__((NSPLIT > 1 ? NSPLIT : WPB) * WAVE, NSG_MIN_WAVES_PER_EU) void coder_step_kernel(StepParams p) {
    constexpr int W = Elem<T>::W;
    constexpr int TS = WAVE * W;  // elements per tile (one 16-byte load per lane)
    static_assert(NSK * WAVE <= CAND - TS, "K must leave room for one tile of appends");
    constexpr int NWG = NSPLIT > 1 ? NSPLIT : WPB;  // waves per workgroup
    __shared__ uint64_t s_keys[NWG][CAND];
    __shared__ __attribute__((aligned(16))) uint32_t s_scr[NWG][SCR_U32];
    __shared__ double s_part[NSPLIT > 1 ? NSPLIT : 1][3];  // split: per-wave fast-sum partials
    __shared__ int s_cnt[NSPLIT > 1 ? NSPLIT : 1][4];      // split: cnt, conv, ncompact, NaN appended

    const int lane = threadIdx.x & (WAVE - 1);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
    const int b = __builtin_amdgcn_readfirstlane(NSPLIT > 1 ? (int)blockIdx.x : (int)blockIdx.x * WPB + wv);
    if (b >= p.B) return;

    NSG_STAMP_RT(p, b, lane, 9);
    NSG_STAMP(p, b, lane, 0);
    ns_stream_state st = p.state[b];
    if (st.flags & NS_ST_DONE) return;
    int64_t nbits = 0;
    if (!DECODE && !p.sample) {
        nbits = p.nbits[b];
        if (st.bit_pos >= nbits) {  // payload consumed: done, or sentence finishing (finish_sent_kernel)
            if (lane == 0 && !(p.flags & NS_STEP_FINISH_SENT)) p.state[b].flags = st.flags | NS_ST_DONE;
            return;
        }
    } else {
        if (p.active && !p.active[b]) return;
    }

    const int V = p.V;
    const int K = p.K;
    const char* rowc = (const char*)p.logits + (int64_t)b * p.ld * (int64_t)sizeof(T);
    const RowReader rd(rowc, (uint32_t)(p.ld * (int64_t)sizeof(T)));
    const int ntiles = (V + TS - 1) / TS;
    const float c32 = p.c32;

    Cand cand;
    cand.keys = s_keys[wv];
    cand.scr = s_scr[wv];
    if (lane == 0) cand.scr[SCR_SLOW] = 0u;
    cand.cnt = 0;
    cand.conv = 0;
    cand.ncompact = 0;
    set_thr(cand, -__builtin_inff());
    cand.nan = 0;
    int nfallback = 0;

    // ---------------- stream order ----------------
    // With a sample (p.spec_j > 0) NSAMP whole tiles spread over the row -- tile s*space + space-1, 4,096 ids --
    // are read first and give r and the speculative threshold.  The last NKEEP of them stay in registers and
    // are accumulated and offered like any other tile; the stream visits every other tile in increasing order,
    // the first NSAMP - NKEEP sample tiles included (fp32 rows: keeping all 16 would spill; those 8 KiB are read
    // again, with the default cache policy on their first read).  The host enables the sample only when
    // ntiles >= 2*NSAMP (space >= 2).
    constexpr int NSAMP = (64 * NSG_SAMPLE) / TS;
    constexpr int NKEEP = NSAMP < 8 ? NSAMP : 8;
    constexpr int S0 = NSAMP - NKEEP;  // first kept sample tile
    static_assert(NKEEP >= PREFETCH && NKEEP % PREFETCH == 0, "kept sample tiles come in ring-sized groups");
    static_assert(NSPLIT == 1 || NSPLIT == NSAMP, "split: one wave per sample tile");
    const bool spec_on = p.spec_j > 0;  // always on in the split form (host)
    const int space = spec_on ? ntiles / NSAMP : 1;
    // split: wave w streams tiles [w*space, end) minus its sample tile w*space + space-1; the last wave takes the rest
    const int nstream = !spec_on ? ntiles
                        : NSPLIT > 1 ? (wv == NSPLIT - 1 ? ntiles : (wv + 1) * space) - wv * space - 1
                                     : ntiles - NKEEP;
    // load cursor (wave-uniform): next tile to load, non-skipped tiles left before the next kept sample tile
    int lt = NSPLIT > 1 ? wv * space : 0;
    int lc = !spec_on ? 0x7FFFFFFF : NSPLIT > 1 ? space - 1 : S0 * space + space - 1;
    int sleft = !spec_on ? 0 : NSPLIT > 1 ? 1 : NKEEP;
    auto next_tile = [&]() -> int {
        const int t = lt++;
        if (--lc == 0) {  // reaches 0 only while kept sample tiles remain: skip one
            ++lt;
            lc = --sleft > 0 ? space - 1 : 0x7FFFFFFF;
        }
        return t;
    };
    // the streaming ring: without a sample its first tiles go out now; with one, once the first sample group has
    // been consumed (the registers it frees hold the ring)
    uint4 buf[PREFETCH];
    int tid[PREFETCH];
    auto issue_ring = [&]() {
#pragma unroll
        for (int d = 0; d < PREFETCH; ++d) {
            tid[d] = next_tile();
            buf[d] = rd.vec(tid[d] * WAVE + lane);
        }
    };
    if (!spec_on) issue_ring();

    // ---------------- prologue: sample tiles -> softmax reference r and speculative threshold -----
    // r = sample max (fast-sum reference); thr = a lower bound of the spec_j-th largest sample value (16-bit
    // prefix), a GUESS verified at the end of the row.  The count runs over each lane's three largest sample
    // values only (4,096 values, ~J/64 per lane above the answer): it can only undercount, which lowers the
    // threshold -- more appends, never a wrong result.
    float r = 0.0f;
    bool spec = false;
    uint4 smp[NKEEP];  // the kept sample tiles as loaded (fp16 stays packed)
    if constexpr (NSPLIT > 1) {
        // wave w reads sample tile w (its slice's last tile), then its ring; per-lane top 3 of the tile goes
        // through LDS, and every wave derives the same r and threshold from the union (the same values as the
        // one-wave form: the top 3 of the per-tile top 3s are the top 3 of all 4,096 values of the lane)
        const int ts = wv * space + space - 1;
        smp[0] = rd.vec(ts * WAVE + lane);
        issue_ring();
        float x[W];
        Elem<T>::unpack(smp[0], x);
        int sbi = 0, snb = p.nbanned > 0 ? p.banned[0] : 0x7FFFFFFF;
        mask_tile<W>(p, x, ts, ntiles, ts * TS + lane * W, sbi, snb);
        uint32_t u0 = 0u, u1 = 0u, u2 = 0u;  // ord32 order; 0 is below every float
        auto top3 = [&](uint32_t v) {
            const uint32_t a = min(u0, v);
            u0 = max(u0, v);
            const uint32_t c = min(u1, a);
            u1 = max(u1, a);
            u2 = max(u2, c);
        };
#pragma unroll
        for (int q = 0; q < W; ++q) top3(ord32(x[q]));
        s_scr[wv][lane] = u0;
        s_scr[wv][WAVE + lane] = u1;
        s_scr[wv][2 * WAVE + lane] = u2;
        __syncthreads();
        u0 = u1 = u2 = 0u;
#pragma unroll
        for (int v = 0; v < NSPLIT; ++v) {
            top3(s_scr[v][lane]);
            top3(s_scr[v][WAVE + lane]);
            top3(s_scr[v][2 * WAVE + lane]);
        }
        __syncthreads();  // every wave has read the exchange area before any scratch is reused
        r = wave_max(unord32(u0));
        if (r == -__builtin_inff()) r = 0.0f;
        uint32_t pre = 0;
        for (int bit = 31; bit >= 16; --bit) {
            const uint32_t c = pre | (1u << bit);
            const int n = popc64(ballot(u0 >= c)) + popc64(ballot(u1 >= c)) + popc64(ballot(u2 >= c));
            if (n >= p.spec_j) pre = c;
        }
        if (pre > 0x00800000u) {
            set_thr(cand, unord32(pre - 1u));
            spec = true;
        }
    } else if (spec_on) {
        uint4 sx[S0 > 0 ? S0 : 1];
#pragma unroll
        for (int s = 0; s < NSAMP; ++s) {
            const int v = (s * space + space - 1) * WAVE + lane;
            if (s < S0) sx[min(s, S0 > 0 ? S0 - 1 : 0)] = rd.vec_keep(v); else smp[max(s - S0, 0)] = rd.vec(v);
        }
        int sbi = 0, snb = p.nbanned > 0 ? p.banned[0] : 0x7FFFFFFF;
        float t0 = -__builtin_inff(), t1 = -__builtin_inff(), t2 = -__builtin_inff();
#pragma unroll
        for (int s = 0; s < NSAMP; ++s) {
            const int ts = s * space + space - 1;
            float x[W];
            Elem<T>::unpack(s < S0 ? sx[min(s, S0 > 0 ? S0 - 1 : 0)] : smp[max(s - S0, 0)], x);
            mask_tile<W>(p, x, ts, ntiles, ts * TS + lane * W, sbi, snb);
#pragma unroll
            for (int q = 0; q < W; ++q) {  // per-lane top 3
                const float v = x[q];
                const float a = fminf(t0, v);
                t0 = fmaxf(t0, v);
                const float c = fminf(t1, a);
                t1 = fmaxf(t1, a);
                t2 = fmaxf(t2, c);
            }
        }
        r = wave_max(t0);
        if (r == -__builtin_inff()) r = 0.0f;
        const uint32_t o0 = ord32(t0), o1 = ord32(t1), o2 = ord32(t2);
        uint32_t pre = 0;
        for (int bit = 31; bit >= 16; --bit) {
            const uint32_t c = pre | (1u << bit);
            const int n = popc64(ballot(o0 >= c)) + popc64(ballot(o1 >= c)) + popc64(ballot(o2 >= c));
            if (n >= p.spec_j) pre = c;
        }
        if (pre > 0x00800000u) {  // above ord(-inf): a finite threshold
            set_thr(cand, unord32(pre - 1u));  // x > thr  <=>  ord(x) >= pre
            spec = true;
        }
    }
    if (p.flags & NS_STEP_DIAG_NO_CANDIDATES) set_thr(cand, __builtin_inff());

    NSG_STAMP(p, b, lane, 1);
    // ---------------- streaming pass (the HBM-bound part) ----------------
    double acc64 = 0.0;
    double b64 = 0.0, u64 = 0.0;  // STATS: sum e (x-r), sum exp(x-r) untempered
    int bi = 0;
    int next_ban = p.nbanned > 0 ? p.banned[0] : 0x7FFFFFFF;
    if (p.spec_j <= 0) {  // no sample (small vocab): reference = max of the first tile
        float x[W];
        Elem<T>::unpack(buf[0], x);
        int bi0 = 0, nb0 = next_ban;
        mask_tile<W>(p, x, 0, ntiles, lane * W, bi0, nb0);
        float mx = x[0];
#pragma unroll
        for (int q = 1; q < W; ++q) mx = fmaxf(mx, x[q]);
        r = wave_max(mx);
        if (r == -__builtin_inff()) r = 0.0f;
    }
    // fp32 partial sums of one group, flushed into float64 (STATS adds sum e*(x-r) and the untempered sum;
    // masked ids are -inf: dx is clamped so e*dx is 0, not NaN)
    // Plain builds take the exponent as ONE fma, x*c32 - fl(r*c32) (fp16 rows: v_fma_mix, the conversion
    // included; fp32 rows: packed pairs), and sum in two fp32 chains; the bound below adds u*|r*c32|.
    const float nrc = -(r * c32);
    auto accumulate = [&](const float* xs, int n) {
        float a = 0.0f, bb = 0.0f, uu = 0.0f;
        if (STATS) {
#pragma unroll
            for (int i = 0; i < n; ++i) {
                const float dx = fmaxf(xs[i] - r, -3.0e38f);
                const float e = __builtin_amdgcn_exp2f(dx * c32);
                a += e;
                bb += e * dx;
                uu += __builtin_amdgcn_exp2f(dx * L2E_F);
            }
        } else if (NSG_FMA_ARG && W == 4) {
            f32x2 a2 = {0.0f, 0.0f};
            const f32x2 c2 = {c32, c32}, n2 = {nrc, nrc};
#pragma unroll
            for (int i = 0; i < n; i += 2) {
                const f32x2 x2 = {xs[i], xs[i + 1]};
                const f32x2 t = __builtin_elementwise_fma(x2, c2, n2);
                const f32x2 e2 = {__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
                a2 += e2;
            }
            a = a2.x + a2.y;
        } else if (NSG_FMA_ARG) {
            float a1 = 0.0f;
#pragma unroll
            for (int i = 0; i < n; i += 2) {
                a += __builtin_amdgcn_exp2f(__builtin_fmaf(xs[i], c32, nrc));
                a1 += __builtin_amdgcn_exp2f(__builtin_fmaf(xs[i + 1], c32, nrc));
            }
            a += a1;
        } else {
#pragma unroll
            for (int i = 0; i < n; ++i) a += __builtin_amdgcn_exp2f((xs[i] - r) * c32);
        }
        acc64 += (double)a;
        if (STATS) {
            b64 += (double)bb;
            u64 += (double)uu;
        }
    };
    auto process = [&](float (&x)[W], int tile) {
        const int j0 = (tile * WAVE + lane) * W;
        mask_tile<W>(p, x, tile, ntiles, j0, bi, next_ban);
        accumulate(x, W);
        offer<W>(cand, x, j0, K, lane);
    };
    // The kept sample tiles first (still in registers), in ring-sized groups; then the ring goes out.
    if constexpr (NSPLIT > 1) {
        const int ts = wv * space + space - 1;
        float x[W];
        Elem<T>::unpack(smp[0], x);
        int sbi = 0, snb = p.nbanned > 0 ? p.banned[0] : 0x7FFFFFFF;
        mask_tile<W>(p, x, ts, ntiles, ts * TS + lane * W, sbi, snb);
        accumulate(x, W);
        offer<W>(cand, x, ts * TS + lane * W, K, lane);
    } else if (spec_on) {
        int sbi = 0, snb = p.nbanned > 0 ? p.banned[0] : 0x7FFFFFFF;
#pragma unroll
        for (int g = 0; g < NKEEP; g += PREFETCH) {
            float xg[PREFETCH][W];
            int tb[PREFETCH];
#pragma unroll
            for (int d = 0; d < PREFETCH; ++d) {
                const int ts = (S0 + g + d) * space + space - 1;
                tb[d] = ts * TS;
                Elem<T>::unpack(smp[g + d], xg[d]);
                mask_tile<W>(p, xg[d], ts, ntiles, tb[d] + lane * W, sbi, snb);
            }
            accumulate(&xg[0][0], PREFETCH * W);
            offer_group<W, PREFETCH>(cand, xg, tb, lane * W, K, lane);
        }
        issue_ring();
    }
    // Full groups: every slot is consumed, then refilled PREFETCH stream positions ahead into the same
    // registers (no copies, so the per-tile wait is a counted vmcnt, never a drain).  Loads past the row are
    // range-checked by the buffer descriptor and return zeros.
    int pos = 0;
    for (; pos + PREFETCH <= nstream; pos += PREFETCH) {
        if constexpr (NSG_F16_NATIVE && sizeof(T) == 2 && !STATS) {
            uint4 raw[PREFETCH];
            int jt[PREFETCH], tb[PREFETCH];
#pragma unroll
            for (int d = 0; d < PREFETCH; ++d) {
                raw[d] = buf[d];
                jt[d] = tid[d];
                tb[d] = jt[d] * TS;
                tid[d] = next_tile();
                buf[d] = rd.vec(tid[d] * WAVE + lane);
            }
            if (!(jt[PREFETCH - 1] == ntiles - 1 || next_ban < (jt[PREFETCH - 1] + 1) * TS)) {
                // the usual group: no masked id, values stay packed (v_fma_mix exponents, two fp32 chains in
                // v_pk_add_f32: 16 terms each, within the (PREFETCH * W + 1) u bound of the tail)
                f32x2 a2 = {0.0f, 0.0f};
#pragma unroll
                for (int d = 0; d < PREFETCH; ++d) {
                    const uint32_t wd[4] = {raw[d].x, raw[d].y, raw[d].z, raw[d].w};
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        const h2v h = as_h2(wd[w]);
                        const f32x2 e2 = {__builtin_amdgcn_exp2f(__builtin_fmaf((float)h.x, c32, nrc)),
                                          __builtin_amdgcn_exp2f(__builtin_fmaf((float)h.y, c32, nrc))};
                        a2 += e2;
                    }
                }
                acc64 += (double)(a2.x + a2.y);
                offer_group_h<PREFETCH>(cand, raw, tb, lane * W, K, lane);
                continue;
            }
            float xg[PREFETCH][W];
#pragma unroll
            for (int d = 0; d < PREFETCH; ++d) {
                Elem<T>::unpack(raw[d], xg[d]);
                mask_tile<W>(p, xg[d], jt[d], ntiles, tb[d] + lane * W, bi, next_ban);
            }
            accumulate(&xg[0][0], PREFETCH * W);
            offer_group<W, PREFETCH>(cand, xg, tb, lane * W, K, lane);
            continue;
        }
        float xg[PREFETCH][W];
        int jt[PREFETCH], tb[PREFETCH];
#pragma unroll
        for (int d = 0; d < PREFETCH; ++d) {
            Elem<T>::unpack(buf[d], xg[d]);
            jt[d] = tid[d];
            tb[d] = jt[d] * TS;
            tid[d] = next_tile();
            buf[d] = rd.vec(tid[d] * WAVE + lane);
        }
        if (jt[PREFETCH - 1] == ntiles - 1 || next_ban < (jt[PREFETCH - 1] + 1) * TS) {  // rare: tail or banned id
#pragma unroll
            for (int d = 0; d < PREFETCH; ++d) mask_tile<W>(p, xg[d], jt[d], ntiles, tb[d] + lane * W, bi, next_ban);
        }
        accumulate(&xg[0][0], PREFETCH * W);
        offer_group<W, PREFETCH>(cand, xg, tb, lane * W, K, lane);
    }
#pragma unroll
    for (int d = 0; d < PREFETCH; ++d) {
        if (pos + d < nstream) {
            float x[W];
            Elem<T>::unpack(buf[d], x);
            process(x, tid[d]);
        }
    }
    NSG_STAMP(p, b, lane, 2);
#if NSG_CODER_TAIL_PRIO
    __builtin_amdgcn_s_setprio(NSG_CODER_TAIL_PRIO);  // the tail is a latency-bound chain: issue priority
#endif
    if constexpr (NSPLIT > 1) {
        // hand the slice results to wave 0: fast-sum partials (reduced per wave, added in wave order) and the
        // candidate buffers (copied into wave 0's, converted to keys; compacted to the top-K when full)
        const double sa = wave_sum_butterfly(acc64);
        const double sb = STATS ? wave_sum_butterfly(b64) : 0.0;
        const double su = STATS ? wave_sum_butterfly(u64) : 0.0;
        if (lane == 0) {
            s_part[wv][0] = sa;
            s_part[wv][1] = sb;
            s_part[wv][2] = su;
            s_cnt[wv][0] = cand.cnt;
            s_cnt[wv][1] = cand.conv;
            s_cnt[wv][2] = cand.ncompact;
        }
        const bool wave_nan = ballot(cand.nan != 0) != 0ull;
        if (lane == 0) s_cnt[wv][3] = wave_nan ? 1 : 0;
        __syncthreads();
        if (wv != 0) return;
        double ta = 0.0, tb = 0.0, tu = 0.0;
        for (int v = 0; v < NSPLIT; ++v) {
            ta += s_part[v][0];
            tb += s_part[v][1];
            tu += s_part[v][2];
        }
        acc64 = lane == 0 ? ta : 0.0;
        b64 = lane == 0 ? tb : 0.0;
        u64 = lane == 0 ? tu : 0.0;
        to_keys(cand, lane);
        for (int v = 1; v < NSPLIT; ++v) {
            const int n = s_cnt[v][0], cv = s_cnt[v][1];
            cand.ncompact += s_cnt[v][2];
            cand.nan |= s_cnt[v][3];
            const uint64_t* src = s_keys[v];
            for (int i0 = 0; i0 < n; i0 += WAVE) {
                if (cand.cnt + WAVE > CAND) {  // cnt > CAND - 64 >= K
                    compact_topk(cand.keys, cand.scr, cand.cnt, K, lane);
                    ++cand.ncompact;
                    cand.cnt = cand.conv = K;
                }
                const int i = i0 + lane;
                if (i < n) {
                    const uint64_t e = src[i];
                    cand.keys[cand.cnt + lane] = i < cv ? e : make_key(__uint_as_float((uint32_t)(e >> 32)), (uint32_t)e);
                }
                cand.cnt += min(WAVE, n - i0);
                cand.conv = cand.cnt;
                lds_fence();
            }
        }
    }
    // speculation check: the buffer holds the true top-K iff at least K elements passed the guess
    // (or a compaction happened, which needs > CAND - TS >= K passes).  Else re-stream, exactly.
    // (a positive NaN appended by the packed fp16 test also re-streams: the fp32 test below never admits NaN)
    const bool nan_cand = ballot(cand.nan != 0) != 0ull;
    if ((spec && cand.ncompact == 0 && cand.cnt < K && !(p.flags & NS_STEP_DIAG_NO_CANDIDATES)) || nan_cand) {
        ++nfallback;
        cand.cnt = 0;
        cand.conv = 0;
        cand.nan = 0;
        set_thr(cand, -__builtin_inff());
        int bj = 0, nbj = p.nbanned > 0 ? p.banned[0] : 0x7FFFFFFF;
        for (int tile = 0; tile < ntiles; ++tile) {
            float x[W];
            Elem<T>::unpack(rd.vec(tile * WAVE + lane), x);
            const int j0 = (tile * WAVE + lane) * W;
            mask_tile<W>(p, x, tile, ntiles, j0, bj, nbj);
            offer<W>(cand, x, j0, K, lane);
        }
    }
    lds_fence();
    if (p.flags & (NS_STEP_DIAG_STREAM_ONLY | NS_STEP_DIAG_NO_CANDIDATES)) {  // diagnostic timing only
        const double s_r = wave_sum_butterfly(acc64);
        if (lane == 0 && p.trace) p.trace[b].S = s_r + (double)cand.cnt + (double)cand.ncompact;
        return;
    }

    // ---------------- exact top-K, ranked ----------------
    uint64_t* keys = cand.keys;
    NSG_STAMP(p, b, lane, 3);
    to_keys(cand, lane);
    NSG_STAMP(p, b, lane, 4);
    if (cand.cnt > K) compact_topk(keys, cand.scr, cand.cnt, K, lane);
    // fewer than K candidates after the exact re-stream: only NaN and -inf logits are never offered (x > thr
    // fails for them even at thr = -inf).  A -inf logit is a valid rank with probability 0 in the reference's
    // softmax (masked ids: the decode's -1e10 on fp16 logits, a caller's -inf mask), so the missing ranks are the
    // lowest valid -inf ids, appended here in id order; a row with a NaN logit reports a range error.
    // Rare path: one more pass over the row by this wave.
    bool short_row = cand.cnt < K;
    if (short_row) {
        bool nan_row = false;
        int have = cand.cnt;
        for (int tile = 0; tile < ntiles; ++tile) {
            float x[W];
            Elem<T>::unpack(rd.vec(tile * WAVE + lane), x);
            const int j0 = (tile * WAVE + lane) * W;
            bool ninf[W];
            uint32_t cl = 0u;
#pragma unroll
            for (int q = 0; q < W; ++q) {
                const bool ok = j0 + q < V && !is_banned(p, j0 + q);
                nan_row = nan_row || (ok && x[q] != x[q]);
                ninf[q] = ok && x[q] == -__builtin_inff();
                cl += ninf[q] ? 1u : 0u;
            }
            const uint32_t incl = wave_incl_scan_u32(cl);
            uint32_t at = (uint32_t)have + incl - cl;  // id order: lane-major, then q (ids j0 .. j0+W-1)
#pragma unroll
            for (int q = 0; q < W; ++q) {
                if (ninf[q]) {
                    if (at < (uint32_t)K) keys[at] = make_key(-__builtin_inff(), (uint32_t)(j0 + q));
                    ++at;
                }
            }
            have += (int)__builtin_amdgcn_readlane((int)incl, WAVE - 1);
        }
        nan_row = ballot(nan_row) != 0ull;
        if (have > K) have = K;
        for (int i = have + lane; i < K; i += WAVE) keys[i] = 0ull;  // no stale LDS past the valid ranks
        lds_fence();
        cand.cnt = have;
        short_row = nan_row || have < K;
    }
    NSG_STAMP(p, b, lane, 5);
    const int nsk = (K + WAVE - 1) / WAVE;
    const int K8 = (K + 7) & ~7;
    if (lane < K8 - K) keys[K + lane] = 0ull;  // zero pad: never counted as greater
    lds_fence();
    uint64_t sk[NSK];
    int rk[NSK];
#pragma unroll
    for (int s = 0; s < NSK; ++s) {
        const int i = s * WAVE + lane;
        sk[s] = (s < nsk && i < K) ? keys[i] : 0ull;
        rk[s] = 0;
    }
    if (!bucket_rank<NSK>(keys, cand.scr, sk, nsk, K, lane, NSG_BUCKET_CAP)) {
        for (int t = 0; t < K8; t += 8) {  // skewed row: rank by counting (one LDS broadcast per key)
            uint64_t o[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) o[u] = keys[t + u];
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
                for (int s = 0; s < NSK; ++s) rk[s] += (o[u] > sk[s]) ? 1 : 0;
        }
        lds_fence();
#pragma unroll
        for (int s = 0; s < NSK; ++s) {
            const int i = s * WAVE + lane;
            if (s < nsk && i < K) keys[rk[s]] = sk[s];
        }
        lds_fence();
    }
#pragma unroll
    for (int s = 0; s < NSK; ++s) {
        const int i = s * WAVE + lane;
        sk[s] = (s < nsk && i < K) ? keys[i] : 0ull;
    }

    if (p.flags & NS_STEP_DIAG_SKIP_CDF) {
        if (lane == 0 && p.trace) p.trace[b].S = (double)key_val(keys[0]) + (double)cand.ncompact;
        return;
    }

    NSG_STAMP(p, b, lane, 6);
    // ---------------- CDF step (canonical float64) ----------------
    const double m = (double)key_val(readlane64(sk[0], 0));
    double e[NSK];
#pragma unroll
    for (int s = 0; s < NSK; ++s) {
        const int i = s * WAVE + lane;
        e[s] = (s < nsk && i < K) ? exp_canon(((double)key_val(sk[s]) - m) * p.inv_temp) : 0.0;
    }
    const double S_r = wave_sum_butterfly(acc64);
    // row statistics (STATS builds; tolerance-checked, not part of the bit contract)
    RowStats rs{0.0, 0.0, 0.0};
    const bool want_stats = STATS && p.stats != nullptr;
    if (want_stats) {
        const double B_r = wave_sum_butterfly(b64);
        const double U_r = wave_sum_butterfly(u64);
        if (!row_stats_from_stream(S_r, B_r, U_r, r, m, p.inv_temp, rs)) rs = wave_row_stats<T>(p, rowc, m, lane);
    }
    if (!DECODE && p.sample) {
        sample_tail<NSK>(p, b, st, sk, e, nsk, K, m, rs, lane, want_stats);
        return;
    }
    const uint64_t R = st.hi - st.lo;
    const double Rd = (double)R;
    const double thr = 1.0 / Rd;

    // fast denominator with a rigorous interval
    const double t_m = (m - (double)r) * (double)c32;
    bool exact = (p.flags & NS_STEP_FORCE_EXACT_SUM) != 0u;
    exact = exact || !(S_r > 0.0 && S_r < 1.0e300) || !(t_m <= 100.0 && t_m >= -60.0);
    double S_used = 0.0;
    int k0 = K;
    if (!exact) {
        const double f = exp_canon(((double)r - m) * p.inv_temp);
        const double Sf = S_r * f;
        const double u24 = 5.9604644775390625e-08;  // 2^-24
        const double eb = 9.5367431640625e-07         // v_exp_f32 error (2^-20, generous)
                          + 3.0 * u24 * 0.6931471805599453 *                     // argument rounding
                                (60.0 + fabs(t_m) + (STATS || !NSG_FMA_ARG ? 0.0 : fabs((double)nrc)))
                          + (double)(PREFETCH * W + 1) * u24                        // fp32 partials
                          + 1.0e-13;
        const double B2 = 2.0 * eb + 1.0e-12;
        // reciprocals with an extra 1e-15 margin stand in for the per-element divisions
        const double inv_lo = 1.0 / (Sf * (1.0 - B2) * (1.0 - 1.0e-15));
        const double inv_hi = 1.0 / (Sf * (1.0 + B2) * (1.0 + 1.0e-15));
        int first_below = K, first_amb = K;
#pragma unroll
        for (int s = 0; s < NSK; ++s) {
            if (s < nsk) {
                const int i = s * WAVE + lane;
                const bool valid = i < K;
                const bool below = valid && (e[s] * inv_lo < thr);
                const bool above = valid && (e[s] * inv_hi >= thr);
                const uint64_t mb = ballot(below);
                const uint64_t ma = ballot(valid && !below && !above);
                if (mb && first_below == K) first_below = s * WAVE + __builtin_ctzll(mb);
                if (ma && first_amb == K) first_amb = s * WAVE + __builtin_ctzll(ma);
            }
        }
        if (first_amb < first_below) {
            exact = true;
        } else {
            k0 = first_below;
            S_used = Sf;
        }
    }
    if (exact) {
        const double S = exact_row_sum<T>(p, rowc, m, lane);
        S_used = S;
        k0 = K;
#pragma unroll
        for (int s = 0; s < NSK; ++s) {
            if (s < nsk) {
                const int i = s * WAVE + lane;
                const uint64_t mb = ballot(i < K && (e[s] / S < thr));
                if (mb && k0 == K) k0 = s * WAVE + __builtin_ctzll(mb);
            }
        }
    }
    int k = k0 < 2 ? 2 : k0;
    if (k > p.topk) k = p.topk;

    // E = sum_{i<k} e_i, order-free (exact limb sums, canonical step 6)
    Mass ms{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < NSK; ++s) {
        const int i = s * WAVE + lane;
        if (s < nsk && i < k) mass_add(ms, e[s]);
    }
    mass_wave_sum(ms);
    const double E = mass_value(ms);

    // q, inclusive prefix, overfill trim
    int64_t cum[NSK];
    int64_t carry = 0;
    int kp = k;
#pragma unroll
    for (int s = 0; s < NSK; ++s) {
        const int i = s * WAVE + lane;
        int64_t q = 0;
        if (s < nsk && i < k) q = (int64_t)__builtin_rint((e[s] / E) * Rd);
        int64_t c = (s < nsk) ? wave_incl_scan(q, lane) + carry : carry;
        cum[s] = c;
        if (s < nsk) {
            carry = (int64_t)readlane64((uint64_t)c, WAVE - 1);
            const uint64_t mo = ballot(i < k && c > (int64_t)R);
            if (mo && kp == k) kp = s * WAVE + __builtin_ctzll(mo);
        }
    }
    auto cum_at = [&](int i) -> int64_t {
        int64_t val = 0;
        const int si = i / WAVE, li = i % WAVE;
#pragma unroll
        for (int s = 0; s < NSK; ++s)
            if (s == si) val = (int64_t)readlane64((uint64_t)cum[s], li);
        return val;
    };
    const int64_t shift = (int64_t)R - cum_at(kp - 1) + (int64_t)st.lo;  // deficit + lo

    // selection
    int sel = -1;
    uint32_t err = 0;
    int32_t token = -1;
    if (!DECODE) {
        const int64_t bp = st.bit_pos + lane;
        uint32_t bit = 0;
        if (lane < p.P && bp < nbits) {
            const uint8_t* pl = p.payload + (int64_t)b * p.payload_stride;
            bit = (pl[bp >> 3] >> (bp & 7)) & 1u;
        }
        const uint64_t mbits = ballot(bit != 0u);
        const uint64_t idx = __builtin_bitreverse64(mbits) >> (64 - p.P);
#pragma unroll
        for (int s = 0; s < NSK; ++s) {
            if (s < nsk) {
                const int i = s * WAVE + lane;
                const uint64_t ms = ballot(i < kp && (uint64_t)(cum[s] + shift) > idx);
                if (ms && sel < 0) sel = s * WAVE + __builtin_ctzll(ms);
            }
        }
        if (sel < 0) err = NS_ST_ERR_RANGE;
    } else {
        const int32_t tok = p.in_token[b];
        if (tok >= 0 && tok < V && !is_banned(p, tok)) {
            const uint64_t kt = make_key(Elem<T>::load1(rowc, tok), (uint32_t)tok);
#pragma unroll
            for (int s = 0; s < NSK; ++s) {
                if (s < nsk) {
                    const int i = s * WAVE + lane;
                    const uint64_t ms = ballot(i < kp && sk[s] == kt);
                    if (ms && sel < 0) sel = s * WAVE + __builtin_ctzll(ms);
                }
            }
        }
        if (sel < 0) {
            err = NS_ST_ERR_DIVERGE;
            if (p.ranked) {  // export the ranked kept ids for the host's BPE repair (arithmetic.py:300-342)
                int32_t* rk_out = p.ranked + (int64_t)b * p.ranked_stride;
#pragma unroll
                for (int s = 0; s < NSK; ++s) {
                    const int i = s * WAVE + lane;
                    if (s < nsk && i < kp && i < p.ranked_stride) rk_out[i] = (int32_t)key_id(sk[s]);
                }
                if (lane == 0 && kp < p.ranked_stride) rk_out[kp] = -1;
            }
        }
    }
    if (short_row || !(E > 0.0 && E <= 1.7976931348623157e308)) {  // NaN / +inf logits (e.g. a poisoned
        sel = -1;  // attention row): the CDF is meaningless, report a range error, emit nothing
        err = NS_ST_ERR_RANGE;
    }

    uint64_t tk = 0;
    if (sel >= 0) {
        const int si = sel / WAVE, li = sel % WAVE;
#pragma unroll
        for (int s = 0; s < NSK; ++s)
            if (s == si) tk = readlane64(sk[s], li);
        token = (int32_t)key_id(tk);
    }

    // statistics of an encode step (code_base/arithmetic.py:193-199): log p(sel) untempered, KL(q || p) over
    // the k' kept entries with q = probs_final / R, entropy of the tempered softmax over V
    if (!DECODE && want_stats && sel >= 0) {
        const int64_t deficit = shift - (int64_t)st.lo;
        double kl = 0.0;
#pragma unroll
        for (int s = 0; s < NSK; ++s) {
            const int i = s * WAVE + lane;
            if (s < nsk && i < kp) {
                int64_t pf = (int64_t)__builtin_rint((e[s] / E) * Rd);
                if (i == 0) pf += deficit;
                const double qd = (double)pf / Rd;
                if (qd > 0.0) kl += qd * (log(qd) - (((double)key_val(sk[s]) - m) - rs.lse1));
            }
        }
        kl = wave_sum_butterfly(kl);
        if (lane == 0) {
            double* a = p.stats + 4 * (int64_t)b;
            a[0] += ((double)key_val(tk) - m) - rs.lse1;
            a[1] += kl / 0.69315;
            a[2] += (rs.lst - rs.a_over_s) / 0.69315;
            a[3] += 1.0;
        }
    }

    NSG_STAMP(p, b, lane, 7);
    // state update: cross-lane values are gathered by shuffles, every lane computes the same scalars
    if (err == 0u) {
        const int P = p.P;
        const uint64_t mask = (P >= 64) ? ~0ull : ((1ull << P) - 1ull);
        const uint64_t new_lo = sel > 0 ? (uint64_t)(cum_at(sel - 1) + shift) : st.lo;
        const uint64_t new_hi = (uint64_t)(cum_at(sel) + shift);
        const uint64_t top = new_hi - 1ull;
        const uint64_t diff = (new_lo ^ top) & mask;
        const int n = diff == 0ull ? P - 1 : P - (64 - __builtin_clzll(diff));
        ns_stream_state ns = st;
        if (DECODE) {
            const bool last = p.is_last[b] != 0;
            const int cntb = last ? P : n;
            const uint64_t src = last ? new_lo : top;
            if (lane == 0) {
                uint8_t* ob = p.out_bits + (int64_t)b * p.out_stride;
                for (int t = 0; t < cntb; ++t) {
                    const int64_t bp = st.bit_pos + t;
                    const uint8_t bitv = (uint8_t)((src >> (P - 1 - t)) & 1u);
                    const uint8_t bm = (uint8_t)(1u << (bp & 7));
                    ob[bp >> 3] = bitv ? (uint8_t)(ob[bp >> 3] | bm) : (uint8_t)(ob[bp >> 3] & ~bm);
                }
            }
            ns.bit_pos = st.bit_pos + cntb;
        } else {
            ns.bit_pos = st.bit_pos + n;
        }
        ns.lo = (new_lo << n) & mask;
        ns.hi = (((top << n) & mask) | ((1ull << n) - 1ull)) + 1ull;
        ns.ntokens = st.ntokens + 1;
        ns.flags = (st.flags & ~NS_ST_EXACT_SUM) | (exact ? NS_ST_EXACT_SUM : 0u);
        if (!DECODE && ns.bit_pos >= nbits && !(p.flags & NS_STEP_FINISH_SENT)) ns.flags |= NS_ST_DONE;
        if (lane == 0) {
            p.state[b] = ns;
            if (!DECODE) {
                p.out_token[b] = token;
                if (p.hist && st.ntokens < p.hist_stride) p.hist[(int64_t)b * p.hist_stride + st.ntokens] = token;
            }
            if (p.trace) {
                ns_step_trace tr;
                tr.k = k;
                tr.kprime = kp;
                tr.sel = sel;
                tr.n = n;
                tr.token = token;
                tr.exact = exact ? 1 : 0;
                tr.S = S_used;
                p.trace[b] = tr;
            }
        }
    } else if (lane == 0) {
        p.state[b].flags = st.flags | err | NS_ST_DONE;
        if (p.trace) {
            ns_step_trace tr;
            tr.k = k;
            tr.kprime = kp;
            tr.sel = -1;
            tr.n = -1;
            tr.token = -1;
            tr.exact = exact ? 1 : 0;
            tr.S = S_used;
            p.trace[b] = tr;
        }
    }
    NSG_STAMP(p, b, lane, 8);
    NSG_STAMP_RT(p, b, lane, 10);
    // rare-event diagnostics only (no per-step atomics): sharded by block so waves never contend
    const int overflow = cand.ncompact;
    lds_fence();
    const uint32_t nslow = cand.scr[SCR_SLOW];
    if (lane == 0 && p.counters && (exact || overflow > 0 || nfallback || nslow)) {
        unsigned long long* c = p.counters + 4 * (blockIdx.x & (NS_COUNTER_SHARDS - 1));
        if (exact) atomicAdd(&c[0], 1ull);
        if (overflow > 0) atomicAdd(&c[1], (unsigned long long)overflow);
        if (nfallback) atomicAdd(&c[2], (unsigned long long)nfallback);
        if (nslow) atomicAdd(&c[3], (unsigned long long)nslow);
    }
}

// finish_sent (code_base/arithmetic.py:114,134-137): once the payload is consumed, emit the top-1 token
// (rank 0: max value, lowest id) each step until a sentence-ending token; the interval is left untouched.
template <typename T>
__global__ __launch_bounds__(WPB* WAVE) void finish_sent_kernel(StepParams p, const uint8_t* sent_end) {
    constexpr int W = Elem<T>::W;
    const int lane = threadIdx.x & (WAVE - 1);
    const int b = __builtin_amdgcn_readfirstlane(blockIdx.x * WPB + (int)(threadIdx.x / WAVE));
    if (b >= p.B) return;
    const ns_stream_state st = p.state[b];
    if ((st.flags & NS_ST_DONE) || st.bit_pos < p.nbits[b]) return;
    const char* rowc = (const char*)p.logits + (int64_t)b * p.ld * (int64_t)sizeof(T);
    const RowReader rd(rowc, (uint32_t)(p.ld * (int64_t)sizeof(T)));
    const int nvec = (p.V + W - 1) / W;
    uint64_t best = 0;  // max (value desc, id asc) key
    for (int v = lane; v < nvec; v += WAVE) {
        float x[W];
        Elem<T>::unpack(rd.vec(v), x);
#pragma unroll
        for (int q = 0; q < W; ++q) {
            const int j = v * W + q;
            if (j < p.V && !is_banned(p, j)) {
                const uint64_t k = make_key(x[q], (uint32_t)j);
                best = k > best ? k : best;
            }
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const uint64_t o = __shfl_xor(best, off);
        best = o > best ? o : best;
    }
    if (lane == 0) {
        const int32_t token = (int32_t)key_id(best);
        ns_stream_state ns = st;
        ns.ntokens = st.ntokens + 1;
        if (sent_end[token]) ns.flags |= NS_ST_DONE;
        p.state[b] = ns;
        p.out_token[b] = token;
        if (p.hist && st.ntokens < p.hist_stride) p.hist[(int64_t)b * p.hist_stride + st.ntokens] = token;
        if (p.trace) {
            ns_step_trace tr = {0, 0, 0, 0, token, 0, 0.0};
            p.trace[b] = tr;
        }
    }
}

__global__ void init_state_kernel(ns_stream_state* st, int B, int P) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < B) {
        ns_stream_state s;
        s.lo = 0;
        s.hi = 1ull << P;
        s.bit_pos = 0;
        s.ntokens = 0;
        s.flags = 0;
        st[b] = s;
    }
}

}  // namespace nsg

// ================================================================================================
// C ABI
// ================================================================================================

static thread_local std::string g_err;

static int fail(ns_ctx* ctx, int code, const std::string& msg) {
    if (ctx)
        ctx->err = msg;
    else
        g_err = msg;
    return code;
}

// Small batches run the split form (one workgroup of 16 fp32 / 8 fp16 waves per stream): below a few thousand
// streams one wave per stream leaves most of the chip idle and the lone wave's dependent chain sets the time.
// Automatic limit: B * NSPLIT <= 6144 waves (fp32 B <= 384, fp16 B <= 768; the forms measured equal at 8192,
// profiles/split_r02y); ns_set_split_max_batch / NSG_SPLIT_MAX_B set an explicit limit for both dtypes.
static int g_split_max_b = -2;  // -2: not read yet, -1: automatic, >= 0: explicit

static int split_setting() {
    if (g_split_max_b == -2) {
        const char* e = getenv("NSG_SPLIT_MAX_B");
        g_split_max_b = e ? std::max(0, atoi(e)) : -1;
    }
    return g_split_max_b;
}

static int split_max_b(int nsplit) {
    const int v = split_setting();
    return v >= 0 ? v : 6144 / nsplit;
}

template <typename T, bool DECODE, int NSK>
static void launch_one(const nsg::StepParams& p, hipStream_t s) {
    constexpr int NSPLIT = (64 * NSG_SAMPLE) / (nsg::WAVE * nsg::Elem<T>::W);
    if (p.spec_j > 0 && p.B <= split_max_b(NSPLIT)) {
        if (!DECODE && p.stats)  // statistics build: the per-wave partials of the extra sums merge like the fast sum
            hipLaunchKernelGGL((nsg::coder_step_kernel<T, DECODE, NSK, !DECODE, NSPLIT>), dim3(p.B),
                               dim3(NSPLIT * nsg::WAVE), 0, s, p);
        else
            hipLaunchKernelGGL((nsg::coder_step_kernel<T, DECODE, NSK, false, NSPLIT>), dim3(p.B),
                               dim3(NSPLIT * nsg::WAVE), 0, s, p);
        return;
    }
    const dim3 grid((p.B + nsg::WPB - 1) / nsg::WPB), block(nsg::WPB * nsg::WAVE);
    if (!DECODE && p.stats)  // statistics build (encode / sample only)
        hipLaunchKernelGGL((nsg::coder_step_kernel<T, DECODE, NSK, !DECODE>), grid, block, 0, s, p);
    else
        hipLaunchKernelGGL((nsg::coder_step_kernel<T, DECODE, NSK, false>), grid, block, 0, s, p);
}

template <typename T, bool DECODE>
static void launch_t(const nsg::StepParams& p, hipStream_t s) {
    // rank slots per lane from K (register footprint of the CDF tail)
    if (p.K <= 128)
        launch_one<T, DECODE, 2>(p, s);
    else if (p.K <= 320)
        launch_one<T, DECODE, 5>(p, s);
    else if (p.K <= 512)
        launch_one<T, DECODE, 8>(p, s);
    else
        launch_one<T, DECODE, (nsg::CAND - nsg::WAVE * 4) / nsg::WAVE>(p, s);
}

template <bool DECODE>
static bool launch(ns_ctx* ctx, const nsg::StepParams& p, hipStream_t s) {
    if (ctx->dtype == NS_DTYPE_F16) {
        if (p.K <= 128)
            launch_one<_Float16, DECODE, 2>(p, s);
        else if (p.K <= 320)
            launch_one<_Float16, DECODE, 5>(p, s);
        else
            launch_one<_Float16, DECODE, (nsg::CAND - nsg::WAVE * 8) / nsg::WAVE>(p, s);
    } else {
        launch_t<float, DECODE>(p, s);
    }
    return hipGetLastError() == hipSuccess;
}

extern "C" {

const char* ns_version(void) { return "nsgcoder 0.25 gfx950"; }

int ns_set_split_max_batch(int max_batch) {
    const int prev = split_setting();
    g_split_max_b = max_batch < 0 ? -1 : max_batch;
    return prev;
}

int ns_max_topk(int logits_dtype) {
    if (logits_dtype == NS_DTYPE_F64) return 0;  // provider rows: rank coder only (wide path)
    const int TS = (logits_dtype == NS_DTYPE_F16) ? nsg::WAVE * 8 : nsg::WAVE * 4;
    return nsg::CAND - TS;
}

const char* ns_last_error(const ns_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

ns_ctx* ns_create(int device, int max_batch, int vocab, int max_k, int precision, int logits_dtype) {
    if (max_batch < 1 || vocab < 2 || max_k < 1 || precision < 1 || precision > 60 ||
        (logits_dtype != NS_DTYPE_F32 && logits_dtype != NS_DTYPE_F16 && logits_dtype != NS_DTYPE_F64)) {
        fail(nullptr, NS_ERR_CONFIG, "ns_create: invalid argument");
        return nullptr;
    }
    if (max_k > ns_max_topk(logits_dtype) && vocab > 0x1FFFF) {
        fail(nullptr, NS_ERR_UNSUPPORTED, "ns_create: the wide (large top-k) path supports vocab < 131072");
        return nullptr;
    }
    if (hipSetDevice(device) != hipSuccess) {
        fail(nullptr, NS_ERR_HIP, "ns_create: hipSetDevice failed");
        return nullptr;
    }
    ns_ctx* ctx = new ns_ctx();
    ctx->device = device;
    ctx->max_batch = max_batch;
    ctx->vocab = vocab;
    ctx->max_k = max_k;
    ctx->precision = precision;
    ctx->dtype = logits_dtype;
    ctx->d_counters = nullptr;
    ctx->wide = NsgWide();
    ctx->sent_end = nullptr;
    ctx->stats = nullptr;
    ctx->ranked = nullptr;
    ctx->ranked_stride = 0;
    ctx->stamps = nullptr;
    ctx->rk_count = nullptr;
    ctx->rk_idmap = nullptr;
    ctx->rk_idmap_stride = 0;
    ctx->rk_dict = 0;
    const size_t cbytes = 4 * NS_COUNTER_SHARDS * sizeof(unsigned long long);
    if (hipMalloc((void**)&ctx->d_counters, cbytes) != hipSuccess || hipMemset(ctx->d_counters, 0, cbytes) != hipSuccess) {
        fail(nullptr, NS_ERR_HIP, "ns_create: hipMalloc failed");
        delete ctx;
        return nullptr;
    }
    if (max_k > ns_max_topk(logits_dtype) && nsg_wide_alloc(ctx) != NS_OK) {
        fail(nullptr, NS_ERR_HIP, "ns_create: allocation of the wide-path scratch failed");
        nsg_wide_free(ctx);
        (void)hipFree(ctx->d_counters);
        delete ctx;
        return nullptr;
    }
    return ctx;
}

void ns_destroy(ns_ctx* ctx) {
    if (!ctx) return;
    if (ctx->d_counters) (void)hipFree(ctx->d_counters);
    nsg_wide_free(ctx);
    delete ctx;
}

int ns_init_state(ns_ctx* ctx, ns_stream_state* d_state, int B, void* hip_stream) {
    if (!ctx || !d_state || B < 1 || B > ctx->max_batch) return fail(ctx, NS_ERR_CONFIG, "ns_init_state: bad argument");
    const int threads = 256;
    hipLaunchKernelGGL(nsg::init_state_kernel, dim3((B + threads - 1) / threads), dim3(threads), 0,
                       (hipStream_t)hip_stream, d_state, B, ctx->precision);
    if (hipGetLastError() != hipSuccess) return fail(ctx, NS_ERR_HIP, "ns_init_state: launch failed");
    return NS_OK;
}

static int prepare(ns_ctx* ctx, nsg::StepParams& p, const void* d_logits, int64_t ld, int B, double temp,
                   int topk, const int32_t* banned, int nbanned, ns_step_trace* d_trace, uint32_t flags,
                   ns_stream_state* d_state) {
    if (!ctx) return fail(ctx, NS_ERR_CONFIG, "null context");
    const int W = ctx->dtype == NS_DTYPE_F16 ? 8 : ctx->dtype == NS_DTYPE_F64 ? 2 : 4;
    const int esz = ctx->dtype == NS_DTYPE_F16 ? 2 : ctx->dtype == NS_DTYPE_F64 ? 8 : 4;
    if (!d_logits || !d_state || B < 1 || B > ctx->max_batch) return fail(ctx, NS_ERR_CONFIG, "bad batch or pointer");
    if (ld < ctx->vocab || (ld % W) != 0) return fail(ctx, NS_ERR_CONFIG, "ld must be >= vocab and a multiple of 16 bytes");
    if (((uintptr_t)d_logits & 15u) != 0u) return fail(ctx, NS_ERR_CONFIG, "logits must be 16-byte aligned");
    if (!(temp > 0.0)) return fail(ctx, NS_ERR_CONFIG, "temperature must be positive");
    if (topk < 1) return fail(ctx, NS_ERR_CONFIG, "topk must be positive");
    if (nbanned < 0 || nbanned > NS_MAX_BANNED || (nbanned > 0 && !banned))
        return fail(ctx, NS_ERR_CONFIG, "too many banned ids");
    int ban[NS_MAX_BANNED];
    int nb = 0;
    for (int i = 0; i < nbanned; ++i)
        if (banned[i] >= 0 && banned[i] < ctx->vocab) ban[nb++] = banned[i];
    std::sort(ban, ban + nb);
    nb = (int)(std::unique(ban, ban + nb) - ban);
    const int nvalid = ctx->vocab - nb;
    if (nvalid < 2) return fail(ctx, NS_ERR_CONFIG, "fewer than two valid token ids");
    const int K = std::min(topk, nvalid);
    if (K > ns_max_topk(ctx->dtype) && !ctx->wide.keys_in)
        return fail(ctx, NS_ERR_UNSUPPORTED,
                    "topk beyond the single-pass limit (ns_max_topk): create the context with max_k >= topk");
    memset(&p, 0, sizeof p);
    p.logits = d_logits;
    p.ld = ld;
    p.B = B;
    p.V = ctx->vocab;
    p.P = ctx->precision;
    p.topk = topk;
    p.K = K;
    p.inv_temp = 1.0 / temp;
    p.c32 = (float)(p.inv_temp * 1.4426950408889634);
    p.nbanned = nb;
    for (int i = 0; i < nb; ++i) p.banned[i] = ban[i];
    p.flags = flags;
    // speculative candidate threshold: the spec_j-th largest of a 64*NSG_SAMPLE-id stratified sample (whole tiles
    // spread over the row; the kernel needs at least two sample spacings, hence vocab >= 2 * 64*NSG_SAMPLE).  The
    // number of sample ids above the row's true K-th key is ~Poisson(lambda = 64*NSG_SAMPLE*K / nvalid); spec_j is
    // the smallest j with P(Poisson(lambda) >= j) <= 1e-6, so a miss (one extra row read by that wave) stays a rare
    // event for every K.  The kernel counts each lane's three largest sample values, so spec_j stays well below
    // 3*64.  NSG_SPEC_FACTOR (tuning override) instead sets spec_j = factor * lambda + 1.
    p.spec_j = 0;
    static const double spec_factor = [] {
        const char* e = getenv("NSG_SPEC_FACTOR");
        return e ? atof(e) : 0.0;
    }();
    if (ctx->vocab >= 2 * 64 * NSG_SAMPLE) {
        const double lambda = (double)K * (64.0 * NSG_SAMPLE) / (double)nvalid;
        int sj;
        if (spec_factor > 0.0) {
            sj = (int)(spec_factor * lambda) + 1;
        } else {
            double term = exp(-lambda), tail = 1.0;  // tail = P(X >= j), term = P(X = j)
            sj = 0;
            while (tail > 1e-6 && sj < 1024) {
                tail -= term;
                ++sj;
                term *= lambda / (double)sj;
            }
        }
        if (sj < 4) sj = 4;
        if (sj <= 160) p.spec_j = sj;
    }
    p.state = d_state;
    p.trace = d_trace;
    p.counters = ctx->d_counters;
    (void)esz;
    return NS_OK;
}

int ns_encode_step(ns_ctx* ctx, const void* d_logits, int64_t ld, int B, const uint8_t* d_payload,
                   int64_t payload_stride, const int64_t* d_payload_nbits, ns_stream_state* d_state,
                   int32_t* d_out_token, int32_t* d_token_hist, int64_t hist_stride, double temp, int topk,
                   const int32_t* banned, int nbanned, ns_step_trace* d_trace, uint32_t step_flags,
                   void* hip_stream) {
    if (ctx && ctx->dtype == NS_DTYPE_F64)
        return fail(ctx, NS_ERR_CONFIG, "ns_encode_step: a NS_DTYPE_F64 context holds provider probability rows (rank coder only)");
    nsg::StepParams p;
    int rc = prepare(ctx, p, d_logits, ld, B, temp, topk, banned, nbanned, d_trace, step_flags, d_state);
    if (rc != NS_OK) return rc;
    if (!d_payload || !d_payload_nbits || !d_out_token || payload_stride < 0)
        return fail(ctx, NS_ERR_CONFIG, "ns_encode_step: null payload/out pointer");
    p.payload = d_payload;
    p.payload_stride = payload_stride;
    p.nbits = d_payload_nbits;
    p.out_token = d_out_token;
    p.hist = d_token_hist;
    p.hist_stride = d_token_hist ? hist_stride : 0;
    p.stats = ctx->stats;
    p.stamps = ctx->stamps;
    if (step_flags & NS_STEP_FINISH_SENT) {
        if (!ctx->sent_end) return fail(ctx, NS_ERR_CONFIG, "NS_STEP_FINISH_SENT needs ns_set_sentence_end");
        const dim3 g((B + nsg::WPB - 1) / nsg::WPB), blk(nsg::WPB * nsg::WAVE);
        if (ctx->dtype == NS_DTYPE_F16)
            hipLaunchKernelGGL(nsg::finish_sent_kernel<_Float16>, g, blk, 0, (hipStream_t)hip_stream, p, ctx->sent_end);
        else
            hipLaunchKernelGGL(nsg::finish_sent_kernel<float>, g, blk, 0, (hipStream_t)hip_stream, p, ctx->sent_end);
    }
    const bool ok = p.K > ns_max_topk(ctx->dtype) ? nsg_wide_launch(ctx, p, false, (hipStream_t)hip_stream)
                                                  : launch<false>(ctx, p, (hipStream_t)hip_stream);
    if (!ok) return fail(ctx, NS_ERR_HIP, "ns_encode_step: launch failed");
    return NS_OK;
}

int ns_decode_step(ns_ctx* ctx, const void* d_logits, int64_t ld, int B, const int32_t* d_in_token,
                   const uint8_t* d_is_last, const uint8_t* d_active, ns_stream_state* d_state,
                   uint8_t* d_out_bits, int64_t out_stride, double temp, int topk, const int32_t* banned,
                   int nbanned, ns_step_trace* d_trace, uint32_t step_flags, void* hip_stream) {
    if (ctx && ctx->dtype == NS_DTYPE_F64)
        return fail(ctx, NS_ERR_CONFIG, "ns_decode_step: a NS_DTYPE_F64 context holds provider probability rows (rank coder only)");
    nsg::StepParams p;
    int rc = prepare(ctx, p, d_logits, ld, B, temp, topk, banned, nbanned, d_trace, step_flags, d_state);
    if (rc != NS_OK) return rc;
    if (!d_in_token || !d_is_last || !d_out_bits || out_stride < 1)
        return fail(ctx, NS_ERR_CONFIG, "ns_decode_step: null token/out pointer");
    p.in_token = d_in_token;
    p.is_last = d_is_last;
    p.active = d_active;
    p.ranked = ctx->ranked;
    p.ranked_stride = ctx->ranked_stride;
    p.out_bits = d_out_bits;
    p.out_stride = out_stride;
    const bool ok = p.K > ns_max_topk(ctx->dtype) ? nsg_wide_launch(ctx, p, true, (hipStream_t)hip_stream)
                                                  : launch<true>(ctx, p, (hipStream_t)hip_stream);
    if (!ok) return fail(ctx, NS_ERR_HIP, "ns_decode_step: launch failed");
    return NS_OK;
}

int ns_sample_step(ns_ctx* ctx, const void* d_logits, int64_t ld, int B, uint64_t seed, int64_t stream_offset,
                   ns_stream_state* d_state, int32_t* d_out_token, int32_t* d_token_hist, int64_t hist_stride,
                   double temp, int topk, const int32_t* banned, int nbanned, double* d_stats,
                   ns_step_trace* d_trace, uint32_t step_flags, void* hip_stream) {
    if (ctx && ctx->dtype == NS_DTYPE_F64)
        return fail(ctx, NS_ERR_CONFIG, "ns_sample_step: a NS_DTYPE_F64 context holds provider probability rows (rank coder only)");
    if (!ctx) return fail(ctx, NS_ERR_CONFIG, "null context");
    nsg::StepParams p;
    const int tk = topk > 0 ? topk : ctx->vocab;  // sample.py: topk <= 0 keeps every id
    int rc = prepare(ctx, p, d_logits, ld, B, temp, tk, banned, nbanned, d_trace, step_flags, d_state);
    if (rc != NS_OK) return rc;
    if (!d_out_token) return fail(ctx, NS_ERR_CONFIG, "ns_sample_step: null output pointer");
    p.sample = 1;
    p.seed = seed;
    p.stream_offset = stream_offset;
    p.stats = d_stats;
    p.out_token = d_out_token;
    p.hist = d_token_hist;
    p.hist_stride = d_token_hist ? hist_stride : 0;
    const bool ok = p.K > ns_max_topk(ctx->dtype) ? nsg_wide_launch(ctx, p, false, (hipStream_t)hip_stream)
                                                  : launch<false>(ctx, p, (hipStream_t)hip_stream);
    if (!ok) return fail(ctx, NS_ERR_HIP, "ns_sample_step: launch failed");
    return NS_OK;
}

static int rank_prepare(ns_ctx* ctx, nsg::StepParams& p, const void* d_logits, int64_t ld, int B, double temp,
                        const ns_rank_quality* q, ns_step_trace* d_trace, uint32_t flags, ns_stream_state* d_state) {
    if (!ctx) return fail(ctx, NS_ERR_CONFIG, "null context");
    if (!q) return fail(ctx, NS_ERR_CONFIG, "rank step: null quality");
    if (q->top_p > 1.0) return fail(ctx, NS_ERR_CONFIG, "top_p must be within (0, 1]");
    if (q->prob_temp > 0.0 && (q->cap_bits > 0 || q->min_prob >= 0.0))
        return fail(ctx, NS_ERR_CONFIG, "crypto quality (prob_temp) takes only top_k and top_p");
    if (ctx->dtype == NS_DTYPE_F64 && temp != 1.0)
        return fail(ctx, NS_ERR_CONFIG, "provider probability rows take no temperature (temp must be 1)");
    if (ctx->vocab > 0x1FFFF) return fail(ctx, NS_ERR_UNSUPPORTED, "rank coder: vocab must be < 131072");
    if (!ctx->wide.keys_in && nsg_wide_alloc(ctx) != NS_OK) {
        nsg_wide_free(ctx);
        return fail(ctx, NS_ERR_HIP, "rank coder: scratch allocation failed");
    }
    const int rc = prepare(ctx, p, d_logits, ld, B, temp, ctx->vocab, nullptr, 0, d_trace, flags, d_state);
    if (rc != NS_OK) return rc;
    p.rank = 1;
    p.rk_top_k = q->top_k;
    p.rk_cap = q->cap_bits;
    p.rk_top_p = q->top_p;
    p.rk_min_prob = q->min_prob;
    // crypto/quality.py:60: the temperature step runs unless math.isclose(T, 1.0) (rel_tol 1e-9)
    const double pt = q->prob_temp;
    p.rk_ptemp = (pt > 0.0 && fabs(pt - 1.0) > 1e-9 * fmax(pt, 1.0)) ? pt : 0.0;
    p.rk_crypto = pt > 0.0 ? 1 : 0;
    if (ctx->dtype == NS_DTYPE_F64) {
        p.rk_count = ctx->rk_count;
        p.rk_idmap = ctx->rk_idmap;
        p.rk_idmap_stride = ctx->rk_idmap_stride;
        p.rk_dict = ctx->rk_dict;
    }
    return NS_OK;
}

int ns_rank_encode_step(ns_ctx* ctx, const void* d_logits, int64_t ld, int B, const uint8_t* d_payload,
                        int64_t payload_stride, const int64_t* d_payload_nbits, ns_stream_state* d_state,
                        int32_t* d_out_token, int32_t* d_token_hist, int32_t* d_consumed_hist, int64_t hist_stride,
                        double temp, const ns_rank_quality* quality, ns_step_trace* d_trace, uint32_t step_flags,
                        void* hip_stream) {
    nsg::StepParams p;
    int rc = rank_prepare(ctx, p, d_logits, ld, B, temp, quality, d_trace, step_flags, d_state);
    if (rc != NS_OK) return rc;
    if (!d_payload || !d_payload_nbits || !d_out_token || payload_stride < 0)
        return fail(ctx, NS_ERR_CONFIG, "ns_rank_encode_step: null payload/out pointer");
    p.payload = d_payload;
    p.payload_stride = payload_stride;
    p.nbits = d_payload_nbits;
    p.out_token = d_out_token;
    p.hist = d_token_hist;
    p.rk_cons = d_consumed_hist;
    p.hist_stride = (d_token_hist || d_consumed_hist) ? hist_stride : 0;
    if (!nsg_rank_launch(ctx, p, false, (hipStream_t)hip_stream))
        return fail(ctx, NS_ERR_HIP, "ns_rank_encode_step: launch failed");
    return NS_OK;
}

int ns_rank_decode_step(ns_ctx* ctx, const void* d_logits, int64_t ld, int B, const int32_t* d_in_token,
                        const int32_t* d_keep_bits, const uint8_t* d_active, ns_stream_state* d_state,
                        uint8_t* d_out_bits, int64_t out_stride, double temp, const ns_rank_quality* quality,
                        ns_step_trace* d_trace, uint32_t step_flags, void* hip_stream) {
    nsg::StepParams p;
    int rc = rank_prepare(ctx, p, d_logits, ld, B, temp, quality, d_trace, step_flags, d_state);
    if (rc != NS_OK) return rc;
    if (!d_in_token || !d_keep_bits || !d_out_bits || out_stride < 1)
        return fail(ctx, NS_ERR_CONFIG, "ns_rank_decode_step: null token/out pointer");
    p.in_token = d_in_token;
    p.rk_keep = d_keep_bits;
    p.active = d_active;
    p.out_bits = d_out_bits;
    p.out_stride = out_stride;
    if (!nsg_rank_launch(ctx, p, true, (hipStream_t)hip_stream))
        return fail(ctx, NS_ERR_HIP, "ns_rank_decode_step: launch failed");
    return NS_OK;
}

int ns_token_probs(ns_ctx* ctx, const void* d_logits, int64_t ld, int B, double temp, const ns_rank_quality* quality,
                   double* d_probs, int64_t probs_stride, ns_stream_state* d_scratch_state, void* hip_stream) {
    if (ctx && ctx->dtype == NS_DTYPE_F64)
        return fail(ctx, NS_ERR_CONFIG, "ns_token_probs: a NS_DTYPE_F64 context holds provider probability rows (rank coder only)");
    nsg::StepParams p;
    int rc = rank_prepare(ctx, p, d_logits, ld, B, temp, quality, nullptr, 0, d_scratch_state);
    if (rc != NS_OK) return rc;
    if (!d_probs || probs_stride < ctx->vocab) return fail(ctx, NS_ERR_CONFIG, "ns_token_probs: bad output");
    p.probs_out = d_probs;
    p.probs_stride = probs_stride;
    hipLaunchKernelGGL(nsg::init_state_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)hip_stream,
                       d_scratch_state, B, ctx->precision);
    if (!nsg_rank_launch(ctx, p, true, (hipStream_t)hip_stream))
        return fail(ctx, NS_ERR_HIP, "ns_token_probs: launch failed");
    return NS_OK;
}

int ns_set_rank_rows(ns_ctx* ctx, const int32_t* d_count, const int32_t* d_idmap, int64_t idmap_stride,
                     int dict_rows) {
    if (!ctx) return fail(ctx, NS_ERR_CONFIG, "ns_set_rank_rows: null context");
    if (ctx->dtype != NS_DTYPE_F64) return fail(ctx, NS_ERR_CONFIG, "ns_set_rank_rows: needs a NS_DTYPE_F64 context");
    if (d_idmap && idmap_stride < ctx->vocab) return fail(ctx, NS_ERR_CONFIG, "ns_set_rank_rows: idmap stride < vocab");
    ctx->rk_count = d_count;
    ctx->rk_idmap = d_idmap;
    ctx->rk_idmap_stride = d_idmap ? idmap_stride : 0;
    ctx->rk_dict = dict_rows ? 1 : 0;
    return NS_OK;
}

int ns_set_rank_export(ns_ctx* ctx, int32_t* d_ranked, int stride) {
    if (!ctx || (d_ranked && stride < 2)) return fail(ctx, NS_ERR_CONFIG, "ns_set_rank_export: bad argument");
    ctx->ranked = d_ranked;
    ctx->ranked_stride = d_ranked ? stride : 0;
    return NS_OK;
}

#ifdef NSG_STAMPS
int ns_set_stamps(ns_ctx* ctx, uint64_t* d_stamps) {  // diagnostic builds only (not in the public header)
    if (!ctx) return NS_ERR_CONFIG;
    ctx->stamps = d_stamps;
    return NS_OK;
}
#endif

int ns_set_stats(ns_ctx* ctx, double* d_stats) {
    if (!ctx) return fail(ctx, NS_ERR_CONFIG, "null context");
    ctx->stats = d_stats;
    return NS_OK;
}

int ns_set_sentence_end(ns_ctx* ctx, const uint8_t* d_table) {
    if (!ctx) return fail(ctx, NS_ERR_CONFIG, "ns_set_sentence_end: null context");
    ctx->sent_end = d_table;
    return NS_OK;
}

int ns_read_counters(ns_ctx* ctx, uint64_t* host_counters4) {
    if (!ctx || !host_counters4) return fail(ctx, NS_ERR_CONFIG, "ns_read_counters: bad argument");
    unsigned long long h[4 * NS_COUNTER_SHARDS];
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(h, ctx->d_counters, sizeof h, hipMemcpyDeviceToHost) != hipSuccess)
        return fail(ctx, NS_ERR_HIP, "ns_read_counters: copy failed");
    for (int i = 0; i < 4; ++i) host_counters4[i] = 0;
    for (int sh = 0; sh < NS_COUNTER_SHARDS; ++sh)
        for (int i = 0; i < 4; ++i) host_counters4[i] += h[4 * sh + i];
    return NS_OK;
}

}  // extern "C"

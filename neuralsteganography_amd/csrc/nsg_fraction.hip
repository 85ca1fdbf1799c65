// The src package's exact-rational arithmetic coder (encode_bits / decode_bits,
// src/neuralstego/codec/arithmetic.py:234-325, 408-550) as a batched device kernel -- include/nsg_fraction.h.
//
// Exact arithmetic without fractions.Fraction.  A step's distribution is V float64 values p_i; the reference
// turns each into f_i = limit_denominator(p_i, 2^30) (:545-550) and normalises by their exact sum T (:469-485),
// token i owning [c_i, c_{i+1}) with c_i = (f_0 + ... + f_{i-1}) / T.  With D = lcm of the f_i's denominators
// every c_i is N_i / N_V for the integers N_i = D (f_0 + ... + f_{i-1}), and the coder's interval is held as
// three integers, lo = PL / Q and hi = PH / Q (start 0/1, 1/1).  Token j's interval is then
//     [ (PL N_V + W N_j) / (Q N_V),  (PL N_V + W N_{j+1}) / (Q N_V) ),   W = PH - PL,
// and choosing it makes those numerators and Q N_V the new PL, PH, Q -- the same rational values as the
// reference's reduced fractions, so every comparison it makes gives the same answer here.
//
// Encode (:408-434): for depth d = 1, 2, ... the next d payload bits v (zero past the end) give the dyadic
// interval [v / 2^d, (v + 1) / 2^d); the first token whose interval contains it is taken, consuming d bits.
// Multiplying through by Q N_V 2^d, token j contains it iff
//     W N_j 2^d <= R1(d)   and   R2(d) <= W N_{j+1} 2^d,
// with R1(d) = N_V (v Q - PL 2^d) and R2(d) = R1(d) + N_V Q.  Going from d to d + 1 doubles every term and adds
// the new bit times N_V Q to R1, so each depth costs a few shifts and compares, not a product.  R1(d) / 2^d only
// grows with d (v / 2^d does), so the last token starting at or below v / 2^d -- the only candidate, intervals
// being disjoint -- only moves forward: it is tracked as one index for the whole step.
//
// Decode (:437-466, 500-530): narrow to the received token, then the ceil / floor of PL 2^L / Q and
// (PH 2^L - 1) / Q (Knuth division) give the L-bit prefix.
//
// Work split: one wavefront per stream.  The lanes convert the V values to fractions (nsg_bigint.h
// to_fraction), form the terms T_i = f_i D (one lane per token) and the prefix sums (all lanes, one 64-limb
// chunk per instruction with a ballot carry chain); lane 0 runs the interval arithmetic, which is sequential by
// nature.  Every integer lives in a per-stream global-memory arena; an integer that outgrows its room ends the
// step with NS_FRAC_ERR_CAPACITY and leaves the stream's state as it was.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "nsg_bigint.h"
#include "nsg_coder.h"
#include "nsg_fraction.h"

using nsg::bi::limb;

namespace nsg {
namespace frac {

struct Stream {
    int64_t pos;    // payload bits consumed (the reference's BitReader position)
    int64_t nbits;  // payload bits
    int32_t npl, nph, nq;
    int32_t pad;
};

constexpr int NTMP = 12;  // integer temporaries per stream

struct Args {
    Stream* st;
    limb* state;  // [B][3][cap]: PL, PH, Q
    int cap;
    limb* scratch;
    int64_t sstride;  // limbs per stream
    int64_t tmp;      // limbs per temporary
    int64_t table_limbs;
    int64_t max_bits;  // encode: payload bits, decode: bits per token -- what the temporaries are sized for
    const double* probs;
    const int32_t* ids;
    int64_t ld;
    const int32_t* count;
    const uint8_t* bits;  // encode: payload bits
    int64_t bits_stride;
    const int32_t* token_in;  // decode
    const int32_t* used_in;
    uint8_t* out_bits;
    int64_t out_stride;
    int64_t* out_pos;
    int32_t* token_out;  // encode
    int32_t* used_out;
    int32_t* status;
    const int32_t* slot;  // scratch slot of stream b (ns_frac_set_slots), or null: slot b
    int64_t nslots;       // scratch slots allocated
};

// dst += src over n limbs, every lane of the wave taking one limb per 64-limb chunk.  Carries between lanes:
// with G = lanes whose sum overflowed and P = lanes whose sum is all ones, the carry into lane i is bit i of
// (G + (G | P) + c_in) ^ P -- the integer addition runs the carry recurrence c_{i+1} = G_i | (P_i & c_i).
__device__ void wave_add(limb* __restrict__ dst, const limb* __restrict__ src, int n) {
    const int lane = threadIdx.x & 63;
    uint64_t cin = 0;
    for (int base = 0; base < n; base += 64) {
        const int i = base + lane;
        uint64_t s = 0;
        if (i < n) s = (uint64_t)dst[i] + src[i];
        const uint32_t lo = (uint32_t)s;
        const uint64_t G = __ballot((s >> 32) != 0);
        const uint64_t P = __ballot(i < n && lo == 0xFFFFFFFFu);
        const uint64_t carries = (G + (G | P) + cin) ^ P;
        if (i < n) dst[i] = lo + (uint32_t)((carries >> lane) & 1);
        cin = ((G >> 63) | ((P >> 63) & (carries >> 63))) & 1;
    }
}

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = max(v, __shfl_xor(v, off));
    return v;
}

// ---------------------------------------------------------------------------------------------- encode step
__device__ int encode_serial(Stream& st, limb* PL, limb* PH, limb* Q, int cap, limb* const* T, int64_t tmp,
                             const limb* tab, int SW, int V, const int32_t* ids, const uint8_t* bits, int32_t* tok,
                             int32_t* used) {
    using namespace nsg::bi;
    const limb* NT = tab + (int64_t)V * SW;
    const int nNT = trim(NT, SW);
    if (nNT == 0) return NS_FRAC_ERR_NO_MASS;
    limb *W = T[0], *NTQ = T[1], *PLNT = T[2], *R1 = T[3], *R2 = T[4], *A = T[5], *Bv = T[6];
    const int npl = st.npl, nph = st.nph, nq = st.nq;
    const int nW = sub(W, PH, nph, PL, npl);
    const int nNTQ = mul(NTQ, NT, nNT, Q, nq);
    const int nPLNT = mul(PLNT, PL, npl, NT, nNT);
    // R1(0) = -N_V PL, kept as sign + magnitude
    int nR1 = copy(R1, PLNT, nPLNT);
    bool neg = nR1 > 0;
    int nA = 0, j = 0;
    int nB = mul(Bv, W, nW, tab + SW, SW);  // W N_1 2^0
    const int64_t total = st.nbits, pos = st.pos, maxd = total + 64;
    const int64_t room = tmp - 2;
    for (int64_t d = 1; d <= maxd; ++d) {
        const int64_t at = pos + d - 1;
        const int bit = at < total ? bits[at] : 0;
        nR1 = shl(R1, R1, nR1, 1);
        if (bit) {
            if (!neg) {
                nR1 = add(R1, R1, nR1, NTQ, nNTQ);
            } else if (cmp(R1, nR1, NTQ, nNTQ) <= 0) {
                nR1 = sub(R1, NTQ, nNTQ, R1, nR1);
                neg = false;
            } else {
                nR1 = sub(R1, R1, nR1, NTQ, nNTQ);
            }
        }
        if (nR1 == 0) neg = false;
        nA = shl(A, A, nA, 1);
        nB = shl(Bv, Bv, nB, 1);
        if (nR1 > room || nB > room) return NS_FRAC_ERR_CAPACITY;
        if (neg) continue;  // v / 2^d < lo: no token starts at or below it
        while (cmp(Bv, nB, R1, nR1) <= 0) {  // token j + 1 starts at or below v / 2^d
            ++j;
            nA = copy(A, Bv, nB);
            if (j == V) break;
            nB = mul(Bv, W, nW, tab + (int64_t)(j + 1) * SW, SW);
            if (nB + (d >> 5) + 2 > room) return NS_FRAC_ERR_CAPACITY;
            nB = shl(Bv, Bv, nB, (int)d);
        }
        // hi <= v / 2^d: no token contains the prefix at this depth, nor at any deeper one (v / 2^d only grows),
        // and the reference's search ends in the same error at depth total + 64
        if (j == V) return NS_FRAC_ERR_UNRESOLVED;
        const int nR2 = add(R2, R1, nR1, NTQ, nNTQ);
        if (cmp(R2, nR2, Bv, nB) <= 0) {
            nA = shr(A, A, nA, (int)d);
            nB = shr(Bv, Bv, nB, (int)d);
            if ((nPLNT > nB ? nPLNT : nB) + 1 > cap || nNTQ > cap) return NS_FRAC_ERR_CAPACITY;
            st.npl = add(PL, PLNT, nPLNT, A, nA);
            st.nph = add(PH, PLNT, nPLNT, Bv, nB);
            st.nq = copy(Q, NTQ, nNTQ);
            *tok = ids[j];
            *used = (int32_t)d;
            const int64_t left = total - pos > 0 ? total - pos : 0;
            st.pos = pos + (d < left ? d : left);
            return NS_FRAC_OK;
        }
    }
    return NS_FRAC_ERR_UNRESOLVED;
}

// ---------------------------------------------------------------------------------------------- decode step
__device__ bool prefix_fits(const limb* c, int nc, const limb* NQ, int nNQ, const limb* X, int nX, const limb* Y,
                            int nY, limb* prod, limb* c1) {
    using namespace nsg::bi;
    const limb one[1] = {1};
    int np = mul(prod, c, nc, NQ, nNQ);
    if (cmp(prod, np, X, nX) < 0) return false;  // c / 2^L < lo
    const int n1 = add(c1, c, nc, one, 1);
    np = mul(prod, c1, n1, NQ, nNQ);
    return cmp(prod, np, Y, nY) <= 0;  // (c + 1) / 2^L <= hi
}

__device__ int decode_serial(Stream& st, limb* PL, limb* PH, limb* Q, int cap, limb* const* T, const limb* tab,
                             int SW, int V, int j, int L, uint8_t* out, int64_t* out_pos) {
    using namespace nsg::bi;
    const limb* NT = tab + (int64_t)V * SW;
    const int nNT = trim(NT, SW);
    if (nNT == 0) return NS_FRAC_ERR_NO_MASS;
    if (j < 0) return NS_FRAC_ERR_NOT_PRESENT;
    const limb* Nj = tab + (int64_t)j * SW;
    const limb* Nj1 = Nj + SW;
    if (cmp(Nj1, SW, Nj, SW) <= 0) return NS_FRAC_ERR_NOT_PRESENT;  // zero probability: not in the reference's cdf
    const int npl = st.npl, nph = st.nph, nq = st.nq;
    limb *W = T[0], *PLNT = T[1], *A = T[2], *Bv = T[3], *NQ = T[4], *PL2 = T[5], *PH2 = T[6];
    const int nW = sub(W, PH, nph, PL, npl);
    const int nPLNT = mul(PLNT, PL, npl, NT, nNT);
    const int nA = mul(A, W, nW, Nj, SW);
    const int nB = mul(Bv, W, nW, Nj1, SW);
    const int nNQ = mul(NQ, Q, nq, NT, nNT);
    const int npl2 = add(PL2, PLNT, nPLNT, A, nA);
    const int nph2 = add(PH2, PLNT, nPLNT, Bv, nB);
    if (npl2 > cap || nph2 > cap || nNQ > cap) return NS_FRAC_ERR_CAPACITY;
    if (L > 0) {
        const limb one[1] = {1};
        limb *X = T[7], *Y = T[8], *UN = T[9], *VN = T[0], *QF = T[1], *RR = T[2], *QL = T[3], *Y1 = T[10];
        limb* P = T[11];
        const int nX = shl(X, PL2, npl2, L);
        const int nY = shl(Y, PH2, nph2, L);
        int nrr = 0;
        int nqf = divmod(QF, RR, &nrr, X, nX, NQ, nNQ, UN, VN);  // ceil(lo 2^L)
        if (nrr) nqf = add(QF, QF, nqf, one, 1);
        const int ny1 = sub(Y1, Y, nY, one, 1);
        const int nql = divmod(QL, RR, &nrr, Y1, ny1, NQ, nNQ, UN, VN);  // largest c with c + 1 <= hi 2^L
        const limb* cand = cmp(QF, nqf, QL, nql) <= 0 ? QF : QL;
        int nc = cand == QF ? nqf : nql;
        if (!prefix_fits(cand, nc, NQ, nNQ, X, nX, Y, nY, P, RR)) {
            cand = QL;
            nc = nql;
            if (!prefix_fits(cand, nc, NQ, nNQ, X, nX, Y, nY, P, RR)) return NS_FRAC_ERR_NO_PREFIX;
        }
        const int64_t o = *out_pos;
        for (int k = 0; k < L; ++k) {
            const int bp = L - 1 - k;
            out[o + k] = (bp >> 5) < nc ? (uint8_t)((cand[bp >> 5] >> (bp & 31)) & 1) : (uint8_t)0;
        }
        *out_pos = o + L;
    }
    st.npl = copy(PL, PL2, npl2);
    st.nph = copy(PH, PH2, nph2);
    st.nq = copy(Q, NQ, nNQ);
    return NS_FRAC_OK;
}

// --------------------------------------------------------------------------------------------------- kernel
template <bool DECODE>
__global__ __launch_bounds__(64) void frac_step_kernel(Args a) {
    using namespace nsg::bi;
    const int b = blockIdx.x, lane = threadIdx.x;
    __shared__ int s_nd, s_sw, s_err;
    Stream& st = a.st[b];
    const int V = a.count[b];
    const int64_t slot = a.slot ? (int64_t)a.slot[b] : (int64_t)b;
    bool skip = V < 0 || slot < 0;
    if constexpr (DECODE) {
        skip = skip || a.used_in[b] < 0;
    } else {
        skip = skip || st.pos >= st.nbits;
    }
    if (skip) {  // token / used are left as they are: a skipped stream may have run in an earlier launch
        if (lane == 0) a.status[b] = NS_FRAC_SKIPPED;
        return;
    }
    bool fits = V <= a.ld && slot < a.nslots;
    if constexpr (DECODE) {
        fits = fits && a.used_in[b] <= a.max_bits && a.out_pos[b] + a.used_in[b] <= a.out_stride;
    } else {
        fits = fits && st.nbits <= a.max_bits;
    }
    if (!fits) {
        if (lane == 0) a.status[b] = NS_FRAC_ERR_CAPACITY;
        return;
    }
    limb* base = a.scratch + slot * a.sstride;
    uint64_t* fm = (uint64_t*)base;
    int* fsh = (int*)(base + 2 * a.ld);
    uint32_t* fd = base + 3 * a.ld;
    limb* D = base + 4 * a.ld;
    limb* T[NTMP];
#pragma unroll
    for (int k = 0; k < NTMP; ++k) T[k] = D + a.cap + 2 + k * a.tmp;
    limb* tab = D + a.cap + 2 + NTMP * a.tmp;
    const double* row = a.probs + (int64_t)b * a.ld;
    const int32_t* idr = a.ids + (int64_t)b * a.ld;

    // 1. fractions (lanes over tokens)
    int maxs = 0;
    for (int i = lane; i < V; i += 64) {
        uint64_t m;
        int s;
        uint32_t d;
        to_fraction(row[i], &m, &s, &d);
        fm[i] = m;
        fsh[i] = s;
        fd[i] = d;
        maxs = max(maxs, s);
    }
    maxs = wave_max(maxs);
    __syncthreads();
    // 2. common denominator D = lcm of the denominators (lane 0: a running product divided by gcds)
    if (lane == 0) {
        int nd = set_u64(D, 1);
        int err = 0;
        uint32_t last = 1;
        for (int i = 0; i < V; ++i) {
            const uint32_t di = fd[i];
            if (di == 1 || di == last) continue;
            last = di;
            const uint32_t g = (uint32_t)gcd_u64(mod_u32(D, nd, di), di);
            const uint32_t f = di / g;
            if (f > 1) {
                if (nd + 2 > a.cap) {
                    err = 1;
                    break;
                }
                nd = mul_u64(D, D, nd, f);
            }
        }
        // a term f_i D < 2^(32 nd + 64 + maxs); V + 1 <= 2^31 of them sum below 2^32 times that
        const int sw = nd + 2 + (maxs + 31) / 32 + 2;
        // the interval arena (cap) bounds D and a table row; only a short table is cured by a larger one
        s_err = (err || sw > a.cap) ? NS_FRAC_ERR_CAPACITY : (int64_t)(V + 1) * sw > a.table_limbs ? NS_FRAC_ERR_TABLE : 0;
        s_nd = nd;
        s_sw = sw;
    }
    __syncthreads();
    if (s_err) {
        if (lane == 0) a.status[b] = s_err;
        return;
    }
    const int nd = s_nd, SW = s_sw;
    // 3. terms T_i = f_i D = m_i 2^s_i (D / d_i) into table slot i + 1 (lanes over tokens); slot 0 = N_0 = 0
    for (int i = lane; i < V; i += 64) {
        limb* slot = tab + (int64_t)(i + 1) * SW;
        int n = 0;
        if (fm[i]) {
            divmod_u32(slot, D, nd, fd[i]);
            n = trim(slot, nd);
            n = mul_u64(slot, slot, n, fm[i]);
            if (fsh[i]) n = shl(slot, slot, n, fsh[i]);
        }
        for (int k = n; k < SW; ++k) slot[k] = 0;
    }
    for (int k = lane; k < SW; k += 64) tab[k] = 0;
    __syncthreads();
    // 4. prefix sums N_{i+1} = N_i + T_i (all lanes, limb-parallel)
    for (int i = 1; i <= V; ++i) wave_add(tab + (int64_t)i * SW, tab + (int64_t)(i - 1) * SW, SW);
    // 5. decode: the received token's position in the distribution
    int jj = -1;
    if constexpr (DECODE) {
        const int t = a.token_in[b];
        for (int base_i = 0; base_i < V; base_i += 64) {
            const int i = base_i + lane;
            const uint64_t m = __ballot(i < V && idr[i] == t);
            if (m) {
                jj = base_i + __builtin_ctzll(m);
                break;
            }
        }
    }
    __syncthreads();
    if (lane != 0) return;
    // 6. the interval arithmetic (lane 0)
    limb* PL = a.state + (int64_t)b * 3 * a.cap;
    limb* PH = PL + a.cap;
    limb* Q = PH + a.cap;
    Stream s = st;
    int rc;
    if constexpr (DECODE) {
        rc = decode_serial(s, PL, PH, Q, a.cap, T, tab, SW, V, jj, a.used_in[b], a.out_bits + (int64_t)b * a.out_stride,
                           a.out_pos + b);
    } else {
        rc = encode_serial(s, PL, PH, Q, a.cap, T, a.tmp, tab, SW, V, idr, a.bits + (int64_t)b * a.bits_stride,
                           a.token_out + b, a.used_out + b);
    }
    if (rc == NS_FRAC_OK) st = s;
    a.status[b] = rc;
}

__global__ void frac_init_kernel(Stream* st, limb* state, int cap, const int64_t* nbits, int B) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    Stream s;
    s.pos = 0;
    s.nbits = nbits[b];
    s.npl = 0;  // lo = 0 / 1
    s.nph = 1;  // hi = 1 / 1
    s.nq = 1;
    s.pad = 0;
    st[b] = s;
    limb* PL = state + (int64_t)b * 3 * cap;
    PL[0] = 0;
    PL[cap] = 1;
    PL[2 * cap] = 1;
}

}  // namespace frac
}  // namespace nsg

// ------------------------------------------------------------------------------------------------------ host
struct ns_frac_ctx {
    int device = 0;
    int max_batch = 0;
    int cap = 0;
    nsg::frac::Stream* st = nullptr;
    limb* state = nullptr;
    int64_t* nbits = nullptr;
    limb* scratch = nullptr;
    size_t scratch_bytes = 0;
    const int32_t* slot = nullptr;  // ns_frac_set_slots
    int nslots = 0;
    std::string err;
};

static thread_local std::string g_frac_err;

static int frac_fail(ns_frac_ctx* ctx, const std::string& msg, int code) {
    if (ctx) ctx->err = msg;
    g_frac_err = msg;
    return code;
}

extern "C" ns_frac_ctx* ns_frac_create(int max_batch, int cap_limbs, int device) {
    if (max_batch <= 0 || cap_limbs < 8 || cap_limbs > (1 << 26)) {
        g_frac_err = "ns_frac_create: max_batch > 0 and 8 <= cap_limbs <= 2^26 required";
        return nullptr;
    }
    if (hipSetDevice(device) != hipSuccess) {
        g_frac_err = "ns_frac_create: hipSetDevice failed";
        return nullptr;
    }
    ns_frac_ctx* ctx = new ns_frac_ctx();
    ctx->device = device;
    ctx->max_batch = max_batch;
    ctx->cap = cap_limbs;
    if (hipMalloc(&ctx->st, sizeof(nsg::frac::Stream) * (size_t)max_batch) != hipSuccess ||
        hipMalloc(&ctx->state, sizeof(limb) * 3 * (size_t)cap_limbs * max_batch) != hipSuccess ||
        hipMalloc(&ctx->nbits, sizeof(int64_t) * (size_t)max_batch) != hipSuccess) {
        g_frac_err = "ns_frac_create: hipMalloc failed";
        ns_frac_destroy(ctx);
        return nullptr;
    }
    return ctx;
}

extern "C" void ns_frac_destroy(ns_frac_ctx* ctx) {
    if (!ctx) return;
    (void)hipFree(ctx->st);
    (void)hipFree(ctx->state);
    (void)hipFree(ctx->nbits);
    (void)hipFree(ctx->scratch);
    delete ctx;
}

extern "C" const char* ns_frac_last_error(const ns_frac_ctx* ctx) {
    return ctx ? ctx->err.c_str() : g_frac_err.c_str();
}

extern "C" int ns_frac_init(ns_frac_ctx* ctx, int B, const int64_t* h_nbits, void* hip_stream) {
    if (!ctx || !h_nbits || B <= 0 || B > ctx->max_batch) return frac_fail(ctx, "ns_frac_init: bad batch", NS_ERR_CONFIG);
    for (int b = 0; b < B; ++b)
        if (h_nbits[b] < 0) return frac_fail(ctx, "ns_frac_init: negative payload length", NS_ERR_CONFIG);
    const hipStream_t s = (hipStream_t)hip_stream;
    if (hipMemcpyAsync(ctx->nbits, h_nbits, sizeof(int64_t) * B, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return frac_fail(ctx, "ns_frac_init: copy failed", NS_ERR_HIP);
    hipLaunchKernelGGL(nsg::frac::frac_init_kernel, dim3((B + 63) / 64), dim3(64), 0, s, ctx->st, ctx->state,
                       ctx->cap, ctx->nbits, B);
    return hipGetLastError() == hipSuccess ? NS_OK : frac_fail(ctx, "ns_frac_init: launch failed", NS_ERR_HIP);
}

// per-stream scratch: fractions (4 limbs per entry), D, NTMP temporaries, the cumulative table
static int64_t frac_tmp_limbs(int cap, int64_t max_bits) { return 2 * (int64_t)cap + (max_bits + 64) / 32 + 8; }

static int64_t frac_stride_limbs(int cap, int64_t ld, int64_t max_bits, int64_t table_limbs) {
    int64_t stride = 4 * ld + cap + 2 + nsg::frac::NTMP * frac_tmp_limbs(cap, max_bits) + table_limbs;
    return stride + (stride & 1);  // 8-byte alignment of the next stream's fraction numerators
}

static int frac_prepare(ns_frac_ctx* ctx, int B, int64_t ld, int64_t max_bits, int64_t table_limbs, hipStream_t s,
                        nsg::frac::Args& a) {
    // max_bits bounds lane 0's depth search (one iteration per payload bit a failing step tries, each linear in
    // the integers' size, which grows by a bit per depth): 2^20 keeps the worst step of a stream to seconds
    if (B <= 0 || B > ctx->max_batch || ld < 0 || ld > (1 << 28) || max_bits < 0 || max_bits > ((int64_t)1 << 20) ||
        table_limbs < 2 || table_limbs > ((int64_t)1 << 30))
        return frac_fail(ctx, "ns_frac step: bad sizes", NS_ERR_CONFIG);
    if (ctx->slot && ctx->nslots > B) return frac_fail(ctx, "ns_frac step: more slots than streams", NS_ERR_CONFIG);
    const int64_t tmp = frac_tmp_limbs(ctx->cap, max_bits);
    const int64_t stride = frac_stride_limbs(ctx->cap, ld, max_bits, table_limbs);
    const size_t bytes = sizeof(limb) * (size_t)stride * (size_t)(ctx->slot ? ctx->nslots : B);
    if (bytes > ctx->scratch_bytes) {
        (void)hipStreamSynchronize(s);
        (void)hipFree(ctx->scratch);
        ctx->scratch = nullptr;
        ctx->scratch_bytes = 0;
        if (hipMalloc(&ctx->scratch, bytes) != hipSuccess)
            return frac_fail(ctx, "ns_frac step: hipMalloc of " + std::to_string(bytes) + " B of scratch failed",
                             NS_ERR_HIP);
        ctx->scratch_bytes = bytes;
    }
    a = nsg::frac::Args{};
    a.st = ctx->st;
    a.state = ctx->state;
    a.cap = ctx->cap;
    a.scratch = ctx->scratch;
    a.sstride = stride;
    a.tmp = tmp;
    a.table_limbs = table_limbs;
    a.max_bits = max_bits;
    a.ld = ld;
    a.slot = ctx->slot;
    a.nslots = ctx->slot ? ctx->nslots : B;
    return NS_OK;
}

extern "C" int ns_frac_set_slots(ns_frac_ctx* ctx, const int32_t* d_slot, int nslots) {
    if (!ctx) return frac_fail(ctx, "ns_frac_set_slots: null context", NS_ERR_CONFIG);
    if (d_slot && (nslots <= 0 || nslots > ctx->max_batch))
        return frac_fail(ctx, "ns_frac_set_slots: 0 < nslots <= max_batch required", NS_ERR_CONFIG);
    ctx->slot = d_slot;
    ctx->nslots = d_slot ? nslots : 0;
    return NS_OK;
}

extern "C" int64_t ns_frac_scratch_bytes(const ns_frac_ctx* ctx, int nslots, int64_t ld, int64_t max_bits,
                                         int64_t table_limbs) {
    if (!ctx || nslots < 0 || ld < 0 || max_bits < 0 || table_limbs < 0) return -1;
    return (int64_t)sizeof(limb) * frac_stride_limbs(ctx->cap, ld, max_bits, table_limbs) * nslots;
}

extern "C" int ns_frac_encode_step(ns_frac_ctx* ctx, int B, const double* d_probs, const int32_t* d_ids, int64_t ld,
                                   const int32_t* d_count, const uint8_t* d_bits, int64_t bits_stride,
                                   int64_t max_bits, int64_t table_limbs, int32_t* d_token, int32_t* d_used,
                                   int32_t* d_status, void* hip_stream) {
    if (!ctx) return frac_fail(ctx, "ns_frac_encode_step: null context", NS_ERR_CONFIG);
    if (!d_probs || !d_ids || !d_count || !d_bits || !d_token || !d_used || !d_status || bits_stride < max_bits)
        return frac_fail(ctx, "ns_frac_encode_step: null buffer or bits_stride < max_bits", NS_ERR_CONFIG);
    const hipStream_t s = (hipStream_t)hip_stream;
    nsg::frac::Args a;
    const int rc = frac_prepare(ctx, B, ld, max_bits, table_limbs, s, a);
    if (rc != NS_OK) return rc;
    a.probs = d_probs;
    a.ids = d_ids;
    a.count = d_count;
    a.bits = d_bits;
    a.bits_stride = bits_stride;
    a.token_out = d_token;
    a.used_out = d_used;
    a.status = d_status;
    hipLaunchKernelGGL(nsg::frac::frac_step_kernel<false>, dim3(B), dim3(64), 0, s, a);
    return hipGetLastError() == hipSuccess ? NS_OK : frac_fail(ctx, "ns_frac_encode_step: launch failed", NS_ERR_HIP);
}

extern "C" int ns_frac_decode_step(ns_frac_ctx* ctx, int B, const double* d_probs, const int32_t* d_ids, int64_t ld,
                                   const int32_t* d_count, const int32_t* d_token, const int32_t* d_used,
                                   int64_t max_used, int64_t table_limbs, uint8_t* d_out_bits, int64_t out_stride,
                                   int64_t* d_out_pos, int32_t* d_status, void* hip_stream) {
    if (!ctx) return frac_fail(ctx, "ns_frac_decode_step: null context", NS_ERR_CONFIG);
    if (!d_probs || !d_ids || !d_count || !d_token || !d_used || !d_out_bits || !d_out_pos || !d_status)
        return frac_fail(ctx, "ns_frac_decode_step: null buffer", NS_ERR_CONFIG);
    if (max_used > (1 << 30)) return frac_fail(ctx, "ns_frac_decode_step: max_used too large", NS_ERR_CONFIG);
    const hipStream_t s = (hipStream_t)hip_stream;
    nsg::frac::Args a;
    const int rc = frac_prepare(ctx, B, ld, max_used, table_limbs, s, a);
    if (rc != NS_OK) return rc;
    a.probs = d_probs;
    a.ids = d_ids;
    a.count = d_count;
    a.token_in = d_token;
    a.used_in = d_used;
    a.out_bits = d_out_bits;
    a.out_stride = out_stride;
    a.out_pos = d_out_pos;
    a.status = d_status;
    hipLaunchKernelGGL(nsg::frac::frac_step_kernel<true>, dim3(B), dim3(64), 0, s, a);
    return hipGetLastError() == hipSuccess ? NS_OK : frac_fail(ctx, "ns_frac_decode_step: launch failed", NS_ERR_HIP);
}

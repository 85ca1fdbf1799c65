// nsg_bigint.h -- unsigned multi-limb integers (base 2^32, little-endian limbs) for the exact-rational
// Fraction coder (nsg_fraction.hip).  Plain fixed-buffer routines: every output buffer is the caller's, every
// length is a limb count, every result length is returned trimmed (no leading zero limb; 0 has length 0).
// The functions are `__host__ __device__` under hipcc so the same text runs in the kernel and in the host unit
// test that checks it against Python integers (tests/native/bigint_check.cpp); nothing here allocates.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define NSG_BI __host__ __device__ inline
#else
#define NSG_BI inline
#endif

namespace nsg {
namespace bi {

typedef uint32_t limb;

NSG_BI int trim(const limb* a, int n) {
    while (n > 0 && a[n - 1] == 0) --n;
    return n;
}

NSG_BI int cmp(const limb* a, int na, const limb* b, int nb) {
    na = trim(a, na);
    nb = trim(b, nb);
    if (na != nb) return na < nb ? -1 : 1;
    for (int i = na - 1; i >= 0; --i)
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    return 0;
}

NSG_BI int copy(limb* o, const limb* a, int na) {
    for (int i = 0; i < na; ++i) o[i] = a[i];
    return trim(o, na);
}

NSG_BI int set_u64(limb* o, uint64_t v) {
    o[0] = (limb)v;
    o[1] = (limb)(v >> 32);
    return v >> 32 ? 2 : v ? 1 : 0;
}

NSG_BI int bit_length(const limb* a, int na) {
    na = trim(a, na);
    return na ? 32 * (na - 1) + (32 - __builtin_clz(a[na - 1])) : 0;
}

// o = a + b; o may alias a or b; room for max(na, nb) + 1 limbs
NSG_BI int add(limb* o, const limb* a, int na, const limb* b, int nb) {
    if (na < nb) {
        const limb* t = a;
        a = b;
        b = t;
        const int tn = na;
        na = nb;
        nb = tn;
    }
    uint64_t c = 0;
    int i = 0;
    for (; i < nb; ++i) {
        c += (uint64_t)a[i] + b[i];
        o[i] = (limb)c;
        c >>= 32;
    }
    for (; i < na; ++i) {
        c += a[i];
        o[i] = (limb)c;
        c >>= 32;
    }
    if (c) o[i++] = (limb)c;
    return trim(o, i);
}

// o = a - b for a >= b; o may alias a or b
NSG_BI int sub(limb* o, const limb* a, int na, const limb* b, int nb) {
    int64_t br = 0;
    int i = 0;
    for (; i < nb; ++i) {
        const int64_t t = (int64_t)a[i] - b[i] - br;
        o[i] = (limb)t;
        br = t < 0;
    }
    for (; i < na; ++i) {
        const int64_t t = (int64_t)a[i] - br;
        o[i] = (limb)t;
        br = t < 0;
    }
    return trim(o, na);
}

// o = a * b (schoolbook); o must not alias a or b; room for na + nb limbs
NSG_BI int mul(limb* o, const limb* a, int na, const limb* b, int nb) {
    na = trim(a, na);
    nb = trim(b, nb);
    if (!na || !nb) return 0;
    for (int i = 0; i < na; ++i) o[i] = 0;
    for (int j = 0; j < nb; ++j) {
        const uint64_t bj = b[j];
        uint64_t c = 0;
        for (int i = 0; i < na; ++i) {
            c += (uint64_t)a[i] * bj + o[i + j];  // <= (2^32-1)^2 + 2 (2^32-1) = 2^64 - 1
            o[i + j] = (limb)c;
            c >>= 32;
        }
        o[j + na] = (limb)c;
    }
    return trim(o, na + nb);
}

// o = a * m; o may alias a; room for na + 2 limbs
NSG_BI int mul_u64(limb* o, const limb* a, int na, uint64_t m) {
    // column i = lo(a[i] m0) + hi(a[i-1] m0) + lo(a[i-1] m1) + hi(a[i-2] m1) + carry: five terms < 2^32 each.
    // The original a[i-1], a[i-2] are kept in registers, so o may overwrite a in place.
    const uint64_t m0 = (uint32_t)m, m1 = m >> 32;
    uint64_t p1 = 0, p2 = 0, c = 0;  // a[i-1], a[i-2]
    for (int i = 0; i < na + 2; ++i) {
        const uint64_t ai = i < na ? a[i] : 0;
        const uint64_t col = (uint32_t)(ai * m0) + ((p1 * m0) >> 32) + (uint32_t)(p1 * m1) + ((p2 * m1) >> 32) + c;
        o[i] = (limb)col;
        c = col >> 32;
        p2 = p1;
        p1 = ai;
    }
    return trim(o, na + 2);
}

// o = a << k; o may alias a; room for na + k/32 + 1 limbs
NSG_BI int shl(limb* o, const limb* a, int na, int k) {
    na = trim(a, na);
    if (!na) return 0;
    const int ws = k >> 5, bs = k & 31;
    if (bs == 0) {
        for (int i = na - 1; i >= 0; --i) o[i + ws] = a[i];
        for (int i = 0; i < ws; ++i) o[i] = 0;
        return na + ws;
    }
    o[na + ws] = a[na - 1] >> (32 - bs);
    for (int i = na - 1; i > 0; --i) o[i + ws] = (a[i] << bs) | (a[i - 1] >> (32 - bs));
    o[ws] = a[0] << bs;
    for (int i = 0; i < ws; ++i) o[i] = 0;
    return trim(o, na + ws + 1);
}

// o = a >> k (floor); o may alias a
NSG_BI int shr(limb* o, const limb* a, int na, int k) {
    na = trim(a, na);
    const int ws = k >> 5, bs = k & 31;
    if (ws >= na) return 0;
    const int n = na - ws;
    for (int i = 0; i < n; ++i) {
        const limb lo = a[i + ws] >> bs;
        const limb hi = (bs && i + ws + 1 < na) ? a[i + ws + 1] << (32 - bs) : 0;
        o[i] = lo | hi;
    }
    return trim(o, n);
}

// remainder of a / d (d > 0)
NSG_BI uint32_t mod_u32(const limb* a, int na, uint32_t d) {
    uint64_t r = 0;
    for (int i = trim(a, na) - 1; i >= 0; --i) r = ((r << 32) | a[i]) % d;
    return (uint32_t)r;
}

// q = a / d, returns the remainder; q may alias a; q gets na limbs
NSG_BI uint32_t divmod_u32(limb* q, const limb* a, int na, uint32_t d) {
    uint64_t r = 0;
    for (int i = na - 1; i >= 0; --i) {
        const uint64_t cur = (r << 32) | a[i];
        q[i] = (limb)(cur / d);
        r = cur - (uint64_t)q[i] * d;
    }
    return (uint32_t)r;
}

// Knuth's algorithm D: q = u / v, r = u % v (r may be null).  v != 0.  Scratch: un (m + 1 limbs), vn (n).
// q gets m - n + 1 limbs, r n limbs.  Returns the trimmed quotient length; *nr the remainder's.
NSG_BI int divmod(limb* q, limb* r, int* nr, const limb* u, int m, const limb* v, int n, limb* un, limb* vn) {
    m = trim(u, m);
    n = trim(v, n);
    if (m < n) {
        if (r) *nr = copy(r, u, m);
        return 0;
    }
    if (n == 1) {
        const uint32_t rem = divmod_u32(q, u, m, v[0]);
        if (r) {
            r[0] = rem;
            *nr = rem ? 1 : 0;
        }
        return trim(q, m);
    }
    const int s = __builtin_clz(v[n - 1]);
    for (int i = n - 1; i > 0; --i) vn[i] = (v[i] << s) | (s ? v[i - 1] >> (32 - s) : 0);
    vn[0] = v[0] << s;
    un[m] = s ? u[m - 1] >> (32 - s) : 0;
    for (int i = m - 1; i > 0; --i) un[i] = (u[i] << s) | (s ? u[i - 1] >> (32 - s) : 0);
    un[0] = u[0] << s;
    const uint64_t B = (uint64_t)1 << 32;
    for (int j = m - n; j >= 0; --j) {
        const uint64_t num = ((uint64_t)un[j + n] << 32) | un[j + n - 1];
        uint64_t qhat = num / vn[n - 1];
        uint64_t rhat = num - qhat * vn[n - 1];
        while (qhat >= B || qhat * vn[n - 2] > ((rhat << 32) | un[j + n - 2])) {
            --qhat;
            rhat += vn[n - 1];
            if (rhat >= B) break;
        }
        int64_t k = 0, t;
        for (int i = 0; i < n; ++i) {
            const uint64_t p = qhat * vn[i];
            t = (int64_t)un[i + j] - k - (int64_t)(p & 0xFFFFFFFFu);
            un[i + j] = (limb)t;
            k = (int64_t)(p >> 32) - (t >> 32);
        }
        t = (int64_t)un[j + n] - k;
        un[j + n] = (limb)t;
        q[j] = (limb)qhat;
        if (t < 0) {  // qhat was one too large (probability ~2/B): add v back
            --q[j];
            uint64_t c = 0;
            for (int i = 0; i < n; ++i) {
                c += (uint64_t)un[i + j] + vn[i];
                un[i + j] = (limb)c;
                c >>= 32;
            }
            un[j + n] += (limb)c;
        }
    }
    if (r) {
        for (int i = 0; i < n; ++i) r[i] = (un[i] >> s) | (s ? un[i + 1] << (32 - s) : 0);
        *nr = trim(r, n);
    }
    return trim(q, m - n + 1);
}

NSG_BI uint64_t gcd_u64(uint64_t a, uint64_t b) {
    while (b) {
        const uint64_t t = a % b;
        a = b;
        b = t;
    }
    return a;
}

// |x| for x = a - b given as two magnitudes: o = |a - b|; o may alias a or b
NSG_BI int absdiff(limb* o, const limb* a, int na, const limb* b, int nb) {
    return cmp(a, na, b, nb) >= 0 ? sub(o, a, na, b, nb) : sub(o, b, nb, a, na);
}

constexpr uint32_t FRACTION_LIMIT = 1u << 30;

// Fraction.from_float(p).limit_denominator(2^30) for a finite p >= 0 (src/neuralstego/codec/arithmetic.py:545-550,
// CPython's Lib/fractions.py limit_denominator): the value num * 2^shift / den, reduced, den <= 2^30.
//   * den(p) <= 2^30: p itself (p >= 1 may be a large integer: num * 2^shift);
//   * else the continued-fraction convergents p1/q1 of p while q <= 2^30, then the nearer of the last convergent
//     and the semiconvergent (p0 + k p1) / (q0 + k q1), k = (2^30 - q0) // q1 -- ties to the convergent;
//   * p < 2^-73 (den > 2^126): the convergent is 0/1 and the semiconvergent 1/2^30, and 0 is the nearer.
// Here den(p) = 2^K with 30 < K <= 126 and num(p) < 2^53, so the expansion runs on <= 4-limb integers.
NSG_BI void to_fraction(double p, uint64_t* num, int* shift, uint32_t* den) {
    const uint64_t bits = __builtin_bit_cast(uint64_t, p);
    *num = 0;
    *shift = 0;
    *den = 1;
    if (p == 0.0) return;
    const int e = (int)((bits >> 52) & 0x7FF);
    uint64_t M = bits & ((1ull << 52) - 1);
    int E;
    if (e) {
        M |= 1ull << 52;
        E = e - 1075;
    } else {
        E = -1074;
    }
    const int tz = __builtin_ctzll(M);
    M >>= tz;
    E += tz;
    if (E >= 0) {
        *num = M;
        *shift = E;
        return;
    }
    if (-E <= 30) {
        *num = M;
        *den = 1u << -E;
        return;
    }
    if (-E > 126) return;  // 0 / 1
    const int K = -E;
    limb n[6] = {0, 0, 0, 0, 0, 0}, d[6] = {0, 0, 0, 0, 0, 0}, q[6], r[6], un[7], vn[6];
    int nn = set_u64(n, M);
    d[K >> 5] = 1u << (K & 31);
    int nd = (K >> 5) + 1;
    uint64_t p0 = 0, q0 = 1, p1 = 1, q1 = 0;
    const uint64_t MAXD = FRACTION_LIMIT;
    for (;;) {
        int nr = 0;
        const int nq = divmod(q, r, &nr, n, nn, d, nd, un, vn);
        const bool huge = nq > 2;
        const uint64_t a = huge ? 0 : nq == 0 ? 0 : nq == 1 ? q[0] : (q[0] | ((uint64_t)q[1] << 32));
        uint64_t q2, p2;
        if (q1 == 0) {
            q2 = q0;
            p2 = p0 + a * p1;  // first step: a = floor(p) < 2^23
        } else {
            if (huge || a > (MAXD - q0) / q1) break;
            q2 = q0 + a * q1;
            p2 = p0 + a * p1;
        }
        if (q2 > MAXD) break;
        p0 = p1;
        q0 = q1;
        p1 = p2;
        q1 = q2;
        nn = copy(n, d, nd);  // n, d = d, n - a d
        nd = copy(d, r, nr);
        if (nd == 0) break;   // exact expansion ended (unreachable: den(p) > 2^30)
    }
    const uint64_t k = (MAXD - q0) / q1;
    const uint64_t b1n = p0 + k * p1, b1d = q0 + k * q1;
    // |p1/q1 - M/2^K| <= |b1n/b1d - M/2^K|  <=>  |p1 2^K - M q1| b1d <= |b1n 2^K - M b1d| q1
    limb x[9], y[9], lhs[11], rhs[11];
    int nx = set_u64(x, p1);
    nx = shl(x, x, nx, K);
    int ny = set_u64(y, M);
    ny = mul_u64(y, y, ny, q1);
    nx = absdiff(x, x, nx, y, ny);
    const int nl = mul_u64(lhs, x, nx, b1d);
    nx = set_u64(x, b1n);
    nx = shl(x, x, nx, K);
    ny = set_u64(y, M);
    ny = mul_u64(y, y, ny, b1d);
    nx = absdiff(x, x, nx, y, ny);
    const int nrh = mul_u64(rhs, x, nx, q1);
    if (cmp(lhs, nl, rhs, nrh) <= 0) {
        *num = p1;
        *den = (uint32_t)q1;
    } else {
        const uint64_t g = gcd_u64(b1n, b1d);
        *num = b1n / g;
        *den = (uint32_t)(b1d / g);
    }
}

}  // namespace bi
}  // namespace nsg
